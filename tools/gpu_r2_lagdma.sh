#!/bin/bash
# lagged rounds: per-layer DMA restage (lagdma, default) vs register prefetch (lagregs)
set -o pipefail
mkdir -p gpurun_out/ab_lagdma
timeout -k 10 500 python -u -m pytest tests/test_peer_allreduce.py tests/test_hip_engine.py tests/test_simulate.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/lagdma_pytest.log 2>&1 || { tail -30 gpurun_out/lagdma_pytest.log; exit 1; }
tail -2 gpurun_out/lagdma_pytest.log
for rep in 1 2; do for v in lagregs lagdma; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python tools/round_emulate.py > gpurun_out/ab_lagdma/emu_$v.$rep.log 2>&1 || { tail gpurun_out/ab_lagdma/emu_$v.$rep.log; exit 1; }
  echo "== $v $rep"; grep -i "lagged eval\|early stopping" gpurun_out/ab_lagdma/emu_$v.$rep.log
done; done
for rep in 1 2; do for v in lagregs lagdma; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 1000 --warmup 100 --no-anchor --no-convergence > gpurun_out/ab_lagdma/n2_$v.$rep.json 2> gpurun_out/ab_lagdma/n2_$v.$rep.err || { tail gpurun_out/ab_lagdma/n2_$v.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_lagdma/n2_$v.$rep.json'));print('n2 $v $rep', round(d['ms_per_step']*1e3,2), 'us/round')"
done; done
