#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_bench.sh gpurun_out/ab_dma 3 head dma || exit 1
timeout -k 10 600 python -u -m pytest tests/test_hip_engine.py tests/test_peer_allreduce.py tests/test_simulate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dma_pytest.log 2>&1 || { tail -30 gpurun_out/dma_pytest.log; exit 1; }
tail -2 gpurun_out/dma_pytest.log
for v in head dma; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 400 --warmup 50 --no-anchor --no-convergence > gpurun_out/ab_dma/n2_$v.json 2> gpurun_out/ab_dma/n2_$v.err || { tail gpurun_out/ab_dma/n2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_dma/n2_$v.json'));print('n2 $v', round(d['ms_per_step']*1e3,2), 'us/round')"
done
