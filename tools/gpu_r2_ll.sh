#!/bin/bash
# LL-specialised Adam kernel: peer tests, then 2 ranks sharing the GPU (interleaved reps) + emulated N>1 round
set -o pipefail
mkdir -p gpurun_out/ab_ll
timeout -k 10 400 python -u -m pytest tests/test_peer_allreduce.py tests/test_bench_contract.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/ll_pytest.log 2>&1 || { tail -30 gpurun_out/ll_pytest.log; exit 1; }
tail -2 gpurun_out/ll_pytest.log
for rep in 1 2 3; do for v in head ll; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 1000 --warmup 100 --no-anchor --no-convergence > gpurun_out/ab_ll/n2_$v.$rep.json 2> gpurun_out/ab_ll/n2_$v.$rep.err || { tail gpurun_out/ab_ll/n2_$v.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_ll/n2_$v.$rep.json'));print('n2 $v $rep', round(d['ms_per_step']*1e3,2), 'us/round')"
done; done
for v in head ll; do FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python tools/round_emulate.py > gpurun_out/ab_ll/emu_$v.log 2>&1 || { tail gpurun_out/ab_ll/emu_$v.log; exit 1; }; echo "== emu $v"; grep -i "FedAvg in Adam\|early stopping" gpurun_out/ab_ll/emu_$v.log; done
