#!/bin/bash
# dgrad-first backward phases with arrival counts (dgf) vs previous commit (head)
set -o pipefail
mkdir -p gpurun_out/ab_dgf
timeout -k 10 500 python -u -m pytest tests/test_hip_engine.py tests/test_peer_allreduce.py tests/test_fed_sweep.py tests/test_simulate.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/dgf_pytest.log 2>&1 || { tail -30 gpurun_out/dgf_pytest.log; exit 1; }
tail -2 gpurun_out/dgf_pytest.log
bash tools/ab_bench.sh gpurun_out/ab_dgf 3 head dgf || exit 1
for rep in 1 2; do for v in head dgf; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 1000 --warmup 100 --no-anchor --no-convergence > gpurun_out/ab_dgf/n2_$v.$rep.json 2> gpurun_out/ab_dgf/n2_$v.$rep.err || { tail gpurun_out/ab_dgf/n2_$v.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_dgf/n2_$v.$rep.json'));print('n2 $v $rep', round(d['ms_per_step']*1e3,2), 'us/round')"
done; done
