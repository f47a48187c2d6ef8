#!/bin/bash
# include-based kernel bodies: sweep/group GPU tests, A/B vs the pre-batch library, config-5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fed_sweep.py tests/test_bench_contract.py tests/test_hip_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3c_pytest.log 2>&1 || { tail -40 gpurun_out/s3c_pytest.log; exit 1; }
tail -2 gpurun_out/s3c_pytest.log
bash tools/ab_bench.sh gpurun_out/ab_inc 3 old new || exit 1
timeout -k 10 120 python bench.py --config sweep --steps 400 --warmup 32 > gpurun_out/s3c_sweep.json 2> gpurun_out/s3c_sweep.err || { tail -20 gpurun_out/s3c_sweep.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s3c_sweep.json'));print('sweep', round(d['value']), d['us_per_trial_round'], d['best_trial'])"
