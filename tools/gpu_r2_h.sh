#!/bin/bash
# round-2 GPU pass h: wide client with whole-shard local evaluation; BASELINE config 3 at its stated size
set -o pipefail
mkdir -p gpurun_out/r2h
export FEDMI_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_wide_fedavg.py tests/test_checkpoint.py tests/test_bench_contract.py -m gpu -k "wide" > gpurun_out/r2h/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2h/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --config wide --steps 5 --warmup 2 > gpurun_out/r2h/bench_wide_131k.json 2> gpurun_out/r2h/bench_wide_131k.err || exit $?
cat gpurun_out/r2h/bench_wide_131k.json
timeout -k 10 400 python bench.py --config wide --wide-rows 12500000 --steps 2 --warmup 1 > gpurun_out/r2h/bench_wide_12p5M.json 2> gpurun_out/r2h/bench_wide_12p5M.err || exit $?
cat gpurun_out/r2h/bench_wide_12p5M.json
