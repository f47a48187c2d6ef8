#!/bin/bash
# round-2 first GPU pass: new RCCL tests, bench contract (incl. self-launched shared-GPU N=2), driver-shaped bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl.py tests/test_bench_contract.py > gpurun_out/r2a_pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a_bench_s20.json 2> gpurun_out/r2a_bench_s20.err || exit $?
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 100 --no-convergence > gpurun_out/r2a_bench_s2000.json 2> gpurun_out/r2a_bench_s2000.err || exit $?
timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 200 --warmup 50 --no-convergence --no-anchor > gpurun_out/r2a_bench_n2share.json 2> gpurun_out/r2a_bench_n2share.err || exit $?
timeout -k 10 200 python bench.py --gpus 4 --share-gpu --steps 200 --warmup 50 --no-convergence --no-anchor > gpurun_out/r2a_bench_n4share.json 2> gpurun_out/r2a_bench_n4share.err
