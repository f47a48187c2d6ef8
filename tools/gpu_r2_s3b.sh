#!/bin/bash
# full GPU suite after the kernel-body refactor + config-5 bench mode + headline regression check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3b_pytest.log 2>&1 || { tail -40 gpurun_out/s3b_pytest.log; exit 1; }
tail -3 gpurun_out/s3b_pytest.log
timeout -k 10 120 python bench.py --config sweep --steps 400 --warmup 32 > gpurun_out/s3b_sweep.json 2> gpurun_out/s3b_sweep.err || { tail -20 gpurun_out/s3b_sweep.err; exit 1; }
cat gpurun_out/s3b_sweep.json
timeout -k 10 180 python bench.py --steps 2000 --warmup 200 --no-convergence > gpurun_out/s3b_bench.json 2> gpurun_out/s3b_bench.err || { tail -20 gpurun_out/s3b_bench.err; exit 1; }
cat gpurun_out/s3b_bench.json
