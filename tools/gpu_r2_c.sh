#!/bin/bash
# round-2 GPU pass c: full GPU suite (peer protocol release/acquire, participation table, early-stop args), measurements
set -o pipefail
mkdir -p gpurun_out/r2c
export FEDMI_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > gpurun_out/r2c/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r2c/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/round_emulate.py --rounds 2000 > gpurun_out/r2c/round_emulate.log 2>&1 || exit $?
cat gpurun_out/r2c/round_emulate.log
timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 400 --warmup 50 --no-anchor > gpurun_out/r2c/bench_n2share.json 2> gpurun_out/r2c/bench_n2share.err || exit $?
cat gpurun_out/r2c/bench_n2share.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 100 --no-convergence --no-anchor > gpurun_out/r2c/bench_s2000.json 2> gpurun_out/r2c/bench_s2000.err || exit $?
cat gpurun_out/r2c/bench_s2000.json
