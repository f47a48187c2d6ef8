#!/bin/bash
# round-2 GPU pass b: split-bf16 forward -- full GPU suite, benches, emulated N>1 round, HIP rounds-to-target
set -o pipefail
mkdir -p gpurun_out/r2b
export FEDMI_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > gpurun_out/r2b/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r2b/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2b/bench_s20.json 2> gpurun_out/r2b/bench_s20.err || exit $?
cat gpurun_out/r2b/bench_s20.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 100 --no-convergence --no-anchor > gpurun_out/r2b/bench_s2000.json 2> gpurun_out/r2b/bench_s2000.err || exit $?
timeout -k 10 200 python tools/round_emulate.py --rounds 2000 > gpurun_out/r2b/round_emulate.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/rounds_to_target.py --backend hip --dtype fp32 bf16 --seeds 10 --out gpurun_out/r2b/rtt_hip.json > gpurun_out/r2b/rtt_hip.log 2>&1
