#!/bin/bash
# round-2 GPU pass g: head split-K -- correctness tests, stamps, bench
set -o pipefail
mkdir -p gpurun_out/r2g
export FEDMI_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_hip_engine.py tests/test_peer_allreduce.py tests/test_simulate.py -m gpu > gpurun_out/r2g/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2g/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/stamps.py 8000 32 50,200 bf16 > gpurun_out/r2g/stamps.log 2>&1 || exit $?
cat gpurun_out/r2g/stamps.log
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 100 --no-convergence --no-anchor > gpurun_out/r2g/bench_s2000.json 2>/dev/null || exit $?
cat gpurun_out/r2g/bench_s2000.json
timeout -k 10 200 python tools/round_emulate.py --rounds 2000 > gpurun_out/r2g/round_emulate.log 2>&1
cat gpurun_out/r2g/round_emulate.log
