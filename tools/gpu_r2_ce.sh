#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_bench.sh gpurun_out/ab_ce2 3 head ce2 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_hip_engine.py tests/test_peer_allreduce.py tests/test_simulate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ce2_pytest.log 2>&1 || { tail -30 gpurun_out/ce2_pytest.log; exit 1; }
tail -2 gpurun_out/ce2_pytest.log
