#!/bin/bash
# wgrad tiles off the long-dgrad waves: fine stamps, A/B vs base, bf16 kernel tests
set -o pipefail
mkdir -p gpurun_out
FEDMI_NATIVE_SO=$PWD/variants/fine.so timeout -k 10 120 python tools/probes/stamps_fine.py > gpurun_out/s3e_stamps.log 2>&1 || { tail gpurun_out/s3e_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s3e_stamps.log
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py tests/test_fed_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3e_pytest.log 2>&1 || { tail -30 gpurun_out/s3e_pytest.log; exit 1; }
tail -2 gpurun_out/s3e_pytest.log
bash tools/ab_bench.sh gpurun_out/ab_pair 3 base cnt pair
