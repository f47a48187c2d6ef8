#!/bin/bash
# round-2 GPU pass e: group-graph trial packing, participation, checkpoints; config-5 and config-4 measurements
set -o pipefail
mkdir -p gpurun_out/r2e
export FEDMI_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fed_sweep.py tests/test_participation.py tests/test_checkpoint.py tests/test_engine_cpu.py -m gpu > gpurun_out/r2e/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2e/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/fed_sweep_bench.py --rounds 100 > gpurun_out/r2e/fed_sweep_packing.log 2>&1 || exit $?
cat gpurun_out/r2e/fed_sweep_packing.log
timeout -k 10 300 python tools/fedprox_config4.py --backend hip --out gpurun_out/r2e/fedprox_config4_hip.json > gpurun_out/r2e/fedprox_config4_hip.log 2>&1 || exit $?
cat gpurun_out/r2e/fedprox_config4_hip.log
