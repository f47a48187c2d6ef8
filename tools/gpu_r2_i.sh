#!/bin/bash
# round-2 GPU pass i: float64 sklearn estimator on the device (f64 MFMA trainer) -- parity tests
# against the float64 host implementation, [S] k=1 five rounds, [H] 90-trial sweep in fp64
set -o pipefail
mkdir -p gpurun_out/r2i
export FEDMI_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_sklearn_estimator.py -m gpu > gpurun_out/r2i/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r2i/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
( time timeout -k 10 400 python -u FL_SkLearn_MLPClassifier_Limitation.py --backend hip --dtype float64 ) > gpurun_out/r2i/s_rounds_fp64.log 2>&1 || exit $?
grep -E "Accuracy|real" gpurun_out/r2i/s_rounds_fp64.log
( time timeout -k 10 400 python -u hyperparameters_tuning.py --backend hip --dtype fp64 --quiet ) > gpurun_out/r2i/h_sweep_fp64.log 2>&1 || exit $?
tail -5 gpurun_out/r2i/h_sweep_fp64.log
