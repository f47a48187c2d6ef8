set -o pipefail
mkdir -p gpurun_out
export FEDMI_NO_BUILD=1
FEDMI_NATIVE_SO=$PWD/variants/skxcd.so timeout -k 10 300 python -u -m pytest tests/test_sklearn_estimator.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/skxcd_tests.log 2>&1 || { tail -20 gpurun_out/skxcd_tests.log; exit 1; }
tail -1 gpurun_out/skxcd_tests.log
timeout -k 10 400 tools/sk_variant_ab.sh 3 skbase skxcd > gpurun_out/skxcd_ab.log 2>&1 || exit 1
for rep in 1 2; do for v in skbase skxcd; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 120 python -u hyperparameters_tuning.py --quiet 2>/dev/null | grep -E "wall|Best Global Hyper" | sed "s/^/$v $rep /" >> gpurun_out/skxcd_ab.log || exit 1
done; done
cat gpurun_out/skxcd_ab.log
