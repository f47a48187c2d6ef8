export FEDMI_NO_BUILD=1
mkdir -p gpurun_out/skcs
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sklearn_estimator.py -m gpu > gpurun_out/skcs/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/skcs/pytest.log; [ $rc = 0 ] || exit $rc
for sp in 1 "" 4 8 2; do
  echo "== FEDMI_SK_SPLIT=$sp"
  FEDMI_SK_SPLIT=$sp timeout -k 10 300 python -u tools/sk_step_bench.py --fused-only 2>/dev/null | tee -a gpurun_out/skcs/bench.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['hidden'], d['trials'], 'split', d['split'], round(d['us_per_step'],1), 'us/step', 'loss', d['final_loss'])" || exit 1
done
