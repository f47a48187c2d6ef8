#!/bin/bash
# sklearn float64 estimator on the GPU: parity tests, then the minibatch step with the tile-split row pass off
# (FEDMI_SK_SPLIT=1) and at its default, then the kernel split of the [S] step under rocprofv3.
export FEDMI_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sklearn_estimator.py -m gpu 2>&1 | tail -3 || exit 1
for sp in 1 ""; do
  echo "== FEDMI_SK_SPLIT=$sp"
  FEDMI_SK_SPLIT=$sp timeout -k 10 300 python -u tools/sk_step_bench.py --fused-only 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['hidden'], d['trials'], 'split', d['split'], round(d['us_per_step'],1), 'us/step', 'loss', d['final_loss'])" || exit 1
done
tools/sk_split_prof.sh ${1:-skprof2} 2>&1 | grep -v amdgpu
