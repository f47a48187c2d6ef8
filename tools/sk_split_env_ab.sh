#!/bin/bash
# Interleaved A/B of the tile-split row pass (FEDMI_SK_SPLIT=1: off, "": default heuristic, or a slice count)
# on the sklearn minibatch step.  Usage (GPU box): tools/sk_split_env_ab.sh <reps> <case> <split>...
export FEDMI_NO_BUILD=1
reps=$1; case=$2; shift 2
for rep in $(seq 1 $reps); do
  for sp in "$@"; do
    FEDMI_SK_SPLIT=$sp timeout -k 10 300 python -u tools/sk_step_bench.py --fused-only --case $case 2>/dev/null | python -c "
import json,sys
print('split=$sp', $rep, ' | '.join(f\"{'x'.join(map(str, d['hidden']))}x{d['trials']} s{d['split']} {d['us_per_step']:.1f} us\" for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
