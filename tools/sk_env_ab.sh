#!/bin/bash
# Interleaved A/B of one environment knob on the sklearn minibatch step (tools/sk_step_bench.py --fused-only).
# Usage (GPU box): tools/sk_env_ab.sh <reps> <VAR> <case|all> <value>...   ("" = unset; case: sk_step_bench's index)
export FEDMI_NO_BUILD=1
reps=$1; var=$2; case=$3; shift 3
sel=""; [ "$case" != "all" ] && sel="--case $case"
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    env $var="$v" timeout -k 10 300 python -u tools/sk_step_bench.py --fused-only $sel 2>/dev/null | python -c "
import json,sys
print('$var=$v', $rep, ' | '.join(f\"{'x'.join(map(str, d['hidden']))}x{d['trials']} s{d['split']} {d['us_per_step']:.1f}\" for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
