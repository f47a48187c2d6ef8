#!/bin/bash
# A/B of native builds (variants/<name>.so) on the sklearn minibatch step (tools/sk_step_bench.py --fused-only),
# interleaved.  Usage (GPU box): tools/sk_variant_ab.sh <reps> <name>...
export FEDMI_NO_BUILD=1
reps=$1; shift
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 300 python -u tools/sk_step_bench.py --fused-only 2>/dev/null | python -c "
import json,sys
print('$v', $rep, ' | '.join(f\"{'x'.join(map(str, d['hidden']))}x{d['trials']} s{d['split']} {d['us_per_step']:.1f}\" for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
