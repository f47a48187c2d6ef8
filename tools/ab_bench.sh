#!/bin/bash
# A/B of alternative native builds (variants/<name>.so) on the 1-GPU bench, interleaved
# repetitions.  Usage (GPU box): tools/ab_bench.sh <out_dir> <reps> <name>...
set -o pipefail
out=$1; reps=$2; shift 2
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 120 python -u bench.py --no-convergence --no-anchor --no-fp32 --steps 3000 --warmup 300 $AB_ARGS \
      > $out/$v.$rep.json 2>$out/$v.$rep.err || exit 1
    python -c "import json,sys;d=json.load(open('$out/$v.$rep.json'));print('$v', $rep, round(d['ms_per_step']*1e3,2), 'us/round')"
  done
done
