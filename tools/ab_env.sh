#!/bin/bash
# A/B of runtime environment settings on the 1-GPU bench, interleaved repetitions.
# Usage (GPU box): tools/ab_env.sh <out_dir> <reps> "NAME=VALUE ..." "NAME=VALUE ..." ...
# ("-" = the unchanged environment); $AB_ARGS are extra bench.py arguments.
set -o pipefail
out=$1; reps=$2; shift 2
mkdir -p $out
for rep in $(seq 1 $reps); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=(); [ "$v" != "-" ] && read -r -a envs <<< "$v"
    env "${envs[@]}" timeout -k 10 120 python -u bench.py --no-convergence --no-anchor --no-fp32 --steps 3000 --warmup 300 $AB_ARGS \
      > $out/v$i.$rep.json 2>$out/v$i.$rep.err || exit 1
    python -c "import json;d=json.load(open('$out/v$i.$rep.json'));print('$v', $rep, round(d['ms_per_step']*1e3,2), 'us/round')"
  done
done
