#!/bin/bash
# usage: tools/prof_round.sh <outdir-name> [bench args...]  (run on the GPU box)
R=$GRAFT_REPO_ROOT; name=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$name -o run --output-format csv -- python $R/bench.py --no-convergence "$@" > $R/gpurun_out/$name.log 2>&1
rc=$?
python - "$R/gpurun_out/$name/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:60]:60s} calls={x['Calls']:>6s} avg_us={float(x['AverageNs'])/1e3:8.2f} pct={float(x['Percentage']):6.2f}")
PY
exit $rc
