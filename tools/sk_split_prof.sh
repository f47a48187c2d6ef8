#!/bin/bash
# Kernel split of the sklearn float64 minibatch step under rocprofv3 (case 0 = (50, 400) x 1 trial, [S];
# tools/sk_step_bench.py lists the cases).  Usage (GPU box): tools/sk_split_prof.sh <out> [case]
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-skprof}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp FEDMI_NO_BUILD=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- \
    python $R/tools/sk_step_bench.py --fused-only --case ${2:-0} > $out/bench.jsonl 2> $out/bench.err || exit 1
python - "$out/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    print(f"{x['Name'][:50]:50s} calls={x['Calls']:>7s} avg_us={float(x['AverageNs'])/1e3:8.2f} pct={float(x['Percentage']):6.2f}")
PY
cat $out/bench.jsonl
