#!/bin/bash
# rocprofv3 kernel stats of the config-5 bench (packed trials, trial batches); run on the GPU box
R=$GRAFT_REPO_ROOT; name=${1:-prof_sweep}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$name -o run --output-format csv -- python $R/bench.py --config sweep --steps 400 --warmup 32 > $R/gpurun_out/$name.log 2>&1
rc=$?
python - "$R/gpurun_out/$name/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} calls={x['Calls']:>6s} avg_us={float(x['AverageNs'])/1e3:8.2f} pct={float(x['Percentage']):6.2f}")
PY
exit $rc
