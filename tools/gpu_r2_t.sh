#!/bin/bash
# round-2 GPU pass t: kernel breakdown of the wide (config 3) round at 131072 rows, current build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=${OUT_T:-$R/gpurun_out/r2t}
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
    -- python $R/tools/wide_prof.py > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
python $R/tools/rocprof_summary.py stats $out/prof > $out/kernel_summary.txt 2>&1
cat $out/kernel_summary.txt
