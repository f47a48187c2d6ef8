#!/bin/bash
# round-2 GPU pass y: row stride of the wide client's transposed operands (FEDMI_WIDE_TPAD extra
# elements) -- kernel breakdown of the 131072-row round per padding
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2y
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
for p in 0 256 64; do
  cd /tmp && FEDMI_WIDE_TPAD=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof$p -o run --output-format csv \
      -- python $R/tools/wide_prof.py > $out/prof$p.log 2>&1 || { tail -20 $out/prof$p.log; exit 1; }
  python $R/tools/rocprof_summary.py stats $out/prof$p > $out/kernel_summary_$p.txt 2>&1
  echo "== TPAD $p"; head -8 $out/kernel_summary_$p.txt; tail -1 $out/kernel_summary_$p.txt
done
