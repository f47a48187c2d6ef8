#!/bin/bash
# round-2 GPU pass r: plain-bf16 training forward of multi-client rounds -- full GPU suite,
# 1-GPU bench, emulated multi-client round
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2r
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
bash tools/gpu_session.sh r2r/session tests bench || exit $?
timeout -k 10 200 python -u tools/round_emulate.py > $out/emulate.log 2>&1 || { tail -20 $out/emulate.log; exit 1; }
cat $out/emulate.log
