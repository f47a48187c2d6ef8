#!/bin/bash
# round-2 GPU pass s: A/B of the plain-bf16 multi-client training forward (variants/plainfwd.so)
# against the previous build (variants/base.so) on one box: 1-GPU bench, emulated multi-client round
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2s
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
bash tools/ab_bench.sh $out/ab 3 base plainfwd || exit 1
for v in base plainfwd; do
  FEDMI_NATIVE_SO=$R/variants/$v.so timeout -k 10 200 python -u tools/round_emulate.py > $out/emulate_$v.log 2>&1 || { tail -20 $out/emulate_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $out/emulate_$v.log
done
