#!/bin/bash
# Interleaved A/B of native builds (variants/<name>.so) on the NT GEMM K sweep (tools/nt_ksweep.py, default variant 3).
# Usage (GPU box): tools/nt_variant_ab.sh <reps> <name>...
export FEDMI_NO_BUILD=1
reps=$1; shift
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    echo "== $v $rep"
    FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 300 python -u tools/nt_ksweep.py 3 2>/dev/null | grep -E "x4096x4096|x4096x8192|8192x8192x8192|fit" || exit 1
  done
done
