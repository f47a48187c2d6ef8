#!/bin/bash
# Interleaved A/B of native builds (variants/<name>.so) on tools/nt_shapes.py.  Usage: tools/nt_variant_shapes_ab.sh <reps> <name>...
export FEDMI_NO_BUILD=1
reps=$1; shift
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    echo "== $v $rep"
    FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 300 python -u tools/nt_shapes.py 2>/dev/null || exit 1
  done
done
