#!/bin/bash
# round-2 GPU pass d: A/B of the peer-protocol fences (variants/fences{0,1,2}.so) on the emulated N>1 round
set -o pipefail
mkdir -p gpurun_out/r2d
export FEDMI_NO_BUILD=1
for rep in 1 2; do
  for v in fences0 fences1 fences2; do
    echo "== $v rep $rep"
    FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 150 python tools/round_emulate.py --rounds 3000 2>/dev/null || exit $?
  done
done > gpurun_out/r2d/peer_fences.log
cat gpurun_out/r2d/peer_fences.log
timeout -k 10 300 python -u -m pytest tests/test_participation.py tests/test_peer_allreduce.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1
tail -3 gpurun_out/r2d/pytest.log
