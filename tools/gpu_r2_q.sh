#!/bin/bash
# round-2 GPU pass q: LL (value + call index in one 8-byte push) weight chunks of the Adam-fused
# exchange: peer / engine GPU tests, then the emulated multi-client round with LL and without
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2q
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_peer_allreduce.py tests/test_rccl.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 200 python -u tools/round_emulate.py > $out/emulate_ll.log 2>&1 || { tail -20 $out/emulate_ll.log; exit 1; }
cat $out/emulate_ll.log
FEDMI_PEER_LL=0 timeout -k 10 200 python -u tools/round_emulate.py > $out/emulate_pull.log 2>&1 || { tail -20 $out/emulate_pull.log; exit 1; }
cat $out/emulate_pull.log
