#!/bin/bash
# round-2 GPU pass w: NT epilogue configurations without transposed copies (wide eval forward,
# last hidden layer, dgrad into layer 0) -- GPU tests of the NT GEMM / wide client, the LL peer
# tests, wide-round kernel breakdown, config 3 at size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2w2
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hip_engine.py tests/test_wide_fedavg.py tests/test_peer_allreduce.py -m gpu -x -v \
    --timeout 120 --timeout-method thread -k "nt or wide or peer or colsum" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
OUT_T=$out/t bash tools/gpu_r2_t.sh || exit 1
timeout -k 10 600 python -u bench.py --config wide --wide-rows 12500000 --steps 2 --warmup 1 > $out/bench_wide_12p5M.json 2> $out/bench_wide.err || { tail -20 $out/bench_wide.err; exit 1; }
cat $out/bench_wide_12p5M.json
