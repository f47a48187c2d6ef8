#!/bin/bash
# round-2 GPU pass u: GPU suite + 1-GPU bench (noisy synthetic labels), 2 clients sharing the GPU
# through the xGMI peer protocol (LL chunks), wide-round kernel breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2u
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
bash tools/gpu_session.sh r2u/session tests bench || exit $?
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 2000 --warmup 200 > $out/bench_n2_share.json 2> $out/bench_n2_share.err || { tail -20 $out/bench_n2_share.err; exit 1; }
cat $out/bench_n2_share.json
bash tools/gpu_r2_t.sh
