#!/bin/bash
# round-2 GPU pass aa: the driver's launch shape (torch.distributed.run, one process per rank)
# with two ranks sharing the box's one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2aa
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --share-gpu --steps 500 --warmup 50 > $out/torchrun_n2.out 2> $out/torchrun_n2.err || { tail -30 $out/torchrun_n2.err; exit 1; }
cat $out/torchrun_n2.out
