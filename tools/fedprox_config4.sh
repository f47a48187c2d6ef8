#!/bin/bash
# BASELINE config 4: 8 clients, Dirichlet label-skew shards (alpha 0.3), 5 local Adam steps per
# round, 50 rounds, FedProx mu in {0, 0.01, 0.1}; one process per client.  Usage:
#   tools/fedprox_config4.sh <out_dir> [extra [C] flags, e.g. --device cpu --backend gloo --engine torch]
set -e -o pipefail
out=$1; shift
mkdir -p $out
for mu in 0 0.01 0.1; do
  OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29611 FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py \
    --partition label_skew --alpha 0.3 --local-steps 5 --rounds 50 --no-early-stop --fedprox-mu $mu \
    --mode correct --jsonl $out/mu_$mu.jsonl "$@" > $out/mu_$mu.log 2>&1
  echo "mu=$mu: $(tail -n 3 $out/mu_$mu.log | tr '\n' ' ')"
done
