#!/bin/bash
# Round-6 refresh of the convergence evidence on the current kernels.
# Usage (repo root, GPU box): tools/r6_convergence.sh <out_dir> [steps...]
#   steps: rtt config4 skparity h8 ctiming (default: all, in that order)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$1; shift
steps=${*:-rtt config4 skparity h8 ctiming}
mkdir -p $out
export FEDMI_NO_BUILD=1 TMPDIR=/tmp OMP_NUM_THREADS=1
port=29731

run_rtt() {   # [C] 10-seed rounds-to-target, k = 1/2/4/8, fp32 and bf16 HIP kernels (one process per run)
    timeout -k 10 900 python -u tools/rounds_to_target.py --backend hip --dtype fp32 bf16 --seeds 10 \
        --out $out/rounds_to_target_r6.json > $out/rounds_to_target_r6.log 2>&1
}
run_config4() {   # BASELINE config 4 on the HIP engine: 8 clients, alpha 0.3, 5 local steps, 50 rounds, mu 0/0.01/0.1
    timeout -k 10 600 python -u tools/fedprox_config4.py --backend hip --out $out/fedprox_config4_hip_r6.json \
        > $out/fedprox_config4_hip_r6.log 2>&1
}
run_skparity() {   # [S] pooled accuracy vs scikit-learn at k = 1/2/4/8 (float64 HIP estimator)
    timeout -k 10 900 python -u tools/sklearn_parity.py --backends hip:float64 \
        --out $out/sklearn_parity_r6.json > $out/sklearn_parity_r6.log 2>&1
}
run_h8() {   # [H] 90-trial sweep with 8 ranks sharing the GPU (whole-script wall)
    local t0=$(date +%s%N)
    timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port $port hyperparameters_tuning.py --device cuda:0 > $out/h_sweep_k8_shared_r6.log 2>&1
    local rc=$?
    echo "[H] k=8 (8 ranks sharing cuda:0) whole-script wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/h_sweep_k8_shared_r6.log
    return $rc
}
run_ctiming() {   # [C] end to end, one client, bf16 and fp32, --timing
    for dt in bf16 fp32; do
        timeout -k 10 300 python -u FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py --timing --dtype $dt \
            > $out/c_entrypoint_e2e_${dt}_r6.log 2>&1 || return 1
    done
}

for s in $steps; do
    echo "== $s $(date +%T)"
    run_$s || { echo "step $s FAILED"; exit 1; }
done
echo "== done $(date +%T)"
