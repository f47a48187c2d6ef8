#!/bin/bash
# Round-6 evidence session on one MI355X box.  Usage (repo root, GPU box): tools/r6_final.sh <out_dir> [steps...]
#   steps: failfast tests bench prof share sk (default: all, in that order)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/$1; shift
steps=${*:-failfast tests bench prof share sk}
mkdir -p $out
export FEDMI_NO_BUILD=1 TMPDIR=/tmp FEDMI_BENCH_PROGRESS=1
(timeout 1180 bash -c "while sleep 30; do date; done" > $out/heartbeat.txt 2>&1 &)
cd $R

run_failfast() {   # fail-fast GPU tests with their timing lines
    timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_fail_fast.py -m gpu \
        > $out/fail_fast.log 2>&1
}
run_tests() {      # the whole GPU suite
    timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1
    local rc=$?; tail -3 $out/pytest_gpu.log; return $rc
}
run_bench() {      # the driver's shape x 3, the steady state x 1
    for i in 1 2 3; do
        timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_driver_shape_$i.json 2> $out/bench_driver_shape_$i.err || return 1
    done
    timeout -k 10 400 python -u bench.py --steps 2000 --warmup 200 --no-convergence > $out/bench_steady_2000.json 2> $out/bench_steady_2000.err
}
run_prof() {       # kernel summary of the bench
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
        -- python $R/bench.py --no-convergence --no-anchor --steps 2000 --warmup 200 > $out/prof.log 2>&1
    local rc=$?; cd $R; python tools/rocprof_summary.py stats $out/prof > $out/kernel_summary.txt 2>&1; return $rc
}
run_share() {      # N = 2 / 4 / 8 ranks sharing the GPU: the N > 1 round designs incl. the plane companions
    for n in 2 4; do
        timeout -k 10 600 python -u bench.py --gpus $n --share-gpu --steps 400 --warmup 50 --no-anchor --no-convergence \
            > $out/bench_n${n}_share.json 2> $out/bench_n${n}_share.err || return 1
    done
    timeout -k 10 700 python -u bench.py --gpus 8 --share-gpu --steps 400 --warmup 50 --no-anchor --no-convergence \
        --companion-timeout 400 > $out/bench_n8_share.json 2> $out/bench_n8_share.err
}
run_sk() {         # [S] 5 rounds and [H] 90 trials, k = 1, whole script; [H] k = 8 sharing the GPU
    local t0=$(date +%s%N)
    timeout -k 10 300 python -u FL_SkLearn_MLPClassifier_Limitation.py > $out/s_rounds_k1.log 2>&1 || return 1
    echo "[S] k=1 whole-script wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/s_rounds_k1.log
    t0=$(date +%s%N)
    timeout -k 10 300 python -u hyperparameters_tuning.py --quiet > $out/h_sweep_k1.log 2>&1 || return 1
    echo "[H] k=1 whole-script wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/h_sweep_k1.log
    t0=$(date +%s%N)
    timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29741 hyperparameters_tuning.py --device cuda:0 --quiet > $out/h_sweep_k8_shared.log 2>&1 || return 1
    echo "[H] k=8 (8 ranks sharing cuda:0) whole-script wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/h_sweep_k8_shared.log
}

for s in $steps; do
    echo "== $s $(date +%T)"
    run_$s || { echo "step $s FAILED"; exit 1; }
done
echo "== done $(date +%T)"
