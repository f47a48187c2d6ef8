#!/bin/bash
# One GPU-box session: GPU tests, 1-GPU bench, rocprofv3 kernel stats and PMC counter passes
# of the flagship round.  Usage (from the repo root, on the GPU box):
#   tools/gpu_session.sh <tag> [tests bench n8 fp32 prof pmc]   (default: tests bench prof pmc, in that order)
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
steps=${*:-tests bench prof pmc}
out=$R/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
export FEDMI_NO_BUILD=1
BENCH_ARGS=${BENCH_ARGS:-}

run_tests() {
    cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --timeout 240 --timeout-method thread \
        > $out/pytest_gpu.log 2>&1
    local rc=$?; tail -3 $out/pytest_gpu.log; return $rc
}
run_bench() {
    cd $R && timeout -k 10 400 python -u bench.py $BENCH_ARGS > $out/bench.json 2> $out/bench.err
    local rc=$?; cat $out/bench.json; return $rc
}
run_n8() {
    # a whole node's world (8 ranks) on the box's one GPU: peer self-test at world 8, classic rounds,
    # replica check (the driver's SCALE run uses 8 real GPUs)
    cd $R && timeout -k 10 500 python -u bench.py --gpus 8 --share-gpu --steps 400 --warmup 50 --no-anchor \
        --no-convergence > $out/bench_n8_share.json 2> $out/bench_n8_share.err
    local rc=$?; cat $out/bench_n8_share.json; return $rc
}
run_fp32() {
    cd $R && timeout -k 10 400 python -u bench.py --dtype fp32 --steps 2000 --warmup 200 --no-anchor \
        > $out/bench_fp32.json 2> $out/bench_fp32.err
    local rc=$?; cat $out/bench_fp32.json; return $rc
}
run_prof() {
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
        -- python $R/bench.py --no-convergence --steps 2000 --warmup 200 $BENCH_ARGS > $out/prof.log 2>&1
    local rc=$?
    python $R/tools/rocprof_summary.py stats $out/prof > $out/kernel_summary.txt 2>&1
    cat $out/kernel_summary.txt
    return $rc
}
PMC_A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
PMC_B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE FETCH_SIZE"
run_pmc() {
    local i=0 rc=0
    for set in "$PMC_A" "$PMC_B"; do
        i=$((i + 1))
        cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set -d $out/pmc$i -o run --output-format csv \
            -- python $R/bench.py --no-convergence --steps 200 --warmup 20 $BENCH_ARGS > $out/pmc$i.log 2>&1
        rc=$?
        [ $rc -ne 0 ] && { tail -5 $out/pmc$i.log; return $rc; }
    done
    python $R/tools/rocprof_summary.py pmc $out/pmc1 $out/pmc2 > $out/pmc_summary.txt 2>&1
    cat $out/pmc_summary.txt
    return 0
}

for s in $steps; do
    echo "== $s"
    run_$s || { echo "step $s failed rc=$?"; exit 1; }
done
