#!/bin/bash
# round-2 GPU pass o: full-line NT GEMM (variant 3) -- PMC pass (MFMA busy share) for variants 2 and 3,
# wide benches (131k rows, 12.5 M rows = BASELINE config 3 at size) with the new default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2o
mkdir -p $out
export FEDMI_NO_BUILD=1 TMPDIR=/tmp
PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in 2 3; do
    cd $R && timeout -s KILL 120 rocprofv3 --pmc $PMC -d $out/pmc_v$v -o run --output-format csv \
        -- python tools/nt_prof.py 16384 4096 4096 $v > $out/pmc_v$v.log 2>&1 || { tail -5 $out/pmc_v$v.log; exit 1; }
done
python tools/rocprof_summary.py pmc $out/pmc_v2 > $out/pmc_v2.txt 2>&1
python tools/rocprof_summary.py pmc $out/pmc_v3 > $out/pmc_v3.txt 2>&1
grep -A16 "gemm_nt" $out/pmc_v2.txt | head -18
grep -A16 "gemm_nt" $out/pmc_v3.txt | head -18
cd $R && timeout -k 10 300 python bench.py --config wide --steps 5 --warmup 2 > $out/bench_wide_131k.json 2> $out/bench_wide_131k.err || exit $?
cat $out/bench_wide_131k.json
cd $R && timeout -k 10 400 python bench.py --config wide --wide-rows 12500000 --steps 2 --warmup 1 > $out/bench_wide_12p5M.json 2> $out/bench_wide_12p5M.err || exit $?
cat $out/bench_wide_12p5M.json
