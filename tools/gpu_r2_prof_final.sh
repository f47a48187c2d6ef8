#!/bin/bash
# final-tree profiles of the one-client round: rocprofv3 kernel stats + two PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/prof_final
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python $R/bench.py --no-convergence --no-anchor --steps 2000 --warmup 200 > $out/stats.log 2>&1 || { tail $out/stats.log; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $out/pmc1 -o run --output-format csv -- python $R/bench.py --no-convergence --no-anchor --steps 400 --warmup 50 > $out/pmc1.log 2>&1 || { tail -5 $out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $out/pmc2 -o run --output-format csv -- python $R/bench.py --no-convergence --no-anchor --steps 400 --warmup 50 > $out/pmc2.log 2>&1 || { tail -5 $out/pmc2.log; exit 1; }
cd $R
python tools/rocprof_summary.py stats $out/stats > $out/stats.txt 2>&1
python tools/rocprof_summary.py pmc $out/pmc1 $out/pmc2 > $out/pmc.txt 2>&1
head -8 $out/stats.txt
grep -A20 "fl_train_bf16_kernel" $out/pmc.txt | head -22
