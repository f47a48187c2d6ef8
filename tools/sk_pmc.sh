#!/bin/bash
# PMC counters of the sklearn float64 minibatch step (tools/sk_step_bench.py --fused-only --case <c>), two passes.
# Usage (GPU box): tools/sk_pmc.sh <out> [case]
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-skpmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp FEDMI_NO_BUILD=1
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE FETCH_SIZE"
i=0
for set in "$A" "$B"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $out/pmc$i -o run --output-format csv -- \
        python $R/tools/sk_step_bench.py --fused-only --case ${2:-0} > $out/pmc$i.log 2>&1 || { tail -5 $out/pmc$i.log; exit 1; }
done
python $R/tools/rocprof_summary.py pmc $out/pmc1 $out/pmc2 > $out/pmc_summary.txt 2>&1
cat $out/pmc_summary.txt
