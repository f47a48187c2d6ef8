#!/bin/bash
# round-2 GPU pass p: instruction-fetch counters of the fused round kernels (is the latency-bound
# train kernel waiting on instruction fetch?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2p
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
PMC="SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_INSTS_SALU"
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $PMC -d $out/pmc -o run --output-format csv \
    -- python $R/bench.py --no-convergence --steps 200 --warmup 20 > $out/pmc.log 2>&1 || { tail -5 $out/pmc.log; exit 1; }
python $R/tools/rocprof_summary.py pmc $out/pmc > $out/pmc_summary.txt 2>&1
head -40 $out/pmc_summary.txt
