#!/bin/bash
# round-2 GPU pass f: profile of the split-bf16 round (kernel stats, PMC, in-kernel phase stamps)
set -o pipefail
mkdir -p gpurun_out/r2f
export FEDMI_NO_BUILD=1
timeout -k 10 120 python tools/stamps.py 8000 32 50,200 bf16 > gpurun_out/r2f/stamps.log 2>&1 || exit $?
cat gpurun_out/r2f/stamps.log
bash tools/gpu_session.sh r2f/session prof pmc
