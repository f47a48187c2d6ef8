#!/bin/bash
# round-2 GPU pass k: bank-conflict-free bf16 LDS layout (level 1 for the flagship): GPU tests,
# bench, kernel stats, PMC (SQ_LDS_BANK_CONFLICT), in-kernel phase stamps incl. the Adam kernel
set -o pipefail
mkdir -p gpurun_out/r2k
export FEDMI_NO_BUILD=1
bash tools/gpu_session.sh r2k/session tests bench prof pmc || exit $?
timeout -k 10 120 python tools/stamps.py 8000 32 50,200 bf16 > gpurun_out/r2k/stamps.log 2>&1 || exit $?
cat gpurun_out/r2k/stamps.log
