set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 120 python tools/stamps.py 8000 32 50,200 bf16 > gpurun_out/r4d/stamps_noes.log 2>&1 &&
FEDMI_STAMPS_ES=1 timeout -k 10 120 python tools/stamps.py 8000 32 50,200 bf16 > gpurun_out/r4d/stamps_es.log 2>&1 &&
timeout -k 10 600 python -u tools/round_emulate.py --rows 8000 4000 2000 1000 --rpb 16 32 --rounds 2000 > gpurun_out/r4d/emulate.log 2>&1
rc=$?; tail -5 gpurun_out/r4d/emulate.log; exit $rc
