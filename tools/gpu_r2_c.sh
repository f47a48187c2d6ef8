#!/bin/bash
# round-2 GPU pass c: peer protocol with release/acquire ordering, early-stop argument test, NT GEMM cleanup
set -o pipefail
mkdir -p gpurun_out/r2c
export FEDMI_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_peer_allreduce.py tests/test_engine_cpu.py tests/test_bench_contract.py tests/test_hip_engine.py -k "peer or early_stop or bench or gemm_nt or wide" > gpurun_out/r2c/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r2c/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/round_emulate.py --rounds 2000 > gpurun_out/r2c/round_emulate.log 2>&1 || exit $?
cat gpurun_out/r2c/round_emulate.log
timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 400 --warmup 50 --no-anchor > gpurun_out/r2c/bench_n2share.json 2> gpurun_out/r2c/bench_n2share.err || exit $?
cat gpurun_out/r2c/bench_n2share.json
