#!/bin/bash
# trial batches: GPU tests of the sweep group + packing bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fed_sweep.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tb_pytest.log 2>&1 || { tail -30 gpurun_out/tb_pytest.log; exit 1; }
tail -3 gpurun_out/tb_pytest.log
timeout -k 10 300 python -u tools/fed_sweep_bench.py > gpurun_out/tb_bench.log 2>&1 || { tail -30 gpurun_out/tb_bench.log; exit 1; }
cat gpurun_out/tb_bench.log
