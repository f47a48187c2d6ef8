#!/bin/bash
# round-2 GPU pass x: wide path with a padded partial last micro-batch -- wide tests, config 3 at size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2x
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hip_engine.py tests/test_wide_fedavg.py -m gpu -x -v \
    --timeout 120 --timeout-method thread -k "wide" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 600 python -u bench.py --config wide --wide-rows 12500000 --steps 2 --warmup 1 > $out/bench_wide_12p5M.json 2> $out/bench_wide.err || { tail -20 $out/bench_wide.err; exit 1; }
cat $out/bench_wide_12p5M.json
