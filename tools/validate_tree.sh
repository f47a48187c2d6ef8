set -o pipefail
D=gpurun_out/${VAL_TAG:-r6v}
mkdir -p $D
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail -20 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $D/driver_$i.json 2> $D/driver_$i.err || { echo "bench $i failed"; tail -20 $D/driver_$i.err; exit 1; }
  grep -o '"us_per_round": [0-9.]*' $D/driver_$i.json | head -1
done
