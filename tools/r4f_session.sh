set -o pipefail
o=gpurun_out/r4f; mkdir -p $o
export FEDMI_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --deselect "tests/test_simulate.py::test_hip_client_group_tracks_torch[fp32-None]" -x --timeout 240 --timeout-method thread > $o/pytest_gpu.log 2>&1; rc=$?
tail -3 $o/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-convergence --no-anchor --no-fp32 >> $o/bench_es.jsonl 2>> $o/bench.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-convergence --no-anchor --no-fp32 --no-early-stop >> $o/bench_noes.jsonl 2>> $o/bench.err || exit 1
done
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-convergence --no-anchor --no-fp32 >> $o/bench_driver_shape.jsonl 2>> $o/bench.err || exit 1; done
timeout -k 10 300 python -u tools/short_region.py --reps 6 > $o/short_region.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/round_emulate.py --rows 8000 2000 1000 --rounds 2000 --cases world1-fused lag+adamx lag+adamx+es rccl-lag rccl-lag+es > $o/emulate.log 2>&1
