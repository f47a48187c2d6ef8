set -o pipefail
o=gpurun_out/r4e; mkdir -p $o
timeout -k 10 300 python -u tools/short_region.py > $o/short_region.log 2>&1 &&
timeout -k 10 300 python -u tools/round_emulate.py --rows 8000 2000 1000 --rounds 2000 --cases world1-fused lag+adamx+es rccl-lag+es > $o/emulate_auto.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-convergence --no-anchor --no-fp32 >> $o/bench_driver_shape.jsonl 2>> $o/bench.err || exit 1; done
rc=$?; cat $o/short_region.log; exit $rc
