set -o pipefail
o=gpurun_out/r4h; mkdir -p $o
export FEDMI_NO_BUILD=1
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-convergence --no-anchor --no-fp32 >> $o/bench_driver_shape.jsonl 2>> $o/bench.err || exit 1; done
timeout -k 10 300 python -u bench.py --config wide --wide-rows 12500000 --steps 3 --warmup 1 > $o/wide_12p5M_fused.json 2>> $o/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config wide --wide-rows 12500000 --steps 3 --warmup 1 --no-fused-eval > $o/wide_12p5M_separate_eval.json 2>> $o/bench.err || exit 1
cat $o/*.json*
