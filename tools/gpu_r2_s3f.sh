#!/bin/bash
# final-tree check: GPU suite, smoke, headline bench (driver-shaped and long), N=2 shared, config-5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3f_pytest.log 2>&1 || { tail -40 gpurun_out/s3f_pytest.log; exit 1; }
tail -2 gpurun_out/s3f_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3f_smoke.log 2>&1 || { tail gpurun_out/s3f_smoke.log; exit 1; }
grep smoke gpurun_out/s3f_smoke.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/s3f_b20.json 2> gpurun_out/s3f_b20.err || { tail gpurun_out/s3f_b20.err; exit 1; }
timeout -k 10 180 python bench.py --steps 2000 --warmup 200 > gpurun_out/s3f_b2000.json 2> gpurun_out/s3f_b2000.err || { tail gpurun_out/s3f_b2000.err; exit 1; }
timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 400 --warmup 50 --no-anchor > gpurun_out/s3f_n2.json 2> gpurun_out/s3f_n2.err || { tail gpurun_out/s3f_n2.err; exit 1; }
timeout -k 10 120 python bench.py --config sweep --steps 400 --warmup 32 > gpurun_out/s3f_sweep.json 2> gpurun_out/s3f_sweep.err || { tail gpurun_out/s3f_sweep.err; exit 1; }
for f in b20 b2000 n2 sweep; do python -c "import json;d=json.load(open('gpurun_out/s3f_$f.json'));print('$f', d['n_gpus'], round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']), d.get('rounds_to_target'))"; done
