#!/bin/bash
# Adam without peer paths (loc) vs general-only (gen) vs previous commit (head): headline + 2 ranks sharing a GPU
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_bench.sh gpurun_out/ab_lag 3 head lag || exit 1
for v in head lag; do
  FEDMI_NATIVE_SO=$PWD/variants/$v.so timeout -k 10 200 python bench.py --gpus 2 --share-gpu --steps 400 --warmup 50 --no-anchor --no-convergence > gpurun_out/ab_lag/n2_$v.json 2> gpurun_out/ab_lag/n2_$v.err || { tail gpurun_out/ab_lag/n2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_lag/n2_$v.json'));print('n2 $v', round(d['ms_per_step']*1e3,2), 'us/round')"
done
