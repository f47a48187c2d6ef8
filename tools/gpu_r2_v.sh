#!/bin/bash
# round-2 GPU pass v: LL exchange with sentinel-first polling -- peer tests, emulated round,
# 2 clients sharing the GPU with LL and with publish / wait / pull chunks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r2v
mkdir -p $out
export TMPDIR=/tmp FEDMI_NO_BUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_peer_allreduce.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 200 python -u tools/round_emulate.py > $out/emulate.log 2>&1 || { tail -20 $out/emulate.log; exit 1; }
grep -v amdgpu.ids $out/emulate.log
for v in 1 0 1 0; do
  FEDMI_PEER_LL=$v timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --no-convergence --steps 2000 --warmup 200 \
      > $out/n2_ll$v.json 2> $out/n2_ll$v.err || { tail -20 $out/n2_ll$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/n2_ll$v.json').read().strip().splitlines()[-1]);print('LL=$v', round(d['us_per_round'],2), 'us/round', d['config']['data_plane'])"
done
