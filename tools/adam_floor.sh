#!/bin/bash
# Floor of the Adam kernel without (part of) its gradient-slab read: rocprofv3 kernel durations and the
# bench's us/round for the default build and FL_PROBE_SLAB_ROWS=0/64/125 variants (variants/slab*.so,
# tools/build_variant.sh slabK -DFL_PROBE_SLAB_ROWS=K).  Usage (GPU box): tools/adam_floor.sh <out_dir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp FEDMI_NO_BUILD=1
for v in default slab0 slab64 slab125 default2; do
    so=""
    case $v in default*) ;; *) so=$R/variants/$v.so ;; esac
    FEDMI_NATIVE_SO=$so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/$v -o run --output-format csv -- \
        python $R/bench.py --no-convergence --no-anchor --no-fp32 --steps 2000 --warmup 200 > $out/$v.json 2> $out/$v.err || exit 1
    python - "$v" "$out/$v" "$out/$v.json" <<'PY'
import csv, glob, json, sys
v, d, js = sys.argv[1:4]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {x["Name"]: x for x in csv.DictReader(open(f))}
us = json.loads([l for l in open(js) if l.startswith("{")][0])["us_per_round"]
ks = ", ".join(f"{n.split('(')[0][:28]} {float(x['AverageNs'])/1e3:.2f}" for n, x in rows.items()
               if "adam" in n or "train" in n)
print(f"{v:9s} bench {us:6.2f} us/round | {ks}", flush=True)
PY
done
