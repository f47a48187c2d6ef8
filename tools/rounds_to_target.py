"""Rounds-to-target of the reference [C] workload (real income CSV, compat mode) with the fp32 and
bf16 kernels on one GPU: early-stop behaviour differs (see bench.py)."""
import sys, json
sys.path.insert(0, ".")
import bench
from fedmi.parallel.comm import get_world
comm = get_world(backend="xgmi", device="cuda")
for dt in ("fp32", "bf16"):
    print(dt, json.dumps(bench.rounds_to_target(comm, dtype=dt)), flush=True)
