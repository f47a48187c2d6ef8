"""Per-kernel device times of the fused round (hipEvent timing), for several R."""
import sys, json, numpy as np, torch
sys.path.insert(0, ".")
from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, HipRoundEngine
from fedmi.models.mlp import init_flat
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
hidden = tuple(int(h) for h in sys.argv[2].split(",")) if len(sys.argv) > 2 else (50, 200)
X, y = make_income_like(rows, seed=1)
dims = [14, *hidden, 2]
for R in (16, 32):
    cfg = EngineConfig(hidden=hidden, max_rounds=100, rows_per_block=R, graph_rounds=0, early_stop=False)
    try:
        e = HipRoundEngine(X, y, 2, cfg, None, init_flat(dims, 0))
    except Exception as ex:
        print("R", R, "skip", ex); continue
    e.run(2)
    t = e.engine.time_kernels(e.rounds_issued - 1, 200, e._stream())
    print(json.dumps({"rows": rows, "hidden": hidden, "R": R, **{k: round(v, 2) for k, v in t.items()}}), flush=True)
