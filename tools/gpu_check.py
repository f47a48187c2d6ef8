"""Quick GPU validation: HIP engine vs torch engine (same init, same data)."""
import sys, time, numpy as np, torch
sys.path.insert(0, ".")
from fedmi.data.tabular import load_tabular
from fedmi.fl.engine import EngineConfig, HipRoundEngine, TorchRoundEngine
from fedmi.models.mlp import init_flat

ds = load_tabular()
X, y = ds.X_train.astype(np.float32), ds.y_train
flat = init_flat([14, 50, 200, 2], seed=0)
for R in (16, 32):
    cfg = EngineConfig(max_rounds=300, rows_per_block=R, graph_rounds=0)
    hip = HipRoundEngine(X, y, 2, cfg, None, flat)
    ref = TorchRoundEngine(X, y, 2, cfg, None, flat)
    hip.run(1); ref.run(1)
    a, b = hip.global_flat(), ref.global_flat()
    print(f"R={R} round1 max abs err {np.abs(a-b).max():.3e} rel {np.abs(a-b).max()/np.abs(b).max():.3e}",
          "metrics", hip.history()["global"][0], ref.history()["global"][0], flush=True)
cfg = EngineConfig(max_rounds=300, rows_per_block=32, graph_rounds=16)
hip = HipRoundEngine(X, y, 2, cfg, None, flat)
ref = TorchRoundEngine(X, y, 2, cfg, None, flat)
t = time.time(); nh = hip.run(300); th = time.time() - t
t = time.time(); nr = ref.run(300); tr = time.time() - t
hh, hr = hip.history(), ref.history()
print("hip rounds", nh, "stop", hh["stop_round"], "final acc", hh["global"][-1], f"{th:.3f}s")
print("ref rounds", nr, "stop", hr["stop_round"], "final acc", hr["global"][-1], f"{tr:.3f}s")
m = min(nh, nr)
print("max |acc diff| over common rounds", np.abs(hh["global"][:m, 0] - hr["global"][:m, 0]).max())
# throughput: eager and graph
for g in (0, 16):
    cfg = EngineConfig(max_rounds=100000, rows_per_block=32, graph_rounds=g, early_stop=False)
    hip = HipRoundEngine(X, y, 2, cfg, None, flat)
    hip.run(64)
    torch.cuda.synchronize()
    t = time.time(); hip.run(2048); torch.cuda.synchronize(); dt = time.time() - t
    print(f"graph_rounds={g}: {dt/2048*1e6:.1f} us/round, {len(X)*2048/dt/1e6:.1f} M samples/s", flush=True)
