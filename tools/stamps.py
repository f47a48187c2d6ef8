"""Per-phase in-kernel timing (s_memrealtime stamps, 10 ns ticks) of the fused kernels.

Train-kernel slots: 0 start, 1 staged, 10+l start of forward layer l, 2 forward done,
3 CE done, 4.. backward phases, 15 end; 13/14 = s_memtime (core clock) at start / after
forward, used to report the effective shader clock.  Adam-kernel slots (parameter blocks):
0 start, 1 first slab batch issued, 2 round state folded, 3 slab sums done, 4 partials
combined, 5 update stored, 15 stores complete; "train->adam" = the gap between the last train
workgroup's end and the first Adam block's start when the two are launched back to back."""
import os, sys, numpy as np, torch
sys.path.insert(0, ".")
from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, HipRoundEngine
from fedmi.models.mlp import init_flat
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 32
hidden = tuple(int(h) for h in sys.argv[3].split(",")) if len(sys.argv) > 3 else (50, 200)
dtype = sys.argv[4] if len(sys.argv) > 4 else "fp32"
X, y = make_income_like(rows, seed=1)
# FEDMI_STAMPS_ES=1: early stopping on (every Adam block's wave 0 folds the round state)
cfg = EngineConfig(hidden=hidden, max_rounds=100, rows_per_block=R, graph_rounds=0,
                   early_stop=os.environ.get("FEDMI_STAMPS_ES", "0") == "1", patience=1000, dtype=dtype)
# 5th argument "emulate": a multi-client engine (emulate_clients: lagged rounds, plain-bf16 training forward)
emulate = len(sys.argv) > 5 and sys.argv[5] == "emulate"
if emulate:
    cfg.fused_eval = False
e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, *hidden, 2], 0), emulate_clients=emulate)
e.run(3)
nb = (rows + R - 1) // R
dbg = torch.zeros(nb * 16, dtype=torch.int64, device=e.device)
order = [0, 8, 9, 1, 10, 11, 12, 2, 3, 4, 5, 6, 7, 15]
kinds = [(0, "train"), (2, "eval")] + ([(3, "train, lagged scoring")] if dtype == "bf16" else [])
nadam = 1 + (e.engine.layout()["P"] + 63) // 64 if "P" in e.engine.layout() else None
for which, name in kinds:
    for rep in range(5):
        dbg.zero_()
        e.set_debug(dbg.data_ptr())
        e.engine.launch_one(e.rounds_issued - 1, which, e._stream())
        e.stream.synchronize()
        e.set_debug(0)
    st = dbg.view(nb, 16).cpu().numpy().astype(np.int64)
    t0 = st[:, 0].min()
    print(f"{name}: blocks={nb} dispatch spread={(st[:,0].max()-t0)*10/1000:.2f}us "
          f"total={(st[:,15].max()-t0)*10/1000:.2f}us")
    if which == 0 and (st[:, 13] > 0).all():
        cyc = st[:, 14] - st[:, 13]
        real = (st[:, 2] - st[:, 0]) * 10e-9
        print(f"   effective shader clock over start..forward: {np.median(cyc / real) / 1e9:.2f} GHz")
    if which == 3 and (st[:, 14] > 0).all():  # register scoring (score_in / score_out)
        fine = ((7, "scoring: rows loaded"), (10, "scoring: first W tile in"), (11, "scoring: first hidden layer"))
        for c, what in fine:
            if (st[:, c] > 0).all():
                d = (st[:, c] - st[:, 0]) * 10 / 1000
                print(f"   {what:28s} 0->{c}: median {np.median(d):7.2f} us  max {d.max():7.2f} us")
        for c, what in ((13, "scoring: past staging"), (12, "scoring: 2 tile pairs"), (14, "scoring: logits")):
            if (st[:, c] > 0).all():
                d = (st[:, c] - st[:, 1]) * 10 / 1000
                print(f"   {what:28s} 1->{c}: median {np.median(d):7.2f} us  max {d.max():7.2f} us")
        d = (st[:, 2] - st[:, 1]) * 10 / 1000
        print(f"   {'training forward':28s} 1->2: median {np.median(d):7.2f} us  max {d.max():7.2f} us")
    cols = [i for i in order if (st[:, i] > 0).all()]
    prev = cols[0]
    for c in cols[1:]:
        d = (st[:, c] - st[:, prev]) * 10 / 1000
        print(f"   phase {prev:2d}->{c:2d}: median {np.median(d):7.2f} us  max {d.max():7.2f} us")
        prev = c

# Adam kernel phases (parameter blocks only: block 0 is the metric-tail block)
if nadam is not None:
    dt = torch.zeros(nb * 16, dtype=torch.int64, device=e.device)
    da = torch.zeros(max(nb, nadam) * 16, dtype=torch.int64, device=e.device)
    gaps = []
    for rep in range(5):
        dt.zero_()
        da.zero_()
        e.set_debug(dt.data_ptr())
        e.engine.launch_one(e.rounds_issued - 1, 0, e._stream())
        e.set_debug(da.data_ptr())
        e.engine.launch_one(e.rounds_issued - 1, 1, e._stream())
        e.stream.synchronize()
        e.set_debug(0)
        t = dt.view(nb, 16).cpu().numpy().astype(np.int64)
        a = da.view(-1, 16).cpu().numpy().astype(np.int64)[1:nadam]
        gaps.append((a[:, 0].min() - t[:, 15].max()) * 10 / 1000)
    t0 = a[:, 0].min()
    print(f"adam: param blocks={nadam - 1} dispatch spread={(a[:,0].max()-t0)*10/1000:.2f}us "
          f"total={(a[:,15].max()-t0)*10/1000:.2f}us  train->adam gap median {np.median(gaps):.2f}us")
    prev = 0
    for c in [1, 2, 3, 4, 5, 15]:
        if not (a[:, c] > 0).all():
            continue
        d = (a[:, c] - a[:, prev]) * 10 / 1000
        print(f"   phase {prev:2d}->{c:2d}: median {np.median(d):7.2f} us  max {d.max():7.2f} us")
        prev = c
