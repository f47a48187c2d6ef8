"""Finer phase split of the bf16 (argv[1] = fp32: the fp32) train kernel's backward pass (a FL_STAMP_FINE build:
tools/build_variant.sh fine -DFL_STAMP_FINE, FEDMI_NATIVE_SO=variants/fine.so).  Per workgroup:
3 -> 14 head wgrad, 14 -> 4 head dgrad + barrier, 4 -> 7 layer L-2 wgrad (+ bias sums),
7 -> 13 its dgrad, 13 -> 5 barrier wait, 5 -> 6 layer 0 wgrad."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, HipRoundEngine
from fedmi.models.mlp import init_flat

rows, R = 8000, 32
dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
X, y = make_income_like(rows, seed=1)
cfg = EngineConfig(hidden=(50, 200), max_rounds=100, rows_per_block=R, graph_rounds=0, early_stop=False,
                   dtype=dtype)
e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 0))
e.run(3)
nb = (rows + R - 1) // R
dbg = torch.zeros(nb * 16, dtype=torch.int64, device=e.device)
meds = []
for rep in range(20):
    dbg.zero_()
    e.engine.set_debug(dbg.data_ptr())
    e.engine.launch_one(e.rounds_issued - 1, 0, e._stream())
    e.stream.synchronize()
    e.engine.set_debug(0)
    st = dbg.view(nb, 16).cpu().numpy().astype(np.int64)
    meds.append(st)
st = np.stack(meds[5:])  # [reps, blocks, 16]
# slots 11 / 12 were overwritten by the last wave's dgrad start / end of layer L-2
d = (st[:, :, 12] - st[:, :, 11]) * 10 / 1000.0
print(f"layer L-2 dgrad on the last wave: median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f} us")
d = (st[:, :, 11] - st[:, :, 4]) * 10 / 1000.0
print(f"  its start after wave 0's stamp 4: median {np.median(d):6.2f} us")
# fp32: slots 13 / 14 hold s_memtime (core clock), 8 / 9 / 14 are not bf16's phases
order = [0, 8, 9, 1, 10, 2, 3, 14, 4, 7, 13, 5, 6, 15] if dtype == "bf16" else [0, 1, 10, 2, 3, 4, 7, 5, 6, 15]
for a, b in zip(order[:-1], order[1:]):
    d = (st[:, :, b] - st[:, :, a]) * 10 / 1000.0
    print(f"phase {a:2d} -> {b:2d}: median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f} us")
tot = (st[:, :, 15].max(axis=1) - st[:, :, 0].min(axis=1)) * 10 / 1000.0
print(f"kernel span median {np.median(tot):.2f} us")
