"""Debug: config-5 bench path, per-trial final metrics (batched vs streams, device vs host data)."""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from fedmi.fl.engine import EngineConfig
from fedmi.hpo.fed_sweep import FedTrialGroup, grid
from fedmi.data.synthetic import device_shard, make_income_like

trials = grid(((50, 200), (100, 50)), (0.002,), (1, 2))
for data in ("device", "host"):
    if data == "device":
        X, y = device_shard(8000, 0, torch.device("cuda", 0), 7)
    else:
        X, y = make_income_like(8000, seed=1)
    for batched in (True, False):
        base = EngineConfig(max_rounds=84, early_stop=False, dtype="bf16", graph_rounds=16)
        g = FedTrialGroup(X, y, 2, grid(((50, 200), (100, 50)), (0.002,), (1, 2)), None, base,
                          group_graph_rounds=16, batched=batched)
        g.run(32)
        a = [(t.rounds_run, round(t.final["accuracy"], 4)) for t in g.trials]
        g.run(32)
        b = [(t.rounds_run, round(t.final["accuracy"], 4)) for t in g.trials]
        print(data, "batched" if batched else "streams", a, b, flush=True)
