"""Fixed cost of a short timed region (the driver's --steps 20 --warmup 5 shape) vs the
steady-state round: host-clock time of K rounds bracketed by synchronize on both sides, for
several graph sizes g (K / g replays), next to hipEvent time of the same replays.
Measured (profiles/launch_overhead_r2.log): a 20-round region costs ~1.5 us/round more than the
steady state (~30 us of graph-launch + synchronisation per region); starting the region with two
direct-launch rounds so the graph launch overlaps them did not help (25.6 vs 25.0 us/round).

    python tools/launch_overhead.py
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import synth_shard  # noqa: E402
from fedmi.fl.engine import EngineConfig, HipRoundEngine  # noqa: E402
from fedmi.models.mlp import init_flat  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    X, y = synth_shard(8000, 0, dev)
    dims = [14, 50, 200, 2]
    for K, gs in ((20, (2, 4, 10, 20)), (2000, (20, 50, 200))):
        for g in gs:
            cfg = EngineConfig(hidden=(50, 200), max_rounds=5 + 3 * K + 3 * g + 64, early_stop=False,
                               rows_per_block=32, graph_rounds=g, dtype="bf16")
            eng = HipRoundEngine(X, y, 2, cfg, None, init_flat(dims, seed=0))
            eng.run(5, check_every=5)
            eng.prime_graph(g)
            eng.stream.synchronize()
            res = []
            for rep in range(3):
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(eng.stream)
                eng._issue(K, close=False)
                e1.record(eng.stream)
                eng.stream.synchronize()
                torch.cuda.synchronize(dev)
                dt = time.perf_counter() - t0
                res.append((dt / K * 1e6, e0.elapsed_time(e1) / K * 1e3))
            print(f"K={K:5d} g={g:3d}: host us/round " + " ".join(f"{h:6.2f}" for h, _ in res) +
                  " | event us/round " + " ".join(f"{e:6.2f}" for _, e in res), flush=True)


if __name__ == "__main__":
    main()
