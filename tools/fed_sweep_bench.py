"""Concurrent-trial packing (BASELINE config 5) on one GPU, one client: trial-rounds/s of a
12-trial federated sweep (hidden {(50,200),(100,50),(50,100)} x lr {0.002,0.004} x local steps
{1,2}, 8000 rows, 100 rounds), for

  * sequential: one trial after another, each engine replaying its own 16-round HIP graphs;
  * packed K:  K trials at once (fedmi.hpo.fed_sweep.FedTrialGroup: same-shape trials as one
               native trial batch -- every kernel of the round launched once for all of them --
               shapes on their own streams, the whole K-trial round captured into ONE graph);
  * streams K: the same without trial batches (every trial on its own stream, round-2 design).

    python tools/fed_sweep_bench.py [--rounds 100]
"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from fedmi.data.synthetic import make_income_like  # noqa: E402
from fedmi.fl.engine import EngineConfig, HipRoundEngine  # noqa: E402
from fedmi.hpo.fed_sweep import FedTrialGroup, grid, run_fed_sweep  # noqa: E402
from fedmi.models.mlp import init_flat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--rows", type=int, default=8000,
                    help="rows per trial (client shard): 8000 = one client, 1000 = the 8-client shard of config 5")
    ap.add_argument("--grids", default="mixed-fp32,mixed-bf16,same-bf16")
    a = ap.parse_args()
    X, y = make_income_like(a.rows, seed=1)
    print(f"== {a.rows} rows per trial", flush=True)
    mixed = grid(((50, 200), (100, 50), (50, 100)), (0.002, 0.004), (1, 2))
    same = grid(((50, 200),), (0.001, 0.002, 0.003, 0.004, 0.006, 0.01), (1, 2))  # one shape: one batch of 12
    R = a.rounds
    want = set(a.grids.split(","))
    cases = [(n, t, d) for n, t, d in (("mixed", mixed, "fp32"), ("mixed", mixed, "bf16"), ("same-shape", same, "bf16"))
             if f"{n.split('-')[0]}-{d}" in want]
    for name, trials, dtype in cases:
        print(f"-- {name} grid: {len(trials)} trials, shapes {sorted({t.hidden for t in trials})}", flush=True)
        base = EngineConfig(max_rounds=R + 48, early_stop=False, dtype=dtype, graph_rounds=16)
        # warm-up: compile / first launches
        run_fed_sweep(X, y, 2, None, trials[:2], rounds=20, trials_per_gpu=2, base=base)
        # sequential, graph-replayed engines
        engines = [HipRoundEngine(X, y, 2, EngineConfig(hidden=t.hidden, lr=t.lr, local_steps=t.local_steps,
                                                        max_rounds=R + 32, early_stop=False, dtype=dtype,
                                                        graph_rounds=16), None, init_flat([14, *t.hidden, 2], 0))
                   for t in trials]
        for e in engines:
            e.run(18)                       # capture + first replay outside the timing
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e in engines:
            e.run(R)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        seq = len(trials) * R / dt
        print(f"{dtype} sequential graph-replayed engines: {len(trials)} trials x {R} rounds in {dt * 1e3:.1f} ms "
              f"({seq:.0f} trial-rounds/s)", flush=True)
        for k, batched in ((1, True), (4, True), (12, True), (12, False)):
            groups = [FedTrialGroup(X, y, 2, trials[g:g + k], None, base, batched=batched)
                      for g in range(0, len(trials), k)]
            for g in groups:
                g.run(16)                   # group graph captured + replayed once outside the timing
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for g in groups:
                g.run(R)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            done = [t for g in groups for t in g.trials]
            best = max(done, key=lambda t: t.final["accuracy"])
            print(f"{dtype} {'packed' if batched else 'streams'} trials_per_gpu={k:2d}: {len(done)} trials x {R} rounds in {dt * 1e3:.1f} ms "
                  f"({len(done) * R / dt:.0f} trial-rounds/s, {len(done) * R / dt / seq:.2f}x sequential); "
                  f"best {best.hidden} lr={best.lr} ls={best.local_steps} acc={best.final['accuracy']:.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
