"""Concurrent-trial packing: wall time of a 12-trial federated sweep, packed K per GPU vs
one trial at a time (1 client)."""
import sys, time, torch
sys.path.insert(0, ".")
from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig
from fedmi.hpo.fed_sweep import grid, run_fed_sweep
X, y = make_income_like(8000, seed=1)

for dtype in ("fp32", "bf16"):
    for k in (1, 4, 12):
        base = EngineConfig(max_rounds=100, early_stop=False, dtype=dtype, graph_rounds=0)
        run_fed_sweep(X, y, 2, None, grid(((16,),), (0.01,), (1,)), rounds=5, trials_per_gpu=1, base=base)
        torch.cuda.synchronize()
        t0 = time.time()
        best, done = run_fed_sweep(X, y, 2, None, grid(((50, 200), (100, 50), (50, 100)), (0.002, 0.004), (1, 2)),
                                   rounds=100, trials_per_gpu=k, base=base)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"{dtype} trials_per_gpu={k:2d}: {len(done)} trials x 100 rounds in {dt:.3f} s "
              f"({len(done) * 100 / dt:.0f} trial-rounds/s); best {best.hidden} lr={best.lr} ls={best.local_steps} "
              f"acc={best.final['accuracy']:.4f}", flush=True)
