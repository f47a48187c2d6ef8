"""Where does the driver-shaped timed region (bench.py --steps 20 --warmup 5) lose time against
the steady state?  Builds bench.py's one-client engine (8000 rows, early-stop rule live), then
for several timed-region shapes reports, per repetition:

  wall    host perf_counter from t0 to after the final synchronize (what bench.py times)
  gpu     hipEvent elapsed from an event recorded just before the first replay to one after
          the last (device time of the region, launch gap of the first kernel excluded)
  issue   host time until the replay call(s) returned
  lead    wall - gpu: host launch latency + synchronize wake-up
  per-replay device time (events between g-round replays) to expose a slow start (clocks,
  cold caches) inside the region

    python tools/short_region.py [--rows 8000] [--reps 8]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--idle-us", type=float, nargs="+", default=[0.0, 200.0, 5000.0],
                    help="host sleep between the pre-region synchronize and t0")
    ap.add_argument("--fresh", type=int, default=3, help="fresh engines whose first timed replays are reported")
    ap.add_argument("--fresh-only", action="store_true")
    ap.add_argument("--shift-kb", type=int, nargs="*", default=[],
                    help="per fresh engine: KB of device memory allocated (and kept) before it")
    a = ap.parse_args()
    import numpy as np
    if os.environ.get("FEDMI_SPIN_SYNC", "0") == "1":
        # synchronizations spin instead of yielding (hipDeviceScheduleSpin = 1), set before torch
        # creates the device context
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)
    import torch
    import bench
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y = bench.synth_shard(a.rows, 0, dev)
    total = 200000

    def engine(g):
        cfg = EngineConfig(max_rounds=total, early_stop=True, patience=total + 1, graph_rounds=g, dtype="bf16")
        e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 0), n_total=a.rows)
        e.run(5, check_every=5)
        e.prime_graph(g)
        e.stream.synchronize()
        return e

    print(f"rows {a.rows}; times in us; device clock not pinned", flush=True)
    # fresh engines, bench.py's exact sequence (warm-up rounds, prime = capture + first replay),
    # then successive K = 20 regions of one g = 20 replay each: is the first timed replay (the
    # graph's second launch, what bench.py times) slower than later ones?
    pads = []
    for trial in range(a.fresh):
        if a.shift_kb:   # shift the engine's allocations: a pad of shift_kb[trial] KB allocated (and kept) first
            kb = a.shift_kb[trial % len(a.shift_kb)]
            if kb:
                pads.append(torch.empty(kb * 256, dtype=torch.float32, device=dev))
        e = engine(20)
        print(f"engine {trial}: slab {e.slab.data_ptr():#x} X {e.X.data_ptr():#x} params {e.params[0].data_ptr():#x} "
              f"(mod 2 MiB: slab {e.slab.data_ptr() % (2 << 20):#x})", flush=True)
        walls, gpus = [], []
        for rep in range(6):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e.stream.synchronize()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ev0.record(e.stream)
            e.engine.replay(e._stream())
            ev1.record(e.stream)
            e.rounds_issued += 20
            e.stream.synchronize()
            torch.cuda.synchronize(dev)
            walls.append((time.perf_counter() - t0) * 1e6 / 20)
            gpus.append(ev0.elapsed_time(ev1) * 1e3 / 20)
        print(f"fresh engine {trial}: launch 2..7 wall/round " + " ".join(f"{w:.2f}" for w in walls)
              + "  gpu/round " + " ".join(f"{g:.2f}" for g in gpus), flush=True)
        del e
    if a.fresh_only:
        return
    for K, g in ((20, 0), (20, 20), (20, 10), (20, 4), (20, 2), (200, 0), (200, 20), (2000, 40)):
        e = engine(g if g else 20)
        for idle in a.idle_us:
            rows = []
            for rep in range(a.reps):
                n_rep = K // g if g else 1
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(n_rep + 1)]
                e.stream.synchronize()
                torch.cuda.synchronize(dev)
                if idle > 0:
                    t_idle = time.perf_counter() + idle * 1e-6
                    while time.perf_counter() < t_idle:
                        pass
                t0 = time.perf_counter()
                s = e._stream()
                evs[0].record(e.stream)
                if g == 0:   # eager: the K rounds' kernels launched by one native call
                    e.engine.run(e.rounds_issued, K, s, None, False)
                    evs[1].record(e.stream)
                for i in range(n_rep if g else 0):
                    e.engine.replay(s)
                    evs[i + 1].record(e.stream)
                e.rounds_issued += K
                t_issue = time.perf_counter()
                e.stream.synchronize()
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                per = [evs[i].elapsed_time(evs[i + 1]) * 1e3 / (g or K) for i in range(n_rep)]
                gpu = evs[0].elapsed_time(evs[-1]) * 1e3
                rows.append(((t1 - t0) * 1e6, gpu, (t_issue - t0) * 1e6, per))
            wall = np.array([r[0] for r in rows])
            gpu = np.array([r[1] for r in rows])
            iss = np.array([r[2] for r in rows])
            per = np.array([r[3] for r in rows])
            print(f"K={K:5d} g={g:3d} idle={idle:7.0f}: wall/round {np.median(wall) / K:6.2f} "
                  f"gpu/round {np.median(gpu) / K:6.2f} lead {np.median(wall - gpu):7.1f} "
                  f"issue {np.median(iss):7.1f}  per-replay us/round (median over reps): "
                  + " ".join(f"{v:.2f}" for v in np.median(per, axis=0)[:12]), flush=True)
        del e


if __name__ == "__main__":
    main()
