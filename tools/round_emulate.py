"""Emulate the multi-client round on ONE GPU (the 1-GPU box cannot run real xGMI): a one-rank
peer all-reduce gives every kernel of a world > 1 round its real shape -- classic evaluation
of the post-step model, the all-reduce kernel with its bf16 pack epilogue -- minus the xGMI
latency of the pulls.  Prints us/round for

  * world 1, fused evaluation (what bench.py runs at N = 1);
  * classic evaluation + separate one-shot all-reduce kernel;
  * the fused evaluation + FedAvg kernel (N > 1 with early stopping);
  * lagged evaluation: round r scored inside round r+1's train kernel, no evaluation kernel,
    with a separate all-reduce kernel or with the FedAvg inside the Adam kernel
    (N > 1 without early stopping: bench.py).

    python tools/round_emulate.py [--rounds 2000] [--dtype bf16]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2000)
    ap.add_argument("--rows", type=int, default=8000)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    import torch
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    from fedmi.ops import native
    import bench
    m = native()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y = bench.synth_shard(a.rows, 0, dev)
    flat = init_flat([14, 50, 200, 2], 0)
    cases = (("world 1, fused evaluation", True, None, False, 0), ("eval + one-shot all-reduce", False, False, False, 0),
             ("fused eval + FedAvg kernel", False, True, False, 0),
             ("lagged eval + all-reduce kernel", False, True, True, 0),
             ("lagged eval + FedAvg in Adam", False, True, True, 1),
             ("same + early stopping (LAG fold)", False, True, True, 2))
    for name, fused, ef, lag, adam_x in cases:
        if lag and a.dtype != "bf16":
            continue
        # adam_x == 2: early stopping on (patience never reached), so every round's Adam blocks
        # wait for the lagged-metric chunk of the round before (N > 1 with early stopping)
        cfg = EngineConfig(max_rounds=a.rounds + 256, early_stop=adam_x == 2, patience=10 ** 6,
                           dtype=a.dtype, graph_rounds=16,
                           fused_eval=fused, eval_fedavg=bool(ef), lagged_eval=lag)
        e = HipRoundEngine(X, y, 2, cfg, None, flat, emulate_clients=lag)
        h = None
        if ef is not None:
            h = m.PeerAllReduce(1, 0, 0, int(e.params[0].numel()), 10.0, (e.P + 63) // 64 + 2 if adam_x else 0)
            h.open([h.handle()])
            h.clear()
            e.engine.attach_peer(h)
        e.run(64)
        e.stream.synchronize()
        t0 = time.perf_counter()
        e._issue(a.rounds)
        e.stream.synchronize()
        dt = (time.perf_counter() - t0) / a.rounds * 1e6
        if h is not None:
            assert h.error() == 0
        print(f"{name:30s} {dt:7.2f} us/round ({a.dtype}, {a.rows} rows)", flush=True)
        del e


if __name__ == "__main__":
    main()
