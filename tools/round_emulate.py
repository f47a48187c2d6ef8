"""Emulate the multi-client round on ONE GPU (the 1-GPU box cannot run real xGMI): a one-rank
peer all-reduce (or a one-rank RCCL communicator) gives every kernel of a world > 1 round its
real shape -- classic evaluation of the post-step model, the all-reduce kernel with its bf16
pack epilogue -- minus the xGMI latency of the pulls.  Prints us/round for

  * world 1, fused evaluation (what bench.py runs at N = 1);
  * classic evaluation + separate one-shot all-reduce kernel;
  * the fused evaluation + FedAvg kernel (N > 1 with early stopping, several local steps);
  * lagged evaluation: round r scored inside round r+1's train kernel, no evaluation kernel,
    with a separate all-reduce kernel or with the FedAvg inside the Adam kernel, early
    stopping off / on (bench.py's N > 1 round);
  * the RCCL data plane (the xGMI set-up's fallback): classic rounds, and lagged rounds with
    early stopping (region A folded one round late, FLState::late).

for every shard size of --rows (the reference's 8000 // k rows per client: 8000 / 4000 / 2000 /
1000) and every rows-per-workgroup choice of --rpb.

    python tools/round_emulate.py [--rounds 2000] [--dtype bf16] [--rows 8000 4000 2000 1000] [--rpb 16 32]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {
    # name: (fused, eval_fedavg (None: no peer), lagged, adam exchange, early stop, rccl)
    "world1-fused": ("world 1, fused evaluation", True, None, False, 0, False, False),
    "eval+ar": ("eval + one-shot all-reduce", False, False, False, 0, False, False),
    "evalfedavg": ("fused eval + FedAvg kernel", False, True, False, 0, False, False),
    "lag+ar": ("lagged eval + all-reduce kernel", False, True, True, 0, False, False),
    "lag+adamx": ("lagged eval + FedAvg in Adam", False, True, True, 1, False, False),
    "lag+adamx+es": ("same + early stopping (in time)", False, True, True, 1, True, False),
    "rccl-classic+es": ("RCCL classic + early stopping", False, None, False, 0, True, True),
    "rccl-lag": ("RCCL lagged", False, None, True, 0, False, True),
    "rccl-lag+es": ("RCCL lagged + ES (late fold)", False, None, True, 0, True, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2000)
    ap.add_argument("--rows", type=int, nargs="+", default=[8000])
    ap.add_argument("--rpb", type=int, nargs="+", default=[0], help="rows per workgroup (0: engine default)")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--cases", nargs="+", default=list(CASES), choices=list(CASES))
    a = ap.parse_args()
    import torch
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    from fedmi.ops import native
    import bench
    m = native()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rc = None
    if any(CASES[k][6] for k in a.cases):
        rc = m.RcclComm(1, 0, m.RcclComm.unique_id(), 0)
    flat = init_flat([14, 50, 200, 2], 0)
    for rows in a.rows:
        X, y = bench.synth_shard(rows, 0, dev)
        for rpb in a.rpb:
            for key in a.cases:
                name, fused, ef, lag, adam_x, es, use_rccl = CASES[key]
                if lag and a.dtype != "bf16":
                    continue
                # early stopping on with a patience never reached: every round's fold runs the rule
                cfg = EngineConfig(max_rounds=a.rounds + 256, early_stop=es, patience=10 ** 6,
                                   dtype=a.dtype, graph_rounds=16, rows_per_block=rpb,
                                   fused_eval=fused, eval_fedavg=bool(ef), lagged_eval=lag)
                e = HipRoundEngine(X, y, 2, cfg, None, flat, emulate_clients=not fused)
                h = None
                if ef is not None:
                    h = m.PeerAllReduce(1, 0, 0, int(e.params[0].numel()), 10.0, (e.P + 63) // 64 + 2 if adam_x else 0)
                    h.open([h.handle()])
                    h.clear()
                    e.engine.attach_peer(h)
                if use_rccl:
                    e._native_comm = rc
                design = ("late-fold" if e.engine.late_fold else "adam-x" if e.engine.adam_exchange else
                          "lagged" if e.engine.lagged else "fused" if e.engine.fused else "classic")
                e.run(64)
                e.stream.synchronize()
                t0 = time.perf_counter()
                e._issue(a.rounds)
                e.stream.synchronize()
                dt = (time.perf_counter() - t0) / a.rounds * 1e6
                if h is not None:
                    assert h.error() == 0
                print(f"{name:34s} {dt:7.2f} us/round ({a.dtype}, {rows} rows, R={e.R}, {design})", flush=True)
                del e
    if rc is not None:
        torch.cuda.synchronize()
        rc.destroy()


if __name__ == "__main__":
    main()
