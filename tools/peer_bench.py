"""Round time of the multi-client data planes with two ranks sharing one GPU (the 1-GPU box
cannot run real xGMI): host (gloo) aggregation, separate eval + one-shot peer all-reduce
kernels, and the fused evaluation + FedAvg kernel.  Both ranks' kernels compete for the same
CUs, so absolute numbers overstate a real 2-GPU round; the comparison between data planes
is what this measures.

    python tools/peer_bench.py [--rounds 400] [--dtype bf16]
"""
import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, a, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from fedmi.data.synthetic import make_income_like
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
    X, y = make_income_like(a.rows, seed=rank)
    flat = init_flat([14, 50, 200, 2], 0)
    out = {}
    for name, peer, ef in (("peer fused eval+fedavg", True, True), ("peer separate kernels", True, False)):
        comm.peer_allreduce = peer
        cfg = EngineConfig(max_rounds=a.rounds + 64, early_stop=False, dtype=a.dtype, graph_rounds=16,
                           eval_fedavg=ef)
        e = HipRoundEngine(X, y, 2, cfg, comm, flat)
        e.run(32)
        e.stream.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        e._issue(a.rounds)
        e.stream.synchronize()
        dist.barrier()
        out[name] = (time.perf_counter() - t0) / a.rounds * 1e6
    q.put((rank, out))
    comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=400)
    ap.add_argument("--rows", type=int, default=8000)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, a, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for name in res[0][1]:
        print(f"{name:28s} {max(r[1][name] for r in res):8.1f} us/round (2 ranks on one GPU, {a.dtype})")


if __name__ == "__main__":
    main()
