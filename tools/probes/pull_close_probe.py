"""Probe: the lagged pull-exchange engine's closing round at world 8 (ranks sharing cuda:0).
Runs the test_peer_allreduce world-8 engine in variants and reports, per rank, the rounds whose
per-rank metrics contain zeros (a tail read before its rank wrote it)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from test_peer_allreduce import _run_engine
    from fedmi.data.synthetic import make_income_like
    from fedmi.models.mlp import init_flat
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
    if os.environ.get("PROBE_RAW", "0") == "1":   # the test's raw communicator + second self-test first
        from fedmi.parallel.peer import make_peer_allreduce, selftest
        h = make_peer_allreduce(comm, 3001, comm.device, timeout_s=30.0, n_chunks=48)
        ok = h is not None and bool(all(comm.allgather(selftest(h, comm, comm.device, calls=4))))
        comm.Barrier()
        if h is not None:
            h.close()
        del h
    X, y = make_income_like(900 + 100 * rank, seed=30 + rank)
    hidden = (24, 12)
    flat = init_flat([14, *hidden, 2], 5)
    out = {}
    for name, env, kw in (("ll", {}, {}), ("pull", {"FEDMI_PEER_LL": "0"}, {}),
                          ("pull_no_evalfedavg", {"FEDMI_PEER_LL": "0"}, {"eval_fedavg": False}),
                          ("pull_again", {"FEDMI_PEER_LL": "0"}, {})):
        os.environ.update(env)
        try:
            w, h, c = _run_engine(comm, True, "bf16", X, y, flat, hidden=hidden, expect_ll=not env, **kw)
        finally:
            for k in env:
                del os.environ[k]
        pr = np.asarray(h["per_rank"])
        zero = [int(r) for r in np.flatnonzero((pr == 0).all(axis=2).any(axis=1))]
        out[name] = {"zero_rounds": zero, "acc_last": [round(float(v), 4) for v in pr[-1, :, 0]]}
    q.put((rank, out))
    comm.close()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in ps:
        p.join(timeout=30)
    for rank, out in res:
        print(rank, {k: v["zero_rounds"] for k, v in out.items()}, "pull last acc", out["pull"]["acc_last"])
