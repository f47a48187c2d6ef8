"""End-of-run replica check (fedmi/parallel/consistency.py) over gloo, world 2 and 3: equal global
models pass on every rank; a single flipped bit on one rank makes EVERY rank raise (they all see
the same digest list), so a benchmark or entrypoint run with a faulty data plane ends with an
error instead of a number.  Also the trainer's own check after a real multi-client run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        torch.set_num_threads(1)
        from fedmi.data.tabular import load_tabular
        from fedmi.fl.engine import EngineConfig
        from fedmi.fl.trainer import FederatedMLPLearning
        from fedmi.parallel.comm import Comm
        from fedmi.parallel.consistency import check_replicas
        comm = Comm(backend="gloo", device="cpu")
        out = {}
        w = np.linspace(-1, 1, 1001, dtype=np.float32)
        out["equal"] = check_replicas(comm, [w, torch.arange(7, dtype=torch.bfloat16)])
        bad = w.copy()
        if rank == world - 1:
            bad.view(np.uint32)[500] ^= 1        # one ulp on one element of one rank
        try:
            check_replicas(comm, [bad])
            out["raised"] = False
        except RuntimeError as e:
            out["raised"] = "replica check failed" in str(e)
        out["nonstrict"] = check_replicas(comm, [bad], strict=False)
        ds = load_tabular()
        tr = FederatedMLPLearning(ds.X_train, ds.y_train, comm.rank, comm.size, comm=comm,
                                  config=EngineConfig(max_rounds=4), backend="torch")
        tr.train_and_evaluate(comm, rounds=4, verbose=False)
        out["trainer"] = tr.replicas_consistent
        q.put((rank, out, None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_replica_check_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for rank, out, err in res:
        assert err is None, f"rank {rank}:\n{err}"
        assert out["equal"] is True
        assert out["raised"] is True, rank          # every rank, not only the one that differs
        assert out["nonstrict"] is False
        assert out["trainer"] is True


def test_digest_is_dtype_and_shape_aware():
    import torch
    from fedmi.parallel.consistency import digest
    a = np.zeros(8, dtype=np.float32)
    assert digest([a]) != digest([a.reshape(2, 4)])
    assert digest([a]) != digest([a.astype(np.float64)])
    assert digest([torch.zeros(8)]) == digest([a])
    assert digest([torch.ones(3, dtype=torch.bfloat16)]) == digest([torch.ones(3, dtype=torch.bfloat16)])
