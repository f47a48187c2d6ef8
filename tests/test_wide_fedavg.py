"""Wide-MLP federated rounds (BASELINE config 3 path, fedmi/fl/wide.py) with two clients sharing
one GPU: the per-layer FedAvg buckets run on the comm stream and the next round's forward of
layer l waits only on bucket l's event.  The result must equal a single-process simulation
that averages the two clients' weights (n_i / N weighted) after every local step."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

DIMS = [14, 256, 128, 2]
ROWS = (1536, 1024)
ROUNDS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank, dev):
    import torch
    from fedmi.data.synthetic import make_income_like
    X, y = make_income_like(ROWS[rank], seed=40 + rank)
    return torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)


def _worker(rank, port, q, wire):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch
        from fedmi.fl.wide import WideClient
        from fedmi.parallel.comm import Comm
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        X, y = _data(rank, comm.device)
        c = WideClient(X, y, DIMS, comm=comm, n_total=sum(ROWS), micro_batch=512, dtype="bf16", allreduce_dtype=wire)
        losses = []
        for _ in range(ROUNDS):
            c.run_round()
            losses.append(c.loss())
        c.sync()
        torch.cuda.synchronize()
        q.put((rank, c.params.cpu().numpy(), losses, None))
        comm.Barrier()
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("wire,tol", [("fp32", 1e-6), ("bf16", 5e-2)])
def test_wide_fedavg_buckets_match_simulation(wire, tol):
    """fp32 buckets: the simulation to fp32 rounding; bf16 buckets (scaled weights rounded to
    bf16 on the wire, fp32 master copy): close to it -- a rounding that flips the sign of a
    small gradient moves that weight by a whole Adam step (lr 0.004) in the next round."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, wire)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=110) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, _, _, err in out:
        assert err is None, f"rank {rank}:\n{err}"
    np.testing.assert_array_equal(out[0][1], out[1][1])

    # single-process simulation of the same two clients
    import torch
    from fedmi.fl.wide import WideClient
    dev = torch.device("cuda", 0)
    cl = [WideClient(*_data(r, dev), DIMS, micro_batch=512, dtype="bf16") for r in range(2)]
    n = sum(ROWS)
    for _ in range(ROUNDS):
        for c in cl:
            c.local_step()
            c.stream.synchronize()
        avg = cl[0].params * (ROWS[0] / n) + cl[1].params * (ROWS[1] / n)
        for c in cl:
            c.params.copy_(avg)
            c._quantize()
            c.stream.synchronize()
            c.round += 1
    ref = cl[0].params.cpu().numpy()
    err = np.max(np.abs(out[0][1] - ref)) / np.max(np.abs(ref))
    assert err < tol, err


def test_wide_local_evaluation_whole_shard():
    """evaluate_shard: micro-batched forward + device argmax / confusion over EVERY row of the
    shard (the reference's per-round local evaluation, C:148); vs an fp32 torch forward."""
    import torch
    from fedmi.fl.wide import WideClient
    from fedmi.models.mlp import flat_to_dict
    dev = torch.device("cuda", 0)
    X, y = _data(0, dev)
    c = WideClient(X, y, DIMS, micro_batch=512, dtype="bf16")
    c.run_round(evaluate=True)
    m = c.metrics()
    cm = c.cm.cpu().numpy()
    assert cm.sum() == ROWS[0]
    # the evaluated model is the post-step local model (before aggregate: one client -> same)
    d = flat_to_dict(c.params.cpu().numpy(), DIMS)
    a = X.float()
    for l in range(len(DIMS) - 1):
        a = a @ torch.as_tensor(d[f"model.{2 * l}.weight"], device=dev).T + torch.as_tensor(d[f"model.{2 * l}.bias"], device=dev)
        if l < len(DIMS) - 2:
            a = torch.relu(a)
    acc = float((a.argmax(1) == y.long()).float().mean())
    assert abs(m["accuracy"] - acc) < 0.01, (m["accuracy"], acc)
