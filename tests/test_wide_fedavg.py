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


def _worker(rank, port, q, wires, rounds, step_size, gamma):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch
        from fedmi.fl.wide import WideClient
        from fedmi.parallel.comm import Comm
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        X, y = _data(rank, comm.device)
        res = {}
        for wire in wires:
            c = WideClient(X, y, DIMS, comm=comm, n_total=sum(ROWS), micro_batch=512, dtype="bf16", lr=0.004,
                           allreduce_dtype=wire, step_size=step_size, gamma=gamma)
            snaps = []
            for _ in range(rounds):
                c.run_round()
                c.loss()
                c.sync()
                torch.cuda.synchronize()
                snaps.append(c.params.cpu().numpy().copy())
            res[wire] = snaps
            comm.Barrier()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run_two(wires, rounds=ROUNDS, step_size=30, gamma=0.5):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, wires, rounds, step_size, gamma)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=150) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, _, err in out:
        assert err is None, f"rank {rank}:\n{err}"
    for w in wires:  # every rank holds the same global model after every round
        for a, b in zip(out[0][1][w], out[1][1][w]):
            np.testing.assert_array_equal(a, b)
    return out[0][1]


@pytest.mark.parametrize("wire,tol", [("fp32", 1e-6), ("bf16", 2e-3)])
def test_wide_fedavg_buckets_match_simulation(wire, tol):
    """fp32 buckets: the simulation to fp32 rounding (max element error); bf16 buckets (the
    scaled round delta rounded to bf16 on the wire, added to the fp32 previous global model):
    close to it in relative L2 -- single elements can differ by a whole Adam step, because
    Adam's normalisation turns a near-zero gradient whose sign flipped into a full lr step."""
    res = _run_two((wire,))
    out = [(0, [res[wire][-1]])]

    # single-process simulation of the same two clients
    import torch
    from fedmi.fl.wide import WideClient
    dev = torch.device("cuda", 0)
    cl = [WideClient(*_data(r, dev), DIMS, micro_batch=512, dtype="bf16", lr=0.004) for r in range(2)]
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
    if wire == "fp32":
        err = np.max(np.abs(out[0][1][0] - ref)) / np.max(np.abs(ref))
    else:
        err = np.linalg.norm(out[0][1][0] - ref) / np.linalg.norm(ref)
    assert err < tol, err


def test_wide_bf16_wire_keeps_fp32_master():
    """with bf16 buckets the master weights must stay fp32.  StepLR decays the LR
    20x per round (0.004 -> 2e-4 -> 1e-5 -> 5e-7): the late Adam steps are far below half a
    bf16 ulp of the weights (~1e-4 relative), so re-rounding the averaged weights to bf16 (round
    2's design) would erase them.  With the delta wire they survive: every round's global update
    matches the fp32 wire's within 5 % (the last one is ~100 fp32 ulps of the weights, so fp32
    rounding of the master copy itself is ~1 % of it)."""
    res = _run_two(("fp32", "bf16"), rounds=4, step_size=1, gamma=0.05)
    f, b = res["fp32"], res["bf16"]
    for r in range(1, 4):
        uf, ub = f[r] - f[r - 1], b[r] - b[r - 1]
        assert np.max(np.abs(uf)) > 0, r
        rel = np.linalg.norm(ub - uf) / np.linalg.norm(uf)
        assert rel < 0.05, (r, rel)
    assert np.linalg.norm(b[-1] - f[-1]) / np.linalg.norm(f[-1]) < 2e-3


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


def test_wide_fused_evaluation_matches_separate_pass():
    """One client: round r's evaluation scored from round r+1's training forward (fused_eval) gives
    the very confusion counts of a separate evaluation pass after round r, and the training itself
    is unchanged (bitwise); metrics() flushes the last round's pending evaluation."""
    import torch
    from fedmi.fl.wide import WideClient
    dev = torch.device("cuda", 0)
    X, y = _data(0, dev)
    sep = WideClient(X, y, DIMS, micro_batch=512, dtype="bf16", fused_eval=False)
    fus = WideClient(X, y, DIMS, micro_batch=512, dtype="bf16")
    assert fus.fused_eval and not sep.fused_eval
    cms = []
    for r in range(4):
        sep.run_round(evaluate=True)
        sep.stream.synchronize()
        cms.append(sep.cm.clone())
        fus.run_round(evaluate=True)
        fus.stream.synchronize()
        assert torch.equal(fus.params, sep.params), r
        if r > 0:  # round r's forward scored round r-1's post-step model
            assert torch.equal(fus.cm, cms[r - 1]), r
    assert fus.metrics() == sep.metrics()
    assert torch.equal(fus.cm, cms[-1])


@pytest.mark.parametrize("lr,tol", [(1e-4, 2e-3), (0.004, 3e-2)])
def test_wide_full_width_matches_torch(lr, tol):
    """BASELINE config 3 at FULL width (14-4096-4096-4096-2, 2048 device-generated rows): three
    full-batch rounds of the wide client (bf16 NT GEMMs, fp32 master / Adam) against an eager
    fp32 torch model from the same weights (nn.Linear / ReLU / cross_entropy / torch.optim.Adam,
    the reference's round C:63-73).  The per-round losses agree -- at the default wide lr 1e-4
    and at the reference's 0.004, where both diverge the same way (loss 0.69 -> ~70 -> ~200):
    the divergence is the optimizer's, not the kernels' (profiles/wide_learn_r3.log)."""
    import torch
    from fedmi.data.synthetic import device_shard
    from fedmi.fl.wide import WideClient
    from fedmi.models.mlp import flat_to_dict
    dev = torch.device("cuda", 0)
    dims = [14, 4096, 4096, 4096, 2]
    X, y = device_shard(2048, 0, dev, seed=7)
    c = WideClient(X, y, dims, micro_batch=2048, dtype="bf16", lr=lr, seed=0)
    d = flat_to_dict(c.params.cpu().numpy(), dims)
    layers = []
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        lin = torch.nn.Linear(a, b)
        with torch.no_grad():
            lin.weight.copy_(torch.as_tensor(d[f"model.{2 * i}.weight"]))
            lin.bias.copy_(torch.as_tensor(d[f"model.{2 * i}.bias"]))
        layers += [lin, torch.nn.ReLU()]
    ref = torch.nn.Sequential(*layers[:-1]).to(dev)
    opt = torch.optim.Adam(ref.parameters(), lr=lr)
    hl, tl = [], []
    for _ in range(3):
        c.run_round(evaluate=False)
        hl.append(c.loss())
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(ref(X), y.long())
        loss.backward()
        opt.step()
        tl.append(float(loss.item()))
    rel = [abs(h - t) / abs(t) for h, t in zip(hl, tl)]
    assert max(rel) < tol, (hl, tl)
    if lr < 1e-3:
        flat = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
        assert float((c.params - flat).norm() / flat.norm()) < 3e-3
