"""HIP kernels of the fused round engine and the layered path vs torch fp32 references."""
import numpy as np
import pytest
import torch

from fedmi.data.synthetic import make_income_like
from fedmi.fl.early_stop import EarlyStopper
from fedmi.fl.engine import EngineConfig, HipRoundEngine, TorchRoundEngine
from fedmi.models.mlp import init_flat
from fedmi.ops import native

pytestmark = pytest.mark.gpu

DIMS = [14, 50, 200, 2]


@pytest.fixture(scope="module")
def shard():
    return make_income_like(3000, seed=5)


def test_native_extension_loaded():
    from fedmi.ops import native
    m = native(build_if_missing=False)
    assert m.__file__.endswith(".so") and "fedmi/ops" in m.__file__
    info = m.device_info(0)
    assert "gfx950" in info["arch"]


@pytest.mark.parametrize("R", [16, 32])
@pytest.mark.parametrize("hidden", [(50, 200), (7,), (33, 17, 9)])
def test_round_matches_torch(shard, R, hidden):
    X, y = shard
    dims = [14, *hidden, 2]
    flat = init_flat(dims, 1)
    cfg = EngineConfig(hidden=hidden, max_rounds=20, rows_per_block=R, graph_rounds=0, early_stop=False)
    hip = HipRoundEngine(X, y, 2, cfg, None, flat)
    ref = TorchRoundEngine(X, y, 2, cfg, None, flat)
    hip.run(3)
    ref.run(3)
    a, b = hip.global_flat(), ref.global_flat()
    assert np.abs(a - b).max() / np.abs(b).max() < 2e-5
    np.testing.assert_allclose(hip.history()["global"], ref.history()["global"], atol=2e-3)
    np.testing.assert_allclose(hip.history()["loss"], ref.history()["loss"], rtol=1e-4)


def test_graph_replay_bitwise_equals_eager(shard):
    X, y = shard
    flat = init_flat(DIMS, 2)
    out = []
    for g in (0, 8):
        cfg = EngineConfig(max_rounds=40, graph_rounds=g, early_stop=False)
        e = HipRoundEngine(X, y, 2, cfg, None, flat)
        e.run(33)
        out.append((e.global_flat(), e.history()["global"]))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_device_early_stop_rule_matches_host_rule(dtype):
    """The device-side stop rule replays the host rule on the device's own metric history, and
    (real CSV, reference hyperparameters) fires inside 300 rounds in both precisions -- bf16
    scores with the split-bf16 forward, so borderline rows stop flipping as the LR decays."""
    from fedmi.data.tabular import load_tabular
    ds = load_tabular()
    e = HipRoundEngine(ds.X_train, ds.y_train, 2, EngineConfig(max_rounds=300, dtype=dtype), None,
                       init_flat(DIMS, 0))
    e.run(300)
    h = e.history()
    assert 100 < h["rounds_run"] < 300 and h["stop_round"] == h["rounds_run"]
    es = EarlyStopper(10, 1e-4)
    stop = None
    for r, v in enumerate(h["global"]):
        if es.update(v):
            stop = r + 1
            break
    assert stop == h["stop_round"]
    assert h["global"][-1][0] > 0.82


def test_step_api_equals_fused(shard):
    X, y = shard
    flat = init_flat(DIMS, 3)
    cfg = EngineConfig(max_rounds=10, graph_rounds=0, early_stop=False)
    a = HipRoundEngine(X, y, 2, cfg, None, flat)
    b = HipRoundEngine(X, y, 2, cfg, None, flat)
    a.run(4)
    for _ in range(4):
        b.step_train()
        cm = b.step_eval()
        assert cm.sum() == len(X)
        b.step_aggregate()
    b.sync_history()
    np.testing.assert_array_equal(a.global_flat(), b.global_flat())


def test_confusion_eval_matches_torch(shard):
    X, y = shard
    flat = init_flat(DIMS, 4)
    hip = HipRoundEngine(X, y, 2, EngineConfig(max_rounds=4), None, flat)
    ref = TorchRoundEngine(X, y, 2, EngineConfig(max_rounds=4), None, flat)
    Xt, yt = make_income_like(777, seed=9)
    np.testing.assert_array_equal(hip.confusion(Xt, yt, flat=flat), ref.confusion(Xt, yt, flat=flat))


def test_local_steps_and_fedprox_match_torch(shard):
    X, y = shard
    dims = [14, 16, 2]
    flat = init_flat(dims, 5)
    cfg = EngineConfig(hidden=(16,), local_steps=3, prox_mu=0.3, max_rounds=5, early_stop=False, graph_rounds=0)
    hip = HipRoundEngine(X, y, 2, cfg, None, flat)
    ref = TorchRoundEngine(X, y, 2, cfg, None, flat)
    hip.run(3)
    ref.run(3)
    a, b = hip.global_flat(), ref.global_flat()
    assert np.abs(a - b).max() / np.abs(b).max() < 2e-5


def test_synthetic_device_generator():
    from fedmi.ops import native
    from fedmi.data.synthetic import teacher_weights
    m = native()
    dev = torch.device("cuda", 0)
    n = 200_000
    X = torch.empty(n, 14, device=dev)
    yv = torch.empty(n, dtype=torch.int32, device=dev)
    w1, w2 = teacher_weights()
    Xs, _ = make_income_like(4096, seed=123)
    th = float(np.median(np.maximum(Xs @ w1.T, 0.0) @ w2))
    tw1 = torch.as_tensor(w1, device=dev)
    tw2 = torch.as_tensor(np.append(w2, th).astype(np.float32), device=dev)
    m.synth(X.data_ptr(), yv.data_ptr(), n, 14, 7, 0, tw1.data_ptr(), tw2.data_ptr(), w1.shape[0],
            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    Xc = X.cpu().numpy()
    assert np.isfinite(Xc).all()
    assert abs(Xc[:, :6].mean()) < 0.02 and abs(Xc[:, :6].std() - 1) < 0.02
    assert 0.35 < yv.float().mean().item() < 0.65
    # label noise: the same rows, each label flipped with probability 0.15 (own Philox stream)
    Xn = torch.empty_like(X)
    yn = torch.empty_like(yv)
    m.synth(Xn.data_ptr(), yn.data_ptr(), n, 14, 7, 0, tw1.data_ptr(), tw2.data_ptr(), w1.shape[0],
            torch.cuda.current_stream().cuda_stream, 0.15)
    torch.cuda.synchronize()
    assert torch.equal(Xn, X)
    flip = (yn != yv).float().mean().item()
    assert 0.145 < flip < 0.155, flip


@pytest.mark.parametrize("dtype", [0, 1])
def test_layered_gemm_variants(dtype):
    from fedmi.ops import native
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    M, N, K = 130, 70, 300
    for epi in (0, 1, 2, 3):
        for akc, bkc in ((1, 1), (1, 0), (0, 0), (0, 1)):
            if epi == 3 and not akc:
                continue
            Af = torch.randn(M, K, device=dev) if akc else torch.randn(K, M, device=dev)
            Bf = torch.randn(N, K, device=dev) if bkc else torch.randn(K, N, device=dev)
            At, Bt = (Af if akc else Af.t()), (Bf.t() if bkc else Bf)
            bias, mask = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
            C = torch.zeros(M, N, device=dev)
            cast = (lambda t: t) if dtype == 0 else (lambda t: t.to(torch.bfloat16))
            Ain, Bin = cast(Af), cast(Bf)
            m.gemm(M, N, K, Ain.data_ptr(), Af.shape[1], akc, Bin.data_ptr(), Bf.shape[1], bkc, C.data_ptr(), N,
                   epi, bias.data_ptr(), mask.data_ptr(), N, 0, 1.0, 0.0, dtype, 1, 0, 0, s)
            ref = (cast(At).float().double() @ cast(Bt).float().double()).float()
            if epi in (1, 2):
                ref = ref + bias
            if epi == 2:
                ref = ref.clamp_min(0)
            if epi == 3:
                ref = ref * (mask > 0)
            torch.cuda.synchronize()
            tol = 5e-6 if dtype == 0 else 1e-2
            assert ((C - ref).abs().max() / ref.abs().max()).item() < tol


@pytest.mark.parametrize("rows,mb", [(1500, 512), (4500, 4096)])
def test_wide_client_fp32_matches_torch(rows, mb):
    """Five fp32 rounds vs torch; mb = 4096 runs the skinny weight gradients split-K (4 slabs)."""
    from fedmi.fl.wide import WideClient
    dev = torch.device("cuda", 0)
    X, y = make_income_like(rows, seed=0)
    Xt, yt = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
    c = WideClient(Xt, yt, [14, 64, 48, 2], micro_batch=mb, dtype="fp32", lr=0.004)
    ref = torch.nn.Sequential(torch.nn.Linear(14, 64), torch.nn.ReLU(), torch.nn.Linear(64, 48), torch.nn.ReLU(),
                              torch.nn.Linear(48, 2)).to(dev)
    with torch.no_grad():
        for p, w in zip(ref.parameters(), [c.W[0], c.b[0], c.W[1], c.b[1], c.W[2], c.b[2]]):
            p.copy_(w)
    opt = torch.optim.Adam(ref.parameters(), lr=0.004)
    for _ in range(3):
        c.run_round()
        opt.zero_grad()
        torch.nn.functional.cross_entropy(ref(Xt), yt.long()).backward()
        opt.step()
    torch.cuda.synchronize()
    flat_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    assert ((c.params - flat_ref).abs().max() / flat_ref.abs().max()).item() < 1e-4


def test_gemm_nt_bf16_epilogues():
    """bf16 NT GEMM vs an fp32 torch reference of the same (bf16-rounded) operands."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    M, N, K = 256, 384, 320
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    ref = A.float() @ B.float().t()
    # bias + ReLU -> bf16 row-major + bf16 transposed
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    CbT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
    m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, CbT.data_ptr(), M,
              bias.data_ptr(), 0, 0, 1, 1.0, 0.0, s)
    r1 = (ref + bias).clamp_min(0)
    torch.cuda.synchronize()
    assert ((Cb.float() - r1).abs().max() / r1.abs().max()).item() < 1e-2
    assert torch.equal(CbT, Cb.t())
    # fp32 accumulate (beta = 1) with mask
    mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
    C0 = torch.randn(M, N, device=dev)
    C = C0.clone()
    m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), N, 0, 0, 0, 0, 0,
              mask.data_ptr(), N, 0, 0.5, 1.0, s)
    r2 = torch.where(mask.float() > 0, 0.5 * ref, torch.zeros_like(ref)) + C0
    torch.cuda.synchronize()
    assert ((C - r2).abs().max() / r2.abs().max()).item() < 1e-5


@pytest.mark.parametrize("M,N,splits", [(1000, 2, 7), (131072, 2, 256), (300, 14, 300)])
def test_colsum_split(M, N, splits):
    """Split few-column sums (wide head bias gradient) vs torch fp32, beta = 1."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(M)
    X = torch.randn(M, N, device=dev)
    out0 = torch.randn(N, device=dev)
    out = out0.clone()
    slab = torch.empty(splits * N, device=dev)
    m.colsum_split(X.data_ptr(), M, N, splits, slab.data_ptr(), out.data_ptr(), 1.0, s)
    torch.cuda.synchronize()
    exp = out0 + X.double().sum(0).float()
    assert torch.allclose(out, exp, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("C,trans,rows,splits", [(2, 0, 1000, 3), (14, 1, 4096, 16), (2, 0, 256, 1)])
def test_skinny_wgrad_bf16(C, trans, rows, splits):
    """Skinny weight gradient (wide MLP layer 0 / logits head) vs an fp32 torch reference of the
    same bf16 operands, accumulating into a non-zero output (beta = 1)."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(C + rows)
    Nw, lds = 2048 + 512, 64
    W = torch.randn(rows, Nw, device=dev).to(torch.bfloat16)
    S = torch.randn(rows, lds, device=dev).to(torch.bfloat16)
    ref = S[:, :C].float().t() @ W.float()          # [C][Nw]
    if trans:
        ref = ref.t().contiguous()                   # [Nw][C]
    out0 = torch.randn_like(ref)
    out = out0.clone()
    slab = torch.empty(splits * (C + 1) * Nw, device=dev)
    b0 = torch.randn(Nw, device=dev)
    bias = b0.clone()
    m.skinny_wgrad(W.data_ptr(), Nw, Nw, S.data_ptr(), lds, C, rows, trans, splits, slab.data_ptr(), out.data_ptr(),
                   1.0, bias.data_ptr() if trans else 0, s)
    torch.cuda.synchronize()
    exp = out0 + ref
    assert ((out - exp).abs().max() / exp.abs().max()).item() < 1e-5
    if trans:  # layer 0: bias gradient = column sums of the wide operand, from the same loads
        bexp = b0 + W.float().sum(0)
        assert ((bias - bexp).abs().max() / bexp.abs().max()).item() < 1e-5


@pytest.mark.parametrize("M,N,K,pad", [(256, 512, 64, 0), (256, 256, 128, 0), (512, 768, 192, 64), (768, 512, 1024, 0),
                                       (2048, 1024, 4096, 8)])
def test_gemm_nt_bf16_pingpong_matches_128_tile(M, N, K, pad):
    """The 256x256 ping-pong main loops (variant 2: half-line DMA pieces, variant 3: whole-line
    pieces and 128-byte LDS rows, with buffer-resource DMAs; variant 10: the same with
    global_load_lds DMAs) against the 128x128 loop (variant 1): same per-element k order, so
    bit-identical, and against an fp32 torch reference; row strides wider than K exercise the
    DMA source addressing."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(K)
    A = torch.randn(M, K + pad, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K + pad, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    outs = []
    try:
        for v in (1, 2, 3, 10):
            m.gemm_nt_set_variant(v)
            Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            CbT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
            C = torch.empty(M, N, device=dev)
            m.gemm_nt(M, N, K, A.data_ptr(), K + pad, B.data_ptr(), K + pad, C.data_ptr(), N, Cb.data_ptr(), N,
                      CbT.data_ptr(), M, bias.data_ptr(), 0, 0, 1, 1.0, 0.0, s)
            torch.cuda.synchronize()
            outs.append((C, Cb))
            assert torch.equal(CbT, Cb.t())
    finally:
        m.gemm_nt_set_variant(3)
    # ReLU-mask epilogue (dgrad: the mask tile is staged through LDS by the ping-pong loop)
    mask = torch.randn(M, N + 8, device=dev).to(torch.bfloat16)
    mouts = []
    try:
        for v in (1, 2, 3, 10):
            m.gemm_nt_set_variant(v)
            Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            m.gemm_nt(M, N, K, A.data_ptr(), K + pad, B.data_ptr(), K + pad, 0, 0, Cb.data_ptr(), N, 0, 0, 0,
                      mask.data_ptr(), N + 8, 0, 1.0, 0.0, s)
            torch.cuda.synchronize()
            mouts.append(Cb)
    finally:
        m.gemm_nt_set_variant(3)
    assert all(torch.equal(mouts[0], o) for o in mouts[1:])
    mref = torch.where(mask[:, :N].float() > 0, A[:, :K].float() @ B[:, :K].float().t(), torch.zeros(M, N, device=dev))
    assert ((mouts[1].float() - mref).abs().max() / mref.abs().max()).item() < 1e-2
    ref = (A[:, :K].float() @ B[:, :K].float().t() + bias).clamp_min(0)
    for v in range(1, len(outs)):
        assert torch.equal(outs[0][0], outs[v][0])
        assert torch.equal(outs[0][1], outs[v][1])
    assert ((outs[1][0] - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("cfg", ["Cb", "Cb+CbT+bias+relu", "Cb+bias+relu", "Cb+CbT+mask", "Cb+mask", "C", "C+beta",
                                 "C+bias"])
def test_gemm_nt_bf16_epilogue_configs(cfg):
    """Every output configuration the full-line loop compiles separately (wide forward, dgrad,
    wgrad, logits, plain) is bit-identical to the 128x128 loop's runtime-configured epilogue."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    M, N, K = 512, 768, 320
    torch.manual_seed(7)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
    C0 = torch.randn(M, N, device=dev)
    outs = []
    try:
        for v in (1, 3, 10):
            m.gemm_nt_set_variant(v)
            C = C0.clone()
            Cb = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            CbT = torch.zeros(N, M, dtype=torch.bfloat16, device=dev)
            has = lambda k: k in cfg.split("+")
            m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr() if has("C") else 0, N,
                      Cb.data_ptr() if has("Cb") else 0, N, CbT.data_ptr() if has("CbT") else 0, M,
                      bias.data_ptr() if has("bias") else 0, mask.data_ptr() if has("mask") else 0, N,
                      1 if has("relu") else 0, 1.0, 0.5 if has("beta") else 0.0, s)
            torch.cuda.synchronize()
            outs.append((C, Cb, CbT))
    finally:
        m.gemm_nt_set_variant(3)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_gemm_nt_bf16_dgrad_column_sums():
    """NT_EPI_CSUM: the dgrad epilogue's per-128-row column sums of its bf16 output (bias
    gradient) fold to torch's column sums of the same output; the other outputs are unchanged,
    and the 128x128 loop refuses the option."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    M, N, K = 1024, 512, 320
    torch.manual_seed(9)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
    outs = []
    for csum in (False, True):
        Cb = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        CbT = torch.zeros(N, M, dtype=torch.bfloat16, device=dev)
        cs = torch.full((M // 128, N), float("nan"), device=dev)
        m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, CbT.data_ptr(), M, 0,
                  mask.data_ptr(), N, 0, 1.0, 0.0, s, cs.data_ptr() if csum else 0, N)
        torch.cuda.synchronize()
        outs.append((Cb, CbT, cs))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    cs = outs[1][2]
    ref = outs[1][0].float().view(M // 128, 128, N).sum(1)
    assert torch.isfinite(cs).all()
    assert ((cs - ref).abs().max() / ref.abs().max()).item() < 1e-5
    gb = torch.zeros(N, device=dev)
    m.colsum(cs.data_ptr(), M // 128, N, N, gb.data_ptr(), 0.0, s)
    torch.cuda.synchronize()
    assert ((gb - ref.sum(0)).abs().max() / ref.sum(0).abs().max()).item() < 1e-5
    try:
        # the global_load_lds form of the full-line loop (variant 10): the same sums, bit for bit
        m.gemm_nt_set_variant(10)
        Cb9 = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        cs9 = torch.full((M // 128, N), float("nan"), device=dev)
        m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb9.data_ptr(), N, 0, 0, 0,
                  mask.data_ptr(), N, 0, 1.0, 0.0, s, cs9.data_ptr(), N)
        torch.cuda.synchronize()
        assert torch.equal(Cb9, outs[1][0]) and torch.equal(cs9, cs)
        m.gemm_nt_set_variant(1)
        with pytest.raises(RuntimeError):
            m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, outs[0][0].data_ptr(), N, 0, 0, 0,
                      mask.data_ptr(), N, 0, 1.0, 0.0, s, cs.data_ptr(), N)
    finally:
        m.gemm_nt_set_variant(3)


@pytest.mark.parametrize("M,N,beta", [(16384, 2, 0.0), (5000, 14, 1.0), (300, 50, 0.5), (700, 100, 1.0)])
def test_colsum_vs_torch(M, N, beta):
    """Bias-gradient column sums (flat few-column kernel for N <= 64, wave-per-64-columns otherwise)."""
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    X = torch.randn(M, N, device=dev)
    out = torch.randn(N, device=dev)
    ref = X.double().sum(dim=0) + beta * out.double()
    m.colsum(X.data_ptr(), M, N, N, out.data_ptr(), beta, s)
    torch.cuda.synchronize()
    assert (out.double() - ref).abs().max().item() < 1e-3


def test_rowsum_and_transpose_bf16():
    m = native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    X = torch.randn(200, 136, device=dev)
    XT = torch.empty(136, 200, dtype=torch.bfloat16, device=dev)
    m.transpose_bf16(X.data_ptr(), 200, 136, 136, XT.data_ptr(), 200, s)
    out = torch.full((136,), 2.0, device=dev)
    m.rowsum_bf16(XT.data_ptr(), 136, 200, 200, out.data_ptr(), 1.0, s)
    torch.cuda.synchronize()
    assert torch.equal(XT, X.t().to(torch.bfloat16))
    ref = XT.float().sum(dim=1) + 2.0
    assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("rows", [1536, 1736])
def test_wide_client_bf16_nt_path_gradients(rows):
    """One full-batch local step on the bf16 NT path: gradients vs torch fp32 autograd.  1736
    rows: the last micro-batch (200 rows) runs padded to 256 rows on the NT GEMM too."""
    from fedmi.fl.wide import WideClient
    dev = torch.device("cuda", 0)
    X, y = make_income_like(rows, seed=1)
    Xt, yt = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
    c = WideClient(Xt, yt, [14, 256, 256, 2], micro_batch=512, dtype="bf16")
    ref = torch.nn.Sequential(torch.nn.Linear(14, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                              torch.nn.Linear(256, 2)).to(dev)
    with torch.no_grad():
        for p, w in zip(ref.parameters(), [c.W[0], c.b[0], c.W[1], c.b[1], c.W[2], c.b[2]]):
            p.copy_(w)
    c.local_step()
    torch.nn.functional.cross_entropy(ref(Xt), yt.long()).backward()
    torch.cuda.synchronize()
    # every micro-batch on the NT GEMM: 3 forward (padded layer 0, hidden, padded head) + 3
    # backward (padded head dgrad, hidden wgrad + dgrad); layer 0's gradient is the skinny kernel
    assert c.nt_calls == 6 * ((rows + 511) // 512), c.nt_calls
    for g, p in zip([c.gW[0], c.gb[0], c.gW[1], c.gb[1], c.gW[2], c.gb[2]], ref.parameters()):
        rel = ((g - p.grad).norm() / p.grad.norm()).item()
        assert rel < 2e-2, rel


def test_hip_resume_is_exact_and_portable(tmp_path):
    from fedmi.ckpt.checkpoint import resume, save_checkpoint
    X, y = make_income_like(2000, seed=7)
    dims = [14, 50, 200, 2]

    def mk(backend_cls, **kw):
        cfg = EngineConfig(max_rounds=80, patience=4, tolerance=1e-3, graph_rounds=4)
        return backend_cls(X, y, 2, cfg, None, init_flat(dims, 9), **kw)

    full = mk(HipRoundEngine)
    full.run(50)
    a = mk(HipRoundEngine)
    a.run(17)
    save_checkpoint(str(tmp_path), a)
    b = mk(HipRoundEngine)
    assert resume(str(tmp_path), b) == 17
    b.run(33)
    hf, hb = full.history(), b.history()
    assert hf["rounds_run"] == hb["rounds_run"] and hf["stop_round"] == hb["stop_round"]
    np.testing.assert_array_equal(hf["global"], hb["global"])
    np.testing.assert_array_equal(full.global_flat(), b.global_flat())
    # HIP checkpoint -> torch engine: continues on the same trajectory (fp32 rounding only)
    t = mk(TorchRoundEngine)
    resume(str(tmp_path), t)
    t.run(5)
    c = mk(HipRoundEngine)
    resume(str(tmp_path), c)
    c.run(5)
    np.testing.assert_allclose(t.global_flat(), c.global_flat(), rtol=1e-4, atol=1e-5)


def test_hip_debug_mode_and_profile():
    X, y = make_income_like(1000, seed=2)
    cfg = EngineConfig(max_rounds=20, debug=True, early_stop=False)
    e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 1))
    e.run(3)
    cfg2 = EngineConfig(max_rounds=20, early_stop=False)
    f = HipRoundEngine(X, y, 2, cfg2, None, init_flat([14, 50, 200, 2], 1))
    f.run(3)
    np.testing.assert_array_equal(e.global_flat(), f.global_flat())
    t = f.profile(4)
    assert f.history()["rounds_run"] == 7
    assert t["train_us"] > 0 and t["eval_us"] > 0 and t["round_us"] >= t["train_us"]
    # trace: the real (fused) round design with an event per launch; the rounds it issues are
    # ordinary rounds (same trajectory as eager/graph rounds)
    for dtype in ("fp32", "bf16"):
        cfg3 = EngineConfig(max_rounds=20, early_stop=False, dtype=dtype)
        a = HipRoundEngine(X, y, 2, cfg3, None, init_flat([14, 50, 200, 2], 1))
        b = HipRoundEngine(X, y, 2, cfg3, None, init_flat([14, 50, 200, 2], 1))
        a.run(2)
        tr = a.trace(6, close=True)
        a.sync_history()
        b.run(8)
        assert a.history()["rounds_run"] == 8
        np.testing.assert_array_equal(a.global_flat(), b.global_flat())
        np.testing.assert_array_equal(np.asarray(a.history()["global"]), np.asarray(b.history()["global"]))
        assert tr["rounds"] == 6 and tr["launches"]["train"] == 6 and tr["launches"]["adam"] == 6
        assert tr["train"] > 0 and tr["adam"] > 0
        assert abs(sum(v for k, v in tr.items() if k not in ("round", "launches", "rounds")) - tr["round"]) \
            < 1e-3 * tr["round"] + 0.01
    # non-finite weights are caught in debug mode
    bad = init_flat([14, 50, 200, 2], 1)
    bad[3] = np.nan
    g = HipRoundEngine(X, y, 2, cfg, None, bad)
    with pytest.raises(FloatingPointError):
        g.run(1)
    # bf16 kernels with the fp16 gradient slab: a NaN gradient partial stays NaN (it is not
    # clamped to a finite bound), so the debug check sees it
    Xn = X.copy()
    Xn[5, 3] = np.nan
    h = HipRoundEngine(Xn, y, 2, EngineConfig(max_rounds=20, debug=True, early_stop=False, dtype="bf16",
                                              grad_slab="fp16"), None, init_flat([14, 50, 200, 2], 1))
    assert h.slab_f16
    with pytest.raises(FloatingPointError):
        h.run(1)


@pytest.mark.parametrize("R", [16, 32, 64])
@pytest.mark.parametrize("hidden", [(50, 200), (7,), (33, 17, 9)])
def test_bf16_engine_tracks_fp32_oracle(R, hidden):
    """bf16 MFMA operands (fp32 accumulate / master weights): one round's update matches the
    fp32 torch oracle to bf16 precision, and training tracks it over many rounds."""
    X, y = make_income_like(3000, seed=5)
    dims = [14, *hidden, 2]
    flat = init_flat(dims, 3)
    mk = lambda cls, **kw: cls(X, y, 2, EngineConfig(hidden=hidden, max_rounds=60, early_stop=False,
                                                      rows_per_block=R, **kw), None, flat)
    try:
        hb = mk(HipRoundEngine, dtype="bf16")
    except RuntimeError as err:  # split-bf16 layout of a big model at R = 64 exceeds the CU's LDS
        assert "LDS" in str(err) and R == 64
        pytest.skip(str(err))
    ref = mk(TorchRoundEngine)
    hb.run(1)
    ref.run(1)
    d0 = flat
    upd_b, upd_r = hb.global_flat() - d0, ref.global_flat() - d0
    # Adam's first step is ~lr * sign(g): compare update directions
    agree = np.mean(np.sign(upd_b) == np.sign(upd_r))
    assert agree > 0.97, agree
    hb.run(59)
    ref.run(59)
    acc_b, acc_r = hb.history()["global"][:, 0], ref.history()["global"][:, 0]
    assert abs(acc_b[-1] - acc_r[-1]) < 0.02, (acc_b[-1], acc_r[-1])
    assert abs(hb.history()["loss"][-1] - ref.history()["loss"][-1]) < 0.02


def test_bf16_grad_slab_auto_and_formats_agree():
    """grad_slab='auto' picks the fp16 slab for standardised features and the fp32 slab when a
    feature exceeds FP16_SLAB_MAX_ABS_X (a partial sum could saturate fp16); 40 rounds with either
    slab land on the same accuracy and loss."""
    from fedmi.fl.engine import FP16_SLAB_MAX_ABS_X
    X, y = make_income_like(3000, seed=5)
    flat = init_flat(DIMS, 3)
    mk = lambda X, **kw: HipRoundEngine(X, y, 2, EngineConfig(max_rounds=40, early_stop=False, dtype="bf16",
                                                              **kw), None, flat)
    auto = mk(X)
    assert auto.slab_f16
    big = X.copy()
    big[0, 0] = 2 * FP16_SLAB_MAX_ABS_X
    assert not mk(big).slab_f16
    assert not mk(X, grad_slab="fp32").slab_f16
    f32 = mk(X, grad_slab="fp32")
    auto.run(40)
    f32.run(40)
    ha, hf = auto.history(), f32.history()
    assert abs(ha["global"][-1, 0] - hf["global"][-1, 0]) < 0.01
    assert abs(ha["loss"][-1] - hf["loss"][-1]) < 0.01
    assert not auto.slab_saturated and int(auto.sat.item()) == 0


def test_bf16_fp16_slab_saturation_is_reported():
    """The fp16 slab clamps partials at +-65504 (slab_store_h); the Adam kernel flags any clamped
    or non-finite partial it reads, and the engine warns (debug mode: raises) at the next history
    read instead of training on silently clipped gradients."""
    import warnings
    X, y = make_income_like(3000, seed=5)
    big = (X * 1e5).astype(np.float32)      # partials of 32 rows x |x| ~ 1e5 >> 65504
    flat = init_flat(DIMS, 3)
    e = HipRoundEngine(big, y, 2, EngineConfig(max_rounds=8, early_stop=False, dtype="bf16", grad_slab="fp16",
                                               graph_rounds=0), None, flat)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        e.run(2)
        e.sync_history()
    assert e.slab_saturated and any("saturated" in str(x.message) for x in w)
    d = HipRoundEngine(big, y, 2, EngineConfig(max_rounds=8, early_stop=False, dtype="bf16", grad_slab="fp16",
                                               graph_rounds=0, debug=True), None, flat)
    with pytest.raises(FloatingPointError, match="saturated"):
        d.run(2)
        d.sync_history()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_eval_equals_classic_rounds(dtype):
    """One client: scoring round r inside round r+1's train kernel (fused evaluation) gives
    bit-identical weights, metric history and early-stop round to the separate eval kernel."""
    X, y = make_income_like(3000, seed=11)
    flat = init_flat(DIMS, 6)
    out = []
    for fused in (False, True):
        cfg = EngineConfig(max_rounds=200, patience=4, tolerance=2e-3, dtype=dtype, fused_eval=fused,
                           graph_rounds=8)
        e = HipRoundEngine(X, y, 2, cfg, None, flat)
        assert e.engine.fused == fused
        e.run(200)
        out.append((e.global_flat(), e.history()))
    (wc, hc), (wf, hf) = out
    assert hc["stop_round"] > 0 and hf["stop_round"] == hc["stop_round"]
    assert hf["rounds_run"] == hc["rounds_run"]
    np.testing.assert_array_equal(wf, wc)
    np.testing.assert_array_equal(hf["global"], hc["global"])
    np.testing.assert_array_equal(hf["loss"], hc["loss"])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("graph_rounds", [0, 16])
def test_fused_eval_launches_no_eval_kernel_per_round(dtype, graph_rounds):
    """A one-client fused run of 64 rounds issues at most one stand-alone evaluation kernel
    (the run's closing flush), eager or graph-replayed.  Round 3's fp32 path flushed one per
    round (need_pack_ was never cleared by the fp32 train launch)."""
    X, y = make_income_like(2000, seed=13)
    cfg = EngineConfig(max_rounds=80, early_stop=False, dtype=dtype, graph_rounds=graph_rounds)
    e = HipRoundEngine(X, y, 2, cfg, None, init_flat(DIMS, 3))
    assert e.engine.fused
    e.run(64, check_every=64)
    assert e.history()["rounds_run"] == 64
    assert e.engine.eval_launches <= 1, e.engine.eval_launches
    # a host-side weight change scores the pending round with the old model once, then fuses again
    e.set_global_flat(e.global_flat())
    e.run(8, check_every=8)
    assert e.engine.eval_launches <= 3, e.engine.eval_launches


def test_fused_eval_mixed_with_step_api():
    """Fused rounds, then reference step-by-step rounds (classic), then fused again: the
    pending/evaluated hand-over keeps every round's metrics exact."""
    X, y = make_income_like(2000, seed=12)
    flat = init_flat(DIMS, 7)
    hist = []
    for fused in (False, True):
        e = HipRoundEngine(X, y, 2, EngineConfig(max_rounds=40, early_stop=False, fused_eval=fused,
                                                 graph_rounds=4), None, flat)
        e.run(5)
        cms = []
        for _ in range(2):
            e.step_train()
            cms.append(e.step_eval())
            e.step_aggregate()
        e.run(7)
        e.sync_history()
        hist.append((e.history(), cms, e.global_flat()))
    assert hist[0][0]["rounds_run"] == hist[1][0]["rounds_run"] == 14
    np.testing.assert_array_equal(hist[0][0]["global"], hist[1][0]["global"])
    np.testing.assert_array_equal(hist[0][1], hist[1][1])
    np.testing.assert_array_equal(hist[0][2], hist[1][2])


def test_bf16_engine_layout_fits_one_cu():
    """The split-bf16 train layout (hi + lo weight images, lo activation buffers) of the reference
    model fits one CU's LDS at the bench's 32 rows per workgroup."""
    X, y = make_income_like(500, seed=1)
    e = HipRoundEngine(X, y, 2, EngineConfig(rows_per_block=32, dtype="bf16"), None, init_flat(DIMS, 0))
    lay = e.engine.layout()
    assert lay["dtype"] == 1 and lay["lds_bytes"] <= 158 * 1024, lay["lds_bytes"]
    assert lay["eval_lds_bytes"] <= lay["lds_bytes"]


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float64)


def _split_bf16_reference_grad(flat, X, y, dims, scaled_delta=False):
    """Host model of the bf16 train kernel's arithmetic (fl_kernels_bf16.hip), in float64:
    split-bf16 forward (hi.hi + lo.hi + hi.lo, hidden outputs split into hi/lo after ReLU),
    softmax-CE deltas rounded to bf16, backward on the hi parts with bf16 deltas."""
    from fedmi.models.mlp import flat_to_dict
    d = flat_to_dict(flat, dims)
    L = len(dims) - 1
    Ws = [torch.as_tensor(d[f"model.{2 * l}.weight"], dtype=torch.float64) for l in range(L)]
    bs = [torch.as_tensor(d[f"model.{2 * l}.bias"], dtype=torch.float64) for l in range(L)]
    a = torch.as_tensor(X, dtype=torch.float32).to(torch.float64)
    yt = torch.as_tensor(y, dtype=torch.long)
    his, pre = [], []
    for l in range(L):
        ah, wh = _bf(a), _bf(Ws[l])
        al, wl = _bf(a - ah), _bf(Ws[l] - wh)
        z = ah @ wh.T + (al @ wh.T + ah @ wl.T) + bs[l]
        his.append(ah)
        pre.append(z)
        a = torch.relu(z).to(torch.float32).to(torch.float64)
    n = len(y)
    p = torch.softmax(z, 1)
    dz = p.clone()
    dz[torch.arange(n), yt] -= 1.0
    # fp16 slab: the kernels back-propagate the unscaled delta (Adam applies the 1/n); fp32
    # slab: the delta of the mean loss
    sc = 1.0 if scaled_delta else float(n)
    dz = _bf(dz / n) if scaled_delta else _bf(dz)
    gW, gb = [None] * L, [None] * L
    for l in range(L - 1, -1, -1):
        gW[l] = dz.T @ his[l] / sc
        gb[l] = dz.sum(0) / sc
        if l:
            dz = _bf((dz @ _bf(Ws[l])) * (his[l] > 0))
    return torch.cat([torch.cat([gW[l].reshape(-1), gb[l]]) for l in range(L)]).numpy()


@pytest.mark.parametrize("R,slab", [(16, "fp16"), (32, "fp16"), (32, "fp32")])
def test_bf16_train_kernel_gradient(R, slab):
    """The slab-reduced gradient of ONE fl_train_bf16 launch (reduced here in float64) vs (a) a
    float64 host model of the kernel's own arithmetic (split-bf16 forward, bf16 backward
    operands): rel. err <= 1e-3 per tensor, and (b) fp32 torch autograd of the exact model: rel.
    err <= 1e-2 per tensor.  R = 16 runs the conflict-free LDS layout (level 2: W row gaps),
    R = 32 the compact one (level 1: swizzled W chunks) -- fl_common.h.  slab fp16: partial sums
    of the unscaled gradient (the Adam kernel applies the 1/n); fp32: partials of the mean."""
    X, y = make_income_like(4000, seed=21)
    dims = DIMS
    flat = init_flat(dims, 8)
    e = HipRoundEngine(X, y, 2, EngineConfig(max_rounds=4, early_stop=False, rows_per_block=R, dtype="bf16",
                                             graph_rounds=0, grad_slab=slab), None, flat)
    assert e.engine.layout()["bank_level"] == (2 if R == 16 else 1)
    e.step_train()
    e.stream.synchronize()
    P = e.P
    lay = e.engine.layout()
    assert lay["slab_f16"] == (slab == "fp16") == e.slab_f16
    g = e.slab_partials().double().sum(0).cpu().numpy()
    if slab == "fp16":
        g /= len(X)
    ref = _split_bf16_reference_grad(flat, X, y, dims, scaled_delta=slab == "fp32")
    model = TorchRoundEngine(X, y, 2, EngineConfig(max_rounds=2), None, flat)
    out = model.model(torch.as_tensor(X))
    torch.nn.functional.cross_entropy(out, torch.as_tensor(y, dtype=torch.long)).backward()
    auto = torch.cat([p.grad.reshape(-1) for p in model.model.parameters()]).double().numpy()
    off = 0
    for l in range(len(dims) - 1):
        for n in (dims[l] * dims[l + 1], dims[l + 1]):
            sl = slice(off, off + n)
            err_k = np.linalg.norm(g[sl] - ref[sl]) / np.linalg.norm(ref[sl])
            err_a = np.linalg.norm(g[sl] - auto[sl]) / np.linalg.norm(auto[sl])
            assert err_k <= 1e-3, (l, n, err_k)
            assert err_a <= 1e-2, (l, n, err_a)
            off += n


@pytest.mark.parametrize("hidden,C,R", [((50, 200), 2, 32), ((50, 200), 2, 16), ((24, 12), 2, 32), ((64,), 2, 32),
                                        ((40, 96), 3, 32), ((40, 96), 5, 32)])
def test_lagged_register_scoring_equals_serial_pass(hidden, C, R, monkeypatch):
    """Lagged rounds (several clients: round r's post-step local model scored inside round r+1's
    train kernel) score in registers on the waves the training forward pass leaves idle
    (fl_kernels_bf16.hip score_rows_regs), and the training forward of several clients is then
    plain bf16 (FLConfig::plain_fwd) in every kind of round: per-client metrics, loss history and
    weights of lagged rounds are bit-identical to classic rounds with a separate evaluation
    kernel.  With FEDMI_LAG_REG=0 the serial scoring pass and the split training forward are
    bit-identical to classic rounds likewise.  One and two hidden layers, 16 / 32 rows per
    workgroup, C = 3, a partial last row block; C = 5 (> FL_LAG_MAX_C) takes the serial pass."""
    X, y = make_income_like(2100, seed=21)
    if C > 2:
        y = ((X[:, 0] > 0).astype(np.int64) + 2 * (X[:, 1] > 0) + (X[:, 2] > 0.5)) % C
    flat = init_flat([14, *hidden, C], 8)
    eligible = C <= 4
    out = {}
    # FEDMI_SPLIT_SCORE: register scoring on workgroups of its own (train kernel LAG 3; the
    # default where 2 n_slabs <= #CUs -- forced here) or on the training workgroups' idle waves (LAG 2)
    for env, split in ((None, "1"), (None, "0"), ("0", None)):
        for lagged in (True, False):
            if env is None:
                monkeypatch.delenv("FEDMI_LAG_REG", raising=False)
            else:
                monkeypatch.setenv("FEDMI_LAG_REG", env)
            if split is None:
                monkeypatch.delenv("FEDMI_SPLIT_SCORE", raising=False)
            else:
                monkeypatch.setenv("FEDMI_SPLIT_SCORE", split)
            cfg = EngineConfig(hidden=tuple(hidden), max_rounds=40, early_stop=False, dtype="bf16", graph_rounds=4,
                               rows_per_block=R, fused_eval=False, lagged_eval=lagged)
            e = HipRoundEngine(X, y, C, cfg, None, flat, emulate_clients=True)
            assert bool(e.engine.lagged) == lagged
            lay = e.engine.layout()
            assert lay["lag_reg"] == (env is None and eligible)
            assert lay["plain_fwd"] == (env is None and eligible)
            assert lay["split_score"] == (lagged and env is None and eligible and split == "1")
            e.run(3)
            e.run(9)
            e.sync_history()
            h = e.history()
            assert h["rounds_run"] == 12
            out[(env, split, lagged)] = (e.global_flat(), h)
    for env, split in ((None, "1"), (None, "0"), ("0", None)):
        (wl, hl), (wc, hc) = out[(env, split, True)], out[(env, split, False)]
        name = f"FEDMI_LAG_REG={env} FEDMI_SPLIT_SCORE={split}"
        np.testing.assert_array_equal(wl, wc, err_msg=name)
        np.testing.assert_array_equal(hl["global"], hc["global"], err_msg=name)
        np.testing.assert_array_equal(hl["per_rank"], hc["per_rank"], err_msg=name)
        np.testing.assert_array_equal(hl["loss"], hc["loss"], err_msg=name)
    if eligible:  # the plain training forward changes the trajectory, not its quality
        a, b = out[(None, "1", True)][1]["global"][-1], out[("0", None, True)][1]["global"][-1]
        assert abs(a[0] - b[0]) < 0.02, (a, b)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("patience", [1, 2, 3, 5])
def test_early_stop_fold_only_where_it_can_stop(dtype, patience):
    """Blocks other than the history block fold the previous round only when the fold can stop
    training (patience counter <= 2, fl_device.h fold_may_stop).  For every patience: the device's
    stop round is the host rule (EarlyStopper, C:181-192) applied to the device's own metric
    history, and the rounds issued past the stop leave the model bit-identical to a run that
    simply ends at the stop round -- so no block ever updated a round the rule had stopped."""
    from fedmi.fl.early_stop import EarlyStopper
    X, y = make_income_like(2500, seed=17)
    flat = init_flat(DIMS, 8)
    cfg = EngineConfig(max_rounds=160, patience=patience, tolerance=3e-3, dtype=dtype, graph_rounds=8)
    e = HipRoundEngine(X, y, 2, cfg, None, flat)
    e.run(160)
    h = e.history()
    s = h["stop_round"]
    assert 0 < s < 160, s
    es = EarlyStopper(patience, 3e-3)
    host = next(r + 1 for r in range(h["rounds_run"]) if es.update(h["global"][r]))
    assert host == s, (host, s)
    ref = HipRoundEngine(X, y, 2, EngineConfig(max_rounds=s, early_stop=False, dtype=dtype, graph_rounds=8), None,
                         flat)
    ref.run(s)
    np.testing.assert_array_equal(e.global_flat(), ref.global_flat())
    np.testing.assert_array_equal(e.history()["global"][:s], ref.history()["global"][:s])


@pytest.mark.parametrize("R", [16, 32])
@pytest.mark.parametrize("es", [False, True])
def test_lagged_graph_captured_behind_self_evaluating_round(R, es):
    """A lagged graph captured right behind a round that followed a self-evaluating one (a run
    that closed on an odd round count, then more rounds; bench.py's warm-up + prime) used to skip
    the region-A fold in the first round of every later replay: those rounds' metrics never
    reached the history and the early-stop rule stopped late (33 vs 58).  The graph now starts
    only behind a lagged round that scored its predecessor (FLEngine::needs_eager_round), so
    lagged rounds (metrics folded one round late, no in-kernel exchange) equal classic rounds
    bit for bit across many replays, in both issue paths."""
    X, y = make_income_like(1500, seed=23)
    flat = init_flat(DIMS, 9)
    n = 120 if es else 40
    out = {}
    for lagged in (True, False):
        cfg = EngineConfig(max_rounds=n, early_stop=es, patience=3, tolerance=3e-3, dtype="bf16", graph_rounds=4,
                           rows_per_block=R, fused_eval=False, lagged_eval=lagged)
        e = HipRoundEngine(X, y, 2, cfg, None, flat, emulate_clients=True)
        assert bool(e.engine.lagged) == lagged
        e.run(3)                       # closes on round 2
        e.run(n - 8)                   # eager rounds, then graph replays (below max_rounds)
        e.sync_history()
        a = (e.global_flat(), e.history())
        # bench.py's shape: warm-up closing on an odd count, prime (eager rounds + capture + one
        # replay), replays with the last round left lagged, one closing round
        cfg2 = EngineConfig(max_rounds=64, early_stop=False, dtype="bf16", graph_rounds=4, rows_per_block=R,
                            fused_eval=False, lagged_eval=lagged)
        e2 = HipRoundEngine(X, y, 2, cfg2, None, flat, emulate_clients=True)
        if lagged:
            e2.run(5, check_every=5)
            e2.prime_graph(4)
            e2._issue(16, close=False)
            e2._issue(1)
            total = e2.rounds_issued
        else:                          # the same number of classic rounds
            e2.run(total)
        e2.sync_history()
        out[lagged] = (a, (e2.global_flat(), e2.history()))
    for j, name in enumerate(("run", "bench shape")):
        (wl, hl), (wc, hc) = out[True][j], out[False][j]
        k = hc["rounds_run"]
        assert hl["rounds_run"] == k and hl["stop_round"] == hc["stop_round"], (name, hl["rounds_run"], k)
        if es and j == 0:
            assert 0 < hc["stop_round"] < n - 5, hc["stop_round"]
        np.testing.assert_array_equal(wl, wc, err_msg=name)
        bad = np.flatnonzero(np.any(hl["global"][:k] != hc["global"][:k], axis=1))
        assert len(bad) == 0, (name, k, bad)
        np.testing.assert_array_equal(hl["per_rank"][:k], hc["per_rank"][:k], err_msg=name)
        np.testing.assert_array_equal(hl["loss"][:k], hc["loss"][:k], err_msg=name)


def test_graph_cache_across_run_and_streaming():
    """run() replays graphs of cfg.graph_rounds rounds, run_streaming (the console) shorter ones
    for lagged engines; the engine caches instantiated graphs per round count, so alternating the
    two APIs captures each length ONCE -- and the rounds stay bit-identical to a
    plain run()."""
    X, y = make_income_like(2000, seed=31)
    flat = init_flat(DIMS, 4)
    cfg = dict(max_rounds=260, early_stop=False, dtype="bf16", graph_rounds=16, fused_eval=False, lagged_eval=True)
    e = HipRoundEngine(X, y, 2, EngineConfig(**cfg), None, flat, emulate_clients=True)
    assert e.engine.lagged
    for _ in range(3):
        e.run(40)
        e.run_streaming(40, chunk=16)
    e.sync_history()
    assert e.engine.graph_captures == 2, e.engine.graph_captures   # one per graph length
    ref = HipRoundEngine(X, y, 2, EngineConfig(**cfg), None, flat, emulate_clients=True)
    ref.run(240)
    ref.sync_history()
    assert e.rounds_issued == ref.rounds_issued
    np.testing.assert_array_equal(e.global_flat(), ref.global_flat())
    np.testing.assert_array_equal(e.history()["global"], ref.history()["global"])


# relative L2 distance of the bf16 engine's global weights from the fp32 torch oracle, one
# client, by round: measured (profiles/bf16_drift_vs_fp32_oracle_r5.jsonl, tools/bf16_drift.py)
# split-bf16 forward 0.0017-0.0018 / 0.0024-0.0040 / 0.0064-0.0108 / 0.0145-0.0176 at rounds
# 1 / 5 / 20 / 60; a plain-bf16 forward 0.0045 / 0.0068 / 0.0118 / 0.024-0.0285 (exact fp32: 1e-7)
BF16_DRIFT_TOL = {1: 3e-3, 5: 5e-3, 20: 1.5e-2, 60: 2.5e-2}


@pytest.mark.parametrize("seed,hidden", [(3, (50, 200)), (5, (50, 200)), (7, (33, 17, 9))])
def test_bf16_weight_drift_vs_fp32_oracle(seed, hidden):
    """Round-by-round bound on the bf16 engine's weight drift from the fp32 torch oracle
    (nn.Linear + autograd + Adam + StepLR) at rounds 1, 5, 20 and 60 -- tight enough that a
    one-client engine silently training with a plain-bf16 forward instead of the split-bf16 one
    fails it (checked below on the same data: the plain forward exceeds the round-1 bound)."""
    X, y = make_income_like(3000, seed=seed)
    dims = [14, *hidden, 2]
    flat = init_flat(dims, seed)
    base = dict(hidden=hidden, max_rounds=80, early_stop=False)
    ref = TorchRoundEngine(X, y, 2, EngineConfig(**base), None, flat)
    hb = HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", **base), None, flat)
    assert not hb.layout.get("plain_fwd", False)       # one client: the split forward
    done = 0
    for r, tol in BF16_DRIFT_TOL.items():
        ref.run(r - done)
        hb.run(r - done)
        done = r
        w, wr = hb.global_flat(), ref.global_flat()
        d = float(np.linalg.norm(w - wr) / np.linalg.norm(wr))
        assert d < tol, (r, d, tol)
        if r == 1:
            w1_ref = wr
    if hidden == (50, 200):
        # negative control: the same engine with a plain-bf16 training forward drifts past round 1's bound
        hp = HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", fused_eval=False, plain_fwd=True, **base), None, flat)
        assert hp.layout.get("plain_fwd", False)
        hp.run(1)
        dp = float(np.linalg.norm(hp.global_flat() - w1_ref) / np.linalg.norm(w1_ref))
        assert dp > BF16_DRIFT_TOL[1], dp
