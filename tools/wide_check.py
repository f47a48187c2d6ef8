"""Wide-MLP client: correctness vs torch (small dims) + NT GEMM and 4096-wide round throughput."""
import sys, time, torch
sys.path.insert(0, ".")
from fedmi.fl.wide import WideClient
from fedmi.data.synthetic import make_income_like
from fedmi.ops import native

dev = torch.device("cuda", 0)
m = native()
s = torch.cuda.current_stream().cuda_stream
# raw NT GEMM throughput at the wide-layer shapes (random operands), both main-loop variants
def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t) / n


for (M, N, K) in [(16384, 4096, 4096), (4096, 4096, 16384), (8192, 8192, 8192)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ref = A @ B.t()
    dtt = bench(lambda: A @ B.t())
    line = f"gemm_nt {M}x{N}x{K}: torch(hipBLASLt) {2*M*N*K/dtt/1e12:.0f} TF/s"
    for v in (1, 2):
        m.gemm_nt_set_variant(v)
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0, 0,
                              1.0, 0.0, s)
        dt = bench(f)
        err = ((Cb.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        line += f" | v{v} {dt*1e3:.3f} ms {2*M*N*K/dt/1e12:.0f} TF/s err {err:.1e}"
    print(line, flush=True)
m.gemm_nt_set_variant(3)

X, y = make_income_like(4096, seed=0)
Xt = torch.as_tensor(X, device=dev); yt = torch.as_tensor(y, device=dev)
for dt_, dims in (("fp32", [14, 64, 48, 2]), ("bf16", [14, 64, 48, 2]), ("bf16", [14, 256, 256, 2])):
    c = WideClient(Xt, yt, dims, micro_batch=1024, dtype=dt_, lr=0.004)
    layers = []
    for a, b in zip(dims[:-1], dims[1:]):
        layers += [torch.nn.Linear(a, b), torch.nn.ReLU()]
    ref = torch.nn.Sequential(*layers[:-1]).to(dev)
    with torch.no_grad():
        ws = [t for pair in zip(c.W, c.b) for t in pair]
        for p, w in zip(ref.parameters(), ws):
            p.copy_(w)
    opt = torch.optim.Adam(ref.parameters(), lr=0.004)
    for r in range(5):
        c.run_round()
        opt.zero_grad(); torch.nn.functional.cross_entropy(ref(Xt), yt.long()).backward(); opt.step()
    torch.cuda.synchronize()
    flat_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    err = ((c.params - flat_ref).abs().max() / flat_ref.abs().max()).item()
    print(f"{dt_} {dims}: 5 rounds rel weight err vs torch fp32 {err:.2e}, loss {c.loss():.4f}, nt_calls {c.nt_calls}",
          flush=True)
rows = 1 << 17
Xw = torch.randn(rows, 14, device=dev); yw = torch.randint(0, 2, (rows,), device=dev)
for mb in [int(a) for a in sys.argv[1:]] or [16384]:
    c = WideClient(Xw, yw, [14, 4096, 4096, 4096, 2], micro_batch=mb, dtype="bf16")
    c.run_round(); torch.cuda.synchronize()
    t = time.time(); n = 3
    for _ in range(n): c.run_round()
    torch.cuda.synchronize(); dt = (time.time() - t) / n
    print(f"wide bf16: rows={rows} micro-batch {mb}: {dt*1e3:.1f} ms/round, {c.flops_per_round/dt/1e12:.1f} TFLOP/s, "
          f"{rows/dt/1e6:.2f} M samples/s", flush=True)
    del c
    torch.cuda.empty_cache()
