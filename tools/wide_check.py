"""Wide-MLP client: correctness vs torch (small dims) + throughput (4096 wide)."""
import sys, time, numpy as np, torch
sys.path.insert(0, ".")
from fedmi.fl.wide import WideClient
from fedmi.data.synthetic import make_income_like
dev = torch.device("cuda", 0)
X, y = make_income_like(3000, seed=0)
Xt = torch.as_tensor(X, device=dev); yt = torch.as_tensor(y, device=dev)
for dt in ("fp32", "bf16"):
    c = WideClient(Xt, yt, [14, 64, 48, 2], micro_batch=1024, dtype=dt)
    ref = torch.nn.Sequential(torch.nn.Linear(14, 64), torch.nn.ReLU(), torch.nn.Linear(64, 48), torch.nn.ReLU(), torch.nn.Linear(48, 2)).to(dev)
    with torch.no_grad():
        for p, (w) in zip([ref[0].weight, ref[0].bias, ref[2].weight, ref[2].bias, ref[4].weight, ref[4].bias],
                          [c.W[0], c.b[0], c.W[1], c.b[1], c.W[2], c.b[2]]):
            p.copy_(w)
    opt = torch.optim.Adam(ref.parameters(), lr=0.004)
    for r in range(5):
        c.run_round()
        opt.zero_grad(); torch.nn.functional.cross_entropy(ref(Xt), yt.long()).backward(); opt.step()
    torch.cuda.synchronize()
    flat_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    err = ((c.params - flat_ref).abs().max() / flat_ref.abs().max()).item()
    print(f"{dt}: 5 rounds rel weight err vs torch fp32 {err:.2e}, loss {c.loss():.4f}", flush=True)
rows = 1 << 17
Xw = torch.randn(rows, 14, device=dev); yw = torch.randint(0, 2, (rows,), device=dev)
c = WideClient(Xw, yw, [14, 4096, 4096, 4096, 2], micro_batch=16384, dtype="bf16")
c.run_round(); torch.cuda.synchronize()
t = time.time(); n = 3
for _ in range(n): c.run_round()
torch.cuda.synchronize(); dt = (time.time() - t) / n
print(f"wide bf16: rows={rows} {dt*1e3:.1f} ms/round, {c.flops_per_round/dt/1e12:.1f} TFLOP/s, {rows/dt/1e6:.2f} M samples/s", flush=True)
