"""NT GEMM epilogue cost: K = 64 (epilogue-bound) and K = 4096 launches with each output kind."""
import sys, time
import torch
sys.path.insert(0, ".")
from fedmi.ops import native

m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
M, N = 16384, 4096
for K in (64, 4096):
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    CbT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
    C = torch.zeros(M, N, device=dev)
    mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    cases = {"none": (0, 0, 0, 0, 0.0), "Cb": (0, Cb.data_ptr(), 0, 0, 0.0), "CbT": (0, 0, CbT.data_ptr(), 0, 0.0),
             "Cb+CbT": (0, Cb.data_ptr(), CbT.data_ptr(), 0, 0.0),
             "Cb+CbT+mask": (0, Cb.data_ptr(), CbT.data_ptr(), mask.data_ptr(), 0.0),
             "C fp32 beta=1": (C.data_ptr(), 0, 0, 0, 1.0)}
    line = f"K={K}:"
    for name, (c, cb, cbt, mk, beta) in cases.items():
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, c, N, cb, N, cbt, M, bias.data_ptr(), mk, N,
                              1, 1.0, beta, s)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        line += f" | {name} {(time.time() - t) / 10 * 1e6:.0f} us"
    print(line, flush=True)
