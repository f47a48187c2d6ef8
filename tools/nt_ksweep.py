"""NT GEMM fixed (prologue + epilogue) vs per-K-tile cost: time M x N x K for a K sweep at fixed
M, N (Cb bf16 output) and fit t(K) = f + K/64 * t_k per tile wave; hipBLASLt alongside.

    python tools/nt_ksweep.py [variant ...]      (default: 2 3)"""
import sys, time
import torch
sys.path.insert(0, ".")
from fedmi.ops import native

m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream


def bench(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


variants = [int(v) for v in sys.argv[1:]] or [2, 3]
for var, (M, N) in [(v, mn) for mn in [(16384, 4096), (8192, 8192)] for v in variants]:
    m.gemm_nt_set_variant(var)
    print(f"-- variant {var}", flush=True)
    Kmax = 8192
    A = (torch.rand(M, Kmax, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kmax, device=dev) * 2 - 1).to(torch.bfloat16)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    pts = []
    for K in (256, 1024, 2048, 4096, 8192):
        a, b = A[:, :K], B[:, :K]
        dtt = bench(lambda: a @ b.t())
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), Kmax, B.data_ptr(), Kmax, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0,
                              0, 1.0, 0.0, s)
        dt = bench(f)
        pts.append((K, dt))
        ref = (a @ b.t()).float()
        err = ((Cb.float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2 * M * N * K
        print(f"{M}x{N}x{K}: fedmi {dt*1e6:8.1f} us {fl/dt/1e12:6.0f} TF/s | hipBLASLt {dtt*1e6:8.1f} us "
              f"{fl/dtt/1e12:6.0f} TF/s | err {err:.1e}", flush=True)
    import numpy as np
    k = np.array([p[0] for p in pts], float) / 64
    t = np.array([p[1] for p in pts]) * 1e6
    waves = M * N / (256 * 256) / 256
    slope, icpt = np.polyfit(k, t / waves, 1)
    print(f"  fit per tile wave: fixed {icpt:.1f} us + {slope:.3f} us per K-tile "
          f"(main loop {256*256*64*2*256/slope/1e6:.0f} TF/s)", flush=True)
