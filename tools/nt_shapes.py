"""NT GEMM (C = A . B^T, bf16 in, bf16 out) at given shapes vs hipBLASLt (torch), hipEvents.

    python tools/nt_shapes.py [M,N,K ...]      (default: the wide client's shapes + the K-sweep shapes)"""
import sys
import torch
sys.path.insert(0, ".")
from fedmi.ops import native

m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or \
    [(131072, 4096, 4096), (4096, 4096, 131072), (16384, 4096, 4096), (16384, 4096, 8192), (8192, 8192, 8192)]
m.gemm_nt_set_variant(3)
for M, N, K in shapes:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0, 0,
                          1.0, 0.0, s)
    dt = bench(f)
    dtt = bench(lambda: A @ B.t())
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K}: fedmi {dt*1e6:9.1f} us {fl/dt/1e12:6.0f} TF/s | hipBLASLt {dtt*1e6:9.1f} us "
          f"{fl/dtt/1e12:6.0f} TF/s | {dtt/dt*100:5.1f} %", flush=True)
    del A, B, Cb
    torch.cuda.empty_cache()
