"""NT GEMM vs hipBLASLt (torch.matmul) at the wide client's own shapes (BASELINE config 3,
131072-row micro-batches of the 14-4096^3-2 MLP): forward / dgrad M=131072 N=4096 K=4096
(bf16 out) and weight gradient M=N=4096 K=131072 (fp32 out); the forward also with its real epilogue
(bias + ReLU + bf16 + transposed bf16 copy).

    python tools/probes/nt_wide_shapes.py [variant ...]      (default: 3)"""
import sys
import torch
sys.path.insert(0, ".")
from fedmi.ops import native

m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream


def bench(fn, n=10):
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


VARIANTS = [int(v) for v in sys.argv[1:]] or [3]
for var, (M, N, K, out) in [(v, c) for c in ((131072, 4096, 4096, "bf16"), (131072, 4096, 4096, "fwd"),
                                             (4096, 4096, 131072, "fp32")) for v in VARIANTS]:
    m.gemm_nt_set_variant(var)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    if out == "bf16":
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0, 0,
                              1.0, 0.0, s)
        ref = lambda: A @ B.t()
    elif out == "fwd":
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        CbT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
        bias = torch.rand(N, device=dev)
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, CbT.data_ptr(), M,
                              bias.data_ptr(), 0, 0, 1, 1.0, 0.0, s)
        ref = lambda: A @ B.t()
    else:
        C = torch.empty(M, N, dtype=torch.float32, device=dev)
        f = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), N, 0, 0, 0, 0, 0, 0, 0, 0,
                              1.0, 0.0, s)
        ref = lambda: torch.mm(A, B.t(), out_dtype=torch.float32)
    dt = bench(f)
    try:
        dtt = bench(ref)
    except (TypeError, RuntimeError):  # no fp32-output bf16 mm in this torch: bf16 output instead
        dtt = bench(lambda: A @ B.t())
    fl = 2 * M * N * K
    print(f"v{var} {M}x{N}x{K} ({out} out): fedmi {dt*1e3:8.3f} ms {fl/dt/1e12:6.0f} TF/s | hipBLASLt {dtt*1e3:8.3f} ms "
          f"{fl/dtt/1e12:6.0f} TF/s | {dtt/dt*100:5.1f} %", flush=True)
m.gemm_nt_set_variant(3)
