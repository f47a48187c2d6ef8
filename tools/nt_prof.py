"""NT GEMM profiling driver: a few launches of one shape/variant (for rocprofv3 --pmc passes)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedmi.ops import native

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 4096)))
v = int(sys.argv[4]) if len(sys.argv) > 4 else 3
m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
m.gemm_nt_set_variant(v)
for _ in range(5):
    m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0, 0, 1.0, 0.0, s)
torch.cuda.synchronize()
print("ok", M, N, K, v)
