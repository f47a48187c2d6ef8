"""Which hipBLASLt kernels does torch pick for the wide path's bf16 NT shapes?  Run under
``rocprofv3 --kernel-trace --stats`` and read the kernel names (macro tile MT, matrix
instruction MI, workgroup mapping, prefetch depths are encoded in them)."""
import torch

dev = torch.device("cuda", 0)
for (M, N, K) in [(16384, 4096, 4096), (131072, 4096, 4096), (4096, 4096, 131072), (8192, 8192, 8192)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        C = A @ B.t()
    torch.cuda.synchronize()
    del A, B, C
    torch.cuda.empty_cache()
