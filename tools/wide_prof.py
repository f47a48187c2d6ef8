"""Wide-MLP round profiling driver (rocprofv3 --kernel-trace --stats): 14-4096^3-2, 131072 rows,
micro-batch 16384, bf16, one warm-up round + 3 rounds."""
import sys
import torch
sys.path.insert(0, ".")
from fedmi.fl.wide import WideClient

dev = torch.device("cuda", 0)
rows = 1 << 17
X = torch.randn(rows, 14, device=dev)
y = torch.randint(0, 2, (rows,), device=dev)
c = WideClient(X, y, [14, 4096, 4096, 4096, 2], micro_batch=16384, dtype="bf16")
for _ in range(4):
    c.run_round()
torch.cuda.synchronize()
print("ok", c.nt_calls)
