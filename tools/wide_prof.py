"""Wide-MLP round profiling driver (rocprofv3 --kernel-trace --stats): 14-4096^3-2, 131072 rows,
micro-batch = argv[1] rows (default: the whole shard), bf16, 4 rounds."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedmi.fl.wide import WideClient

dev = torch.device("cuda", 0)
rows = 1 << 17
X = torch.randn(rows, 14, device=dev)
y = torch.randint(0, 2, (rows,), device=dev)
mb = int(sys.argv[1]) if len(sys.argv) > 1 else rows
c = WideClient(X, y, [14, 4096, 4096, 4096, 2], micro_batch=mb, dtype="bf16")
for _ in range(4):
    c.run_round()
torch.cuda.synchronize()
print("ok", c.nt_calls)
