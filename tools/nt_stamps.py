"""In-kernel phase stamps (s_memrealtime, 100 MHz) of the full-line NT GEMM: per block, start ->
prologue landed -> steady main loop done -> last two K-tiles done -> epilogue stores issued,
plus the gap between a block's end and the next block's start on the same slot.

    python tools/nt_stamps.py [M N K]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from fedmi.ops import native  # noqa: E402

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 4096)))
m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
nb = (M // 256) * (N // 256)
dbg = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
run = lambda: m.gemm_nt(M, N, K, A.data_ptr(), K, B.data_ptr(), K, 0, 0, Cb.data_ptr(), N, 0, 0, 0, 0, 0, 0, 1.0,
                        0.0, s)
for _ in range(3):
    run()
m.gemm_nt_set_debug(dbg.data_ptr())
run()
torch.cuda.synchronize()
m.gemm_nt_set_debug(0)
st_all = dbg.view(nb, 8).cpu().numpy().astype(np.int64)
st = st_all[:, :5]
t0 = st[:, 0].min()
us = (st - t0) * 0.01
print(f"{M}x{N}x{K}: {nb} blocks, kernel span {us[:, 4].max():.1f} us (stamps)")
names = ["prologue (start -> first K-tile landed)", "steady main loop", "last two K-tiles",
         "epilogue (until the stores are issued)"]
order = np.argsort(us[:, 0])
first = np.zeros(nb, bool)
first[order[:min(256, nb)]] = True
for i, nm in enumerate(names):
    d = us[:, i + 1] - us[:, i]
    print(f"  {nm:42s} median {np.median(d):7.2f} us  p10 {np.percentile(d, 10):7.2f}  p90 {np.percentile(d, 90):7.2f}"
          f"  | first wave {np.median(d[first]):7.2f}, later {np.median(d[~first]) if (~first).any() else 0:7.2f}")
if (st_all[:, 5] > 0).all():
    e = (st_all[:, [3, 5, 6, 4]] - t0) * 0.01
    for nm, a, b in (("  epilogue: values into the LDS tile", 0, 1), ("  epilogue: barrier", 1, 2),
                     ("  epilogue: LDS reads + global stores issued", 2, 3)):
        print(f"  {nm:42s} median {np.median(e[:, b] - e[:, a]):7.2f} us")
# slot reuse: sort blocks by start; the k-th block of wave w+1 starts after some block of wave w ends
starts = np.sort(us[:, 0])
ends = np.sort(us[:, 4])
ncu = 256
if nb > ncu:
    gaps = starts[ncu:] - ends[:nb - ncu]
    print(f"  relaunch gap (k-th end -> (k+{ncu})-th start) median {np.median(gaps):.2f} us, p90 {np.percentile(gaps, 90):.2f}")
print(f"  block lifetime median {np.median(us[:, 4] - us[:, 0]):.1f} us; first wave start spread {starts[ncu - 1] - starts[0]:.2f} us")
