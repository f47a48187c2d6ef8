"""GPU validation of the layered path: GEMM variants vs torch fp32, and the sklearn-style
estimator (HIP fp32, packed trials) vs the float64 numpy backend."""
import sys, time, warnings
import numpy as np, torch
sys.path.insert(0, ".")
warnings.filterwarnings("ignore")
from fedmi.ops import native
m = native()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
worst = 0
for dtype in (0, 1):
    for (M, N, K) in [(200, 50, 14), (200, 400, 50), (97, 33, 130), (512, 256, 1024)]:
        for epi in (0, 1, 2, 3):
            for akc, bkc in ((1, 1), (1, 0), (0, 0), (0, 1)):
                if epi == 3 and not akc: continue
                Af = torch.randn(M, K, device=dev) if akc else torch.randn(K, M, device=dev)
                Bf = torch.randn(N, K, device=dev) if bkc else torch.randn(K, N, device=dev)
                At = Af if akc else Af.t()
                Bt = Bf.t() if bkc else Bf
                bias = torch.randn(N, device=dev)
                mask = torch.randn(M, N, device=dev)
                C = torch.zeros(M, N, device=dev)
                Ain = Af if dtype == 0 else Af.to(torch.bfloat16)
                Bin = Bf if dtype == 0 else Bf.to(torch.bfloat16)
                m.gemm(M, N, K, Ain.data_ptr(), Af.shape[1], akc, Bin.data_ptr(), Bf.shape[1], bkc, C.data_ptr(), N, epi,
                       bias.data_ptr(), mask.data_ptr(), N, 0, 1.0, 0.0, dtype, 1, 0, 0, s)
                Aref = At.float() if dtype == 0 else At.to(torch.bfloat16).float()
                Bref = Bt.float() if dtype == 0 else Bt.to(torch.bfloat16).float()
                ref = (Aref.double() @ Bref.double()).float()
                if epi in (1, 2): ref = ref + bias
                if epi == 2: ref = ref.clamp_min(0)
                if epi == 3: ref = ref * (mask > 0)
                torch.cuda.synchronize()
                err = ((C - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
                worst = max(worst, err)
                if err > (2e-6 if dtype == 0 else 1e-2):
                    print("FAIL", dtype, M, N, K, epi, akc, bkc, err)
    # split-K
    M, N, K = 64, 96, 5000
    A = torch.randn(K, M, device=dev); Bm = torch.randn(K, N, device=dev)
    C = torch.ones(M, N, device=dev); slab = torch.zeros(4 * M * N, device=dev)
    Ain = A if dtype == 0 else A.to(torch.bfloat16); Bin = Bm if dtype == 0 else Bm.to(torch.bfloat16)
    m.gemm(M, N, K, Ain.data_ptr(), M, 0, Bin.data_ptr(), N, 0, C.data_ptr(), N, 0, 0, 0, 0, 0, 1.0, 1.0, dtype, 4,
           slab.data_ptr(), 0, s)
    ref = 1.0 + (Ain.float().t().double() @ Bin.float().double()).float()
    torch.cuda.synchronize()
    e = ((C - ref).abs().max() / ref.abs().max()).item()
    print(f"dtype={dtype} split-K rel err {e:.2e}")
print(f"GEMM worst rel err {worst:.2e}", flush=True)

from fedmi.models.sklearn_mlp import MLPClassifier, fit_packed
from fedmi.data.tabular import load_tabular
ds = load_tabular(with_mean=False)
X, y = ds.X_train, ds.y_train
for hl in [(50,), (50, 400)]:
    a = MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=0.004, max_iter=40, random_state=42, backend="numpy")
    t = time.time(); a.fit(X, y); ta = time.time() - t
    b = MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=0.004, max_iter=40, random_state=42, backend="hip")
    t = time.time(); b.fit(X, y); tb = time.time() - t
    print(hl, "n_iter", a.n_iter_, b.n_iter_, "loss", a.loss_curve_[:3], b.loss_curve_[:3], a.loss_, b.loss_,
          "agree", (a.predict(X) == b.predict(X)).mean(), "acc", a.score(X, y), b.score(X, y), f"{ta:.2f}s {tb:.2f}s", flush=True)
lrs = [0.002, 0.005, 0.004]
packed = [MLPClassifier(hidden_layer_sizes=(50, 200), learning_rate_init=lr, max_iter=60, random_state=42, backend="hip") for lr in lrs]
t = time.time(); fit_packed(packed, X, y); tp = time.time() - t
single = MLPClassifier(hidden_layer_sizes=(50, 200), learning_rate_init=0.005, max_iter=60, random_state=42, backend="hip").fit(X, y)
print("packed n_iter", [e.n_iter_ for e in packed], "single", single.n_iter_,
      "max coef diff packed[1] vs single", max(abs(u - v).max() for u, v in zip(packed[1].coefs_, single.coefs_)), f"{tp:.2f}s")
