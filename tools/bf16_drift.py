"""Relative L2 drift of the HIP engines' global weights from the fp32 torch oracle
(TorchRoundEngine: nn.Linear + autograd + torch.optim.Adam + StepLR) at rounds 1, 5, 20, 60, one
client: bf16 with the split-bf16 forward (the one-client default), bf16 with a plain-bf16 forward
(forced: fused_eval off, plain_fwd on), and the exact-fp32 kernels.  Sets the tolerances of
tests/test_hip_engine.py::test_bf16_weight_drift_vs_fp32_oracle."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fedmi.data.synthetic import make_income_like  # noqa: E402
from fedmi.fl.engine import EngineConfig, HipRoundEngine, TorchRoundEngine  # noqa: E402
from fedmi.models.mlp import init_flat  # noqa: E402

CHECK = (1, 5, 20, 60)


def drift(mk_eng, ref_w):
    e = mk_eng()
    out, done = [], 0
    for r in CHECK:
        e.run(r - done)
        done = r
        w = e.global_flat()
        out.append(float(np.linalg.norm(w - ref_w[r]) / np.linalg.norm(ref_w[r])))
    return out


def main():
    for seed, hidden in ((3, (50, 200)), (5, (50, 200)), (7, (33, 17, 9))):
        X, y = make_income_like(3000, seed=seed)
        dims = [14, *hidden, 2]
        flat = init_flat(dims, seed)
        base = dict(hidden=hidden, max_rounds=80, early_stop=False)
        ref = TorchRoundEngine(X, y, 2, EngineConfig(**base), None, flat)
        ref_w, done = {}, 0
        for r in CHECK:
            ref.run(r - done)
            done = r
            ref_w[r] = ref.global_flat()
        rec = {"seed": seed, "hidden": list(hidden), "rounds": list(CHECK)}
        rec["bf16_split"] = drift(lambda: HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", **base), None, flat), ref_w)
        e = HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", **base), None, flat)
        rec["split_layout"] = bool(not e.layout.get("plain_fwd", False))
        rec["bf16_plain"] = drift(lambda: HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", fused_eval=False,
                                                                               plain_fwd=True, **base), None, flat),
                                  ref_w)
        e = HipRoundEngine(X, y, 2, EngineConfig(dtype="bf16", fused_eval=False, plain_fwd=True, **base), None, flat)
        rec["plain_layout"] = bool(e.layout.get("plain_fwd", False))
        rec["fp32"] = drift(lambda: HipRoundEngine(X, y, 2, EngineConfig(dtype="fp32", **base), None, flat), ref_w)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
