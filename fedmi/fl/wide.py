"""Wide-MLP federated client (BASELINE config 3: MLP 14-4096-4096-4096-2 on large
synthetic income-shaped shards, MFMA-GEMM bound).

The fused round engine (``fedmi/fl/engine.py``) keeps a whole small MLP in one workgroup;
a 33.6 M-parameter model does not fit, so this client runs the same round semantics
(full-batch local Adam step(s) over the shard + StepLR, local eval, sample-weighted FedAvg)
layer by layer on the grid-level MFMA GEMMs of ``fedmi/ops/csrc/gemm_mfma.hip``:

* bf16 operands, fp32 accumulation, fp32 master weights / Adam state / gradients;
* the shard is processed in micro-batches with gradient accumulation (beta = 1 in the
  wgrad epilogue), which is exactly the full-batch gradient (row-wise scale-up);
* FedAvg = one RCCL all-reduce per layer bucket of the pre-scaled (n_i / N) fp32 weights,
  issued in FORWARD order on a side stream, each followed (same stream) by the bf16
  re-quantisation of its layer and an event.  FedAvg's data dependency is per layer: the
  next round's forward of layer l waits only on bucket l's event, so the all-reduce of the
  deeper (larger) buckets overlaps the first micro-batch's forward of the layers before
  them (SURVEY §5.8 "bucket per layer in forward order").
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..models.mlp import init_flat, param_layout


# Learning rate of the 4096-wide client (BASELINE config 3).  The reference's 0.004 (C:44) is
# tuned for the 14-50-200-2 MLP; a full-batch Adam step moves every one of a 4096-wide layer's
# inputs by ~lr at once, and at 0.004 the wide model diverges (loss 0.69 -> 74 -> 213 in rounds
# 1-3) -- exactly as an eager fp32 torch model from the same weights does (profiles/wide_learn_r3.log:
# per-round losses within 1 %), so it is the optimizer's divergence, not the kernels'.  At 1e-4 the
# same client reaches the synthetic task's Bayes accuracy (0.85) by round 6 and tracks torch to
# 2e-4 in loss.
WIDE_LR = 1e-4


class WideClient:
    def __init__(self, X: torch.Tensor, y: torch.Tensor, dims: Sequence[int], comm=None, n_total: Optional[int] = None,
                 micro_batch: int = 131072, lr: Optional[float] = None, betas=(0.9, 0.999), eps: float = 1e-8,
                 step_size: int = 30, gamma: float = 0.5, seed: int = 0, dtype: str = "bf16",
                 eval_rows: int = 0, allreduce_dtype: str = "fp32", warmup_rounds: int = 0,
                 fused_eval: Optional[bool] = None):
        from ..ops import native
        self.m = native()
        self.dev = X.device
        self.X, self.y = X.contiguous(), y.to(torch.int32).contiguous()
        self.n = int(X.shape[0])
        self.dims = [int(d) for d in dims]
        self.L = len(self.dims) - 1
        self.comm = comm
        self.world = comm.size if comm is not None else 1
        self.n_total = n_total or self.n * self.world
        self.agg = self.n / self.n_total
        self.mb = min(micro_batch, self.n)
        # (None: WIDE_LR -- the reference's 0.004 diverges at width 4096, see WIDE_LR)
        self.lr, self.betas, self.eps = (WIDE_LR if lr is None else float(lr)), betas, eps
        self.step_size, self.gamma = step_size, gamma
        # linear LR warm-up over the first rounds (0: none, the reference's schedule), then StepLR
        self.warmup_rounds = int(warmup_rounds)
        self.dtype = 1 if dtype == "bf16" else 0
        self.eval_rows = eval_rows
        if allreduce_dtype not in ("fp32", "bf16"):
            raise ValueError("allreduce_dtype: fp32 | bf16")
        self.allreduce_dtype = allreduce_dtype
        f32 = dict(dtype=torch.float32, device=self.dev)
        flat = torch.as_tensor(init_flat(self.dims, seed), **f32)
        self.layout = param_layout(self.dims)
        self.params = flat
        self.grads = torch.zeros_like(flat)
        self.m_ = torch.zeros_like(flat)
        self.v_ = torch.zeros_like(flat)
        self.W = [flat[off:off + int(np.prod(s))].view(*s) for n_, s, off in self.layout[0::2]]
        self.b = [flat[off:off + int(np.prod(s))].view(*s) for n_, s, off in self.layout[1::2]]
        self.gW = [self.grads[off:off + int(np.prod(s))].view(*s) for n_, s, off in self.layout[0::2]]
        self.gb = [self.grads[off:off + int(np.prod(s))].view(*s) for n_, s, off in self.layout[1::2]]
        gdt = torch.bfloat16 if self.dtype else torch.float32
        dev = self.dev
        mb, dims = self.mb, self.dims
        self.Wq = [torch.empty(w.shape, dtype=gdt, device=dev) for w in self.W]
        # W^T copies: B operand of the NT dgrad GEMM (hidden layers that take the NT path)
        self.WqT = [torch.empty(w.shape[1], w.shape[0], dtype=gdt, device=dev) if self.dtype else None
                    for w in self.W]
        # activations / deltas of one micro-batch: row-major GEMM operands + transposed
        # (k = rows contiguous) copies for the NT weight-gradient GEMMs
        self.hq = [torch.empty(mb, d, dtype=gdt, device=dev) for d in dims[1:-1]]
        # (row stride ldt: 256 extra elements (FEDMI_WIDE_TPAD) break the power-of-two stride; the
        # weight-gradient GEMM reading them as its A operand runs ~4 % faster, profiles/wide_tpad_r2.log)
        self.ldt = mb + int(os.environ.get("FEDMI_WIDE_TPAD", "256"))
        assert self.ldt % 8 == 0
        self.hT = [torch.empty(d, self.ldt, dtype=gdt, device=dev) for d in dims[1:-1]]
        self.dzq = [torch.empty(mb, d, dtype=gdt, device=dev) for d in dims[1:]]
        self.dzT = [torch.empty(d, self.ldt, dtype=gdt, device=dev) for d in dims[1:-1]]
        self.xq = torch.empty(mb, dims[0], dtype=gdt, device=dev)
        self.scratch = torch.empty(mb * max(dims[1:]), **f32)  # fp32 epilogue target of the generic GEMM
        self.logits = torch.empty(mb, dims[-1], **f32)
        # split-K slabs of the two skinny weight gradients (layer 0: [H1][14], head: [C][H_last]),
        # whose 64x64 output tiles alone would leave all but ~64 CUs idle over a long contraction
        self.wg_splits = max(1, min(16, mb // 1024))
        self.wg_slab = torch.empty(self.wg_splits * max(dims[0] * dims[1], dims[-1] * dims[-2]), **f32)
        # bf16: the two skinny gradients run on a bandwidth-bound kernel instead (8 columns x C
        # accumulators per thread, up to 256 row splits, fixed-order slab reduction)
        self._skinny = (bool(self.dtype) and self.L >= 2 and dims[0] == 14 and dims[-1] == 2
                        and dims[1] % 8 == 0 and dims[-2] % 8 == 0)
        self.sk_splits = max(1, min(256, mb // 256))
        self.sk_slab = (torch.empty(self.sk_splits * max((dims[0] + 1) * dims[1], dims[-1] * dims[-2]), **f32)
                        if self._skinny else None)
        self.dz_out = torch.empty(mb, dims[-1], **f32)
        # bias gradients of the hidden layers: column sums of each dgrad's bf16 output, one row per
        # 128 output rows, written by the NT epilogue (NT_EPI_CSUM) and folded by colsum -- instead
        # of re-reading the whole transposed delta (rowsum_bf16)
        self.cs_slab = torch.empty((mb // 128) * max(dims[1:-1]), **f32) if len(dims) > 2 else None
        self._cs_layer: Optional[int] = None
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self.cm = torch.zeros(dims[-1] * dims[-1], dtype=torch.float32, device=dev)  # local confusion counts
        self.evaluated = False
        # Fused evaluation (one client: FedAvg is the identity, so the post-step local model IS the
        # next round's model): the local evaluation of round r is scored from round r+1's training
        # forward -- the same kernels on the same weights and rows, so bit-identical logits, one
        # forward pass fewer per round.  metrics() flushes a pending evaluation with its own
        # forward pass when it is asked for before the next round runs.
        self.fused_eval = (comm is None or self.world == 1) if fused_eval is None else bool(fused_eval)
        if self.fused_eval and self.world > 1:
            raise ValueError("fused_eval needs one client (with FedAvg the next forward sees the global model)")
        self._eval_pending = False
        self.round = 0
        self.stream = torch.cuda.Stream(device=dev)
        self.comm_stream = torch.cuda.Stream(device=dev)
        self.nt_calls = 0
        # transposed (k = rows) operands need 16-byte aligned rows of the micro-batch buffers
        self._t_ok = bool(self.dtype) and mb % 128 == 0
        self._bucket_ev: List[Optional[torch.cuda.Event]] = [None] * self.L  # pending FedAvg buckets
        # K-padded (to 64, zeros) operands so the layer-0 forward (K = 14 features) and the head's
        # dgrad (K = C classes) also run on the NT GEMM with fused epilogues + transposed outputs
        KP = 64
        self._pad = (self._t_ok and self.L >= 2 and dims[0] <= KP and dims[-1] <= KP
                     and self._nt_ok(mb, dims[1], KP) and self._nt_ok(mb, dims[-2], KP))
        if self._pad:
            self.xp = torch.empty(mb, KP, dtype=gdt, device=dev)        # bf16 X, zero-padded
            self.W0p = torch.empty(dims[1], KP, dtype=gdt, device=dev)   # bf16 W0, zero-padded
            self.dzp = torch.empty(mb, KP, dtype=gdt, device=dev)       # bf16 head delta, padded
            self.WhTp = torch.empty(dims[-2], KP, dtype=gdt, device=dev)  # bf16 head W^T, padded
            # logits head on the NT GEMM: classes zero-padded to N = 256 (fp32 logits, ld 256)
            self.Whp = torch.zeros(256, dims[-2], dtype=gdt, device=dev)
            self.bhp = torch.zeros(256, **f32)
            self.logits_p = torch.empty(mb, 256, **f32)
            self.logits = self.logits_p[:, :dims[-1]]
        # bf16 FedAvg buckets (allreduce_dtype="bf16"): half the bytes on the links.  What crosses
        # them is the scaled round DELTA n_i/N * (w_local - w_global_prev) in bf16 (summed by RCCL),
        # added back to the fp32 previous global model ``gprev``: the master weights stay fp32 and
        # bf16 rounds only the (small) update, so late-schedule Adam steps are not rounded away
        # (every rank starts from the same init, so gprev is the same on every rank)
        self.send_bf16 = (torch.empty(flat.numel(), dtype=torch.bfloat16, device=dev)
                          if allreduce_dtype == "bf16" and self.world > 1 else None)
        self.gprev = flat.clone() if self.send_bf16 is not None else None
        self._quantize()

    # ------------------------------------------------------------------
    def _s(self) -> int:
        return self.stream.cuda_stream

    def _quantize_layer(self, l: int, stream: torch.cuda.Stream):
        """GEMM operand copies of layer l (bf16 W and W^T, or fp32 W) on `stream`."""
        w, q = self.W[l], self.Wq[l]
        with torch.cuda.stream(stream):
            if self.dtype:
                self.m.to_bf16(w.data_ptr(), q.data_ptr(), w.numel(), stream.cuda_stream)
                if getattr(self, "_pad", False):
                    N, K = w.shape
                    if l == 0:
                        self.m.pad_bf16(w.data_ptr(), N, K, K, 1, self.W0p.data_ptr(), 64, stream.cuda_stream)
                    if l == self.L - 1:  # head W [C][H] -> W^T [H][64]; W rows 0..C-1 of [256][H]
                        self.m.pad_bf16(w.data_ptr(), K, N, 1, K, self.WhTp.data_ptr(), 64, stream.cuda_stream)
                        self.m.to_bf16(w.data_ptr(), self.Whp.data_ptr(), w.numel(), stream.cuda_stream)
                        self.bhp[:N].copy_(self.b[l])
                if self.WqT[l] is not None:
                    N, K = w.shape
                    self.m.transpose_bf16(w.data_ptr(), N, K, K, self.WqT[l].data_ptr(), N, stream.cuda_stream)
            else:
                q.copy_(w)

    def _quantize(self):
        for l in range(self.L):
            self._quantize_layer(l, self.stream)

    def _wait_bucket(self, l: int):
        """The compute stream's first use of layer l after FedAvg waits for its bucket only."""
        ev = self._bucket_ev[l]
        if ev is not None:
            self.stream.wait_event(ev)
            self._bucket_ev[l] = None

    def _csum_ok(self, rp: int, n: int) -> bool:
        """The dgrad of an [rp][n] delta can emit its column sums (256x256 NT loops)."""
        return self.cs_slab is not None and rp % 256 == 0 and n % 256 == 0

    def _rows_p(self, rows: int) -> Optional[int]:
        """Rows a micro-batch of `rows` runs as on the padded NT path, or None (generic path:
        a partial micro-batch pads only when every hidden layer runs on the NT GEMM, so every
        operand's padded rows are written by the same pass)."""
        if not self._pad:
            return None
        if rows % 128 == 0:
            return rows
        if not all(d % 128 == 0 for d in self.dims[1:-1]):
            return None
        g = 256 if self.mb % 256 == 0 else 128  # (256: the column-sum epilogue's tile)
        return min((rows + g - 1) // g * g, self.mb)

    @staticmethod
    def _nt_ok(M: int, N: int, K: int) -> bool:
        return M % 128 == 0 and N % 128 == 0 and K % 64 == 0

    def _forward(self, r0: int, rows: int, keep_t: bool = True):
        """Forward of one micro-batch.  Hidden layers write bf16 row-major (next layer's A
        operand, ReLU mask) and, when training, bf16 transposed (wgrad B operand)."""
        m, s, mb = self.m, self._s(), self.ldt
        x = self.X[r0:r0 + rows]
        # a partial last micro-batch runs as rp = roundup(rows, 128) rows on the NT GEMM: its
        # extra input rows are zeros, their deltas are zeroed before the backward pass (they add
        # exact zeros to every gradient), and the loss / confusion kernels see the real rows only
        rp = self._rows_p(rows)
        pad = rp is not None
        rp = rp if pad else rows
        if pad:
            m.pad_bf16(x.data_ptr(), rows, self.dims[0], self.dims[0], 1, self.xp.data_ptr(), 64, s)
            if rp > rows:
                self.xp[rows:rp].zero_()
            inp = self.xp
        elif self.dtype:
            m.to_bf16(x.data_ptr(), self.xq.data_ptr(), x.numel(), s)
            inp = self.xq
        else:
            inp = x
        for l in range(self.L):
            K, N = self.dims[l], self.dims[l + 1]
            self._wait_bucket(l)
            if l == 0 and pad:  # K = 14 zero-padded to 64: NT GEMM, bias + ReLU, bf16 + transposed out
                hT = self.hT[0].data_ptr() if (keep_t and self.L > 2) else 0
                m.gemm_nt(rp, N, 64, self.xp.data_ptr(), 64, self.W0p.data_ptr(), 64, 0, 0, self.hq[0].data_ptr(),
                          N, hT, mb, self.b[0].data_ptr(), 0, 0, 1, 1.0, 0.0, s)
                self.nt_calls += 1
                inp = self.hq[0]
                continue
            if l + 1 == self.L and pad:  # logits head, classes padded to 256: fp32 [rows][256]
                m.gemm_nt(rp, 256, K, inp.data_ptr(), K, self.Whp.data_ptr(), K, self.logits_p.data_ptr(), 256,
                          0, 0, 0, 0, self.bhp.data_ptr(), 0, 0, 0, 1.0, 0.0, s)
                self.nt_calls += 1
                break
            if l + 1 == self.L:  # logits head: fp32 output for the loss
                m.gemm(rows, N, K, inp.data_ptr(), K, 1, self.Wq[l].data_ptr(), K, 1, self.logits.data_ptr(),
                       self.logits.stride(0), 1, self.b[l].data_ptr(), 0, 0, 0, 1.0, 0.0, self.dtype, 1, 0, 0, s)
                break
            hq = self.hq[l]
            # the transposed copy feeds layer l+1's NT weight gradient: none for the last hidden
            # layer, whose consumer (the head's skinny / generic weight gradient) reads hq
            hT = self.hT[l].data_ptr() if (keep_t and self.dtype and l + 2 < self.L) else 0
            if self._t_ok and self._nt_ok(rp, N, K):
                m.gemm_nt(rp, N, K, inp.data_ptr(), K, self.Wq[l].data_ptr(), K, 0, 0, hq.data_ptr(), N, hT, mb,
                          self.b[l].data_ptr(), 0, 0, 1, 1.0, 0.0, s)
                self.nt_calls += 1
            else:
                m.gemm(rows, N, K, inp.data_ptr(), K, 1, self.Wq[l].data_ptr(), K, 1, self.scratch.data_ptr(), N, 2,
                       self.b[l].data_ptr(), 0, 0, 0, 1.0, 0.0, self.dtype, 1, 0,
                       hq.data_ptr() if self.dtype else 0, s)
                if self.dtype:
                    if hT:
                        m.transpose_bf16(self.scratch.data_ptr(), rows, N, N, hT, mb, s)
                else:
                    hq[:rows].copy_(self.scratch[:rows * N].view(rows, N))
            inp = hq

    def _wg_split(self, rows: int) -> int:
        """K-split count of a skinny weight gradient over `rows` contraction rows (>= 1024 rows per split)."""
        return max(1, min(self.wg_splits, rows // 1024))

    def _sk_split(self, rows: int) -> int:
        """Row splits of the skinny-gradient kernel (>= 256 rows per split)."""
        return max(1, min(self.sk_splits, rows // 256))

    def _backward(self, r0: int, rows: int, beta: float):
        m, s, mb, L = self.m, self._s(), self.ldt, self.L  # mb: row stride of the transposed operands
        C = self.dims[-1]
        # output layer (N = classes): tiny GEMMs on the generic kernel
        K = self.dims[L - 1]
        rp = self._rows_p(rows)  # (see _forward: padded rows carry zero deltas)
        pad = rp is not None
        rp = rp if pad else rows
        self._cs_layer = None
        dzo, ldo = self.dzq[L - 1], C
        if pad:
            dzo, ldo = self.dzp, 64
            m.pad_bf16(self.dz_out.data_ptr(), rows, C, C, 1, dzo.data_ptr(), 64, s)
            if rp > rows:
                dzo[rows:rp].zero_()
        elif self.dtype:
            m.to_bf16(self.dz_out.data_ptr(), dzo.data_ptr(), rows * C, s)
        else:
            dzo[:rows].copy_(self.dz_out[:rows])
        h_in = self.hq[L - 2] if L >= 2 else (self.xq if self.dtype else self.X[r0:r0 + rows])
        if self._skinny:
            m.skinny_wgrad(h_in.data_ptr(), K, K, dzo.data_ptr(), ldo, C, rows, 0, self._sk_split(rows),
                           self.sk_slab.data_ptr(), self.gW[L - 1].data_ptr(), beta, 0, s)
        else:
            m.gemm(C, K, rows, dzo.data_ptr(), ldo, 0, h_in.data_ptr(), K, 0, self.gW[L - 1].data_ptr(), K, 0, 0, 0, 0,
                   0, 1.0, beta, self.dtype, self._wg_split(rows), self.wg_slab.data_ptr(), 0, s)
        if self._skinny:  # head bias gradient, rows split 256 ways (the slab is free again here)
            m.colsum_split(self.dz_out.data_ptr(), rows, C, self._sk_split(rows), self.sk_slab.data_ptr(),
                           self.gb[L - 1].data_ptr(), beta, s)
        else:
            m.colsum(self.dz_out.data_ptr(), rows, C, C, self.gb[L - 1].data_ptr(), beta, s)
        if L >= 2 and pad:
            # dgrad into the last hidden layer: C classes zero-padded to K = 64 on the NT GEMM,
            # ReLU-masked, bf16 row-major + transposed outputs
            cs = self._csum_ok(rp, K)
            m.gemm_nt(rp, K, 64, dzo.data_ptr(), 64, self.WhTp.data_ptr(), 64, 0, 0, self.dzq[L - 2].data_ptr(), K,
                      self.dzT[L - 2].data_ptr(), mb, 0, self.hq[L - 2].data_ptr(), K, 0, 1.0, 0.0, s,
                      self.cs_slab.data_ptr() if cs else 0, K)
            self._cs_layer = L - 2 if cs else None
            self.nt_calls += 1
        elif L >= 2:
            # dgrad into the last hidden layer (K = C: bandwidth-bound), ReLU-masked
            m.gemm(rows, K, C, dzo.data_ptr(), C, 1, self.Wq[L - 1].data_ptr(), K, 0, self.scratch.data_ptr(), K, 3, 0,
                   self.hq[L - 2].data_ptr(), K, 1 if self.dtype else 0, 1.0, 0.0, self.dtype, 1, 0,
                   self.dzq[L - 2].data_ptr() if self.dtype else 0, s)
            if self.dtype:
                m.transpose_bf16(self.scratch.data_ptr(), rows, K, K, self.dzT[L - 2].data_ptr(), mb, s)
            else:
                self.dzq[L - 2][:rows].copy_(self.scratch[:rows * K].view(rows, K))
        # hidden layers, top down
        for l in range(L - 2, -1, -1):
            K, N = self.dims[l], self.dims[l + 1]
            dq = self.dzq[l]
            ldi = K
            if l == 0:
                inp = self.xq if self.dtype else self.X[r0:r0 + rows]
                if pad:
                    inp, ldi = self.xp, 64
            else:
                inp = self.hq[l - 1]
            # wgrad (+= over micro-batches): dW[N][K] = dZ^T . in;  bias: row sums of dZ^T
            if self._t_ok and l > 0 and self._nt_ok(N, K, rp):
                m.gemm_nt(N, K, rp, self.dzT[l].data_ptr(), mb, self.hT[l - 1].data_ptr(), mb,
                          self.gW[l].data_ptr(), K, 0, 0, 0, 0, 0, 0, 0, 0, 1.0, beta, s)
                self.nt_calls += 1
            elif l == 0 and self._skinny:
                # + layer 0's bias gradient (column sums of dZ0) from the same loads
                m.skinny_wgrad(dq.data_ptr(), N, N, inp.data_ptr(), ldi, K, rows, 1, self._sk_split(rows),
                               self.sk_slab.data_ptr(), self.gW[0].data_ptr(), beta, self.gb[0].data_ptr(), s)
            else:
                m.gemm(N, K, rows, dq.data_ptr(), N, 0, inp.data_ptr(), ldi, 0, self.gW[l].data_ptr(), K, 0, 0, 0, 0, 0,
                       1.0, beta, self.dtype, self._wg_split(rows) if l == 0 else 1, self.wg_slab.data_ptr(), 0, s)
            if l == 0 and self._skinny:
                pass  # bias gradient produced by the skinny weight-gradient kernel above
            elif self._cs_layer == l:  # column sums from the dgrad epilogue that produced dZ_l
                m.colsum(self.cs_slab.data_ptr(), rp // 128, N, N, self.gb[l].data_ptr(), beta, s)
            elif self.dtype and rows % 8 == 0 and mb % 8 == 0:
                m.rowsum_bf16(self.dzT[l].data_ptr(), N, rows, mb, self.gb[l].data_ptr(), beta, s)
            else:
                dzf = dq[:rows].float()
                m.colsum(dzf.data_ptr(), rows, N, N, self.gb[l].data_ptr(), beta, s)
            if l == 0:
                break
            # dgrad: dIn[rows][K] = dZ . W, masked by in > 0
            if self._t_ok and self._nt_ok(rp, K, N):
                # dZ_{l-1}^T feeds the NT weight gradient and row sums of layer l-1; layer 0's
                # skinny kernel reads dZ_0 row-major (weights and bias), so no transposed copy
                dT = 0 if (l == 1 and self._skinny) else self.dzT[l - 1].data_ptr()
                cs = dT != 0 and self._csum_ok(rp, K)  # (layer 0 + skinny: its kernel sums the bias)
                m.gemm_nt(rp, K, N, dq.data_ptr(), N, self.WqT[l].data_ptr(), N, 0, 0, self.dzq[l - 1].data_ptr(), K,
                          dT, mb, 0, self.hq[l - 1].data_ptr(), K, 0, 1.0, 0.0, s,
                          self.cs_slab.data_ptr() if cs else 0, K)
                self._cs_layer = l - 1 if cs else None
                self.nt_calls += 1
            else:
                m.gemm(rows, K, N, dq.data_ptr(), N, 1, self.Wq[l].data_ptr(), K, 0, self.scratch.data_ptr(), K, 3, 0,
                       self.hq[l - 1].data_ptr(), K, 1 if self.dtype else 0, 1.0, 0.0, self.dtype, 1, 0,
                       self.dzq[l - 1].data_ptr() if self.dtype else 0, s)
                if self.dtype:
                    m.transpose_bf16(self.scratch.data_ptr(), rows, K, K, self.dzT[l - 1].data_ptr(), mb, s)
                else:
                    self.dzq[l - 1][:rows].copy_(self.scratch[:rows * K].view(rows, K))

    def local_step(self):
        """One full-batch Adam step over the whole shard (micro-batched accumulation)."""
        self._local_quantized = False
        C = self.dims[-1]
        s = self._s()
        fuse = self._eval_pending  # this forward also scores the previous round's evaluation
        self._eval_pending = False
        with torch.cuda.stream(self.stream):
            self.loss_acc.zero_()
            if fuse:
                self.cm.zero_()
            for r0 in range(0, self.n, self.mb):
                rows = min(self.mb, self.n - r0)
                self._forward(r0, rows)
                if fuse:
                    self.m.logits_confusion(self.logits.data_ptr(), self.logits.stride(0), self.y[r0:].data_ptr(),
                                            rows, C, self.cm.data_ptr(), s)
                # loss head: softmax CE, dZ = (p - onehot) / n (full-batch mean)
                self.m.xent(self.logits.data_ptr(), self.logits.stride(0), self.y[r0:].data_ptr(), rows, C, 0,
                            1.0 / self.n,
                            self.dz_out.data_ptr(), C, self.loss_acc.data_ptr(), s)
                self._backward(r0, rows, 0.0 if r0 == 0 else 1.0)
            # torch Adam + StepLR (scalars computed on host: the schedule is known)
            t = self.round + 1
            lr = self.lr * self.gamma ** (self.round // self.step_size)
            if self.warmup_rounds > 0:
                lr *= min(1.0, (self.round + 1) / self.warmup_rounds)
            self.m.adam_flat(self.params.data_ptr(), self.m_.data_ptr(), self.v_.data_ptr(), self.grads.data_ptr(),
                             self.params.numel(), lr, self.betas[0], self.betas[1], self.eps, t, s)

    def aggregate(self):
        """Sample-size-weighted FedAvg: per layer bucket [W_l | b_l], in forward order on the
        comm stream: one all-reduce of n_i/N * bucket (fp32 buckets, or bf16 buckets filled by
        one fused scale + round pass), re-quantise, record the bucket's event.  The compute
        stream does not wait here: its next use of layer l waits on event l."""
        if self.world == 1:
            # FedAvg of one client is the identity: its operand copies are the local model's
            if not getattr(self, "_local_quantized", False):
                self._quantize()
            self._local_quantized = False
            return
        self.comm_stream.wait_stream(self.stream)  # the Adam step (and evaluation) are done
        for l, ((name, shape, off), (bn, bs, boff)) in enumerate(zip(self.layout[0::2], self.layout[1::2])):
            end = boff + int(np.prod(bs))
            with torch.cuda.stream(self.comm_stream):
                seg = self.params[off:end]
                if self.send_bf16 is None:
                    self.comm.allreduce_(seg, scale=self.agg)
                else:
                    # bf16 delta on the wire, fp32 master kept: one pass fills the bucket with
                    # bf16(n_i/N * (w - gprev)), one adds the reduced deltas to gprev (and w)
                    bseg, gseg = self.send_bf16[off:end], self.gprev[off:end]
                    cs = self.comm_stream.cuda_stream
                    self.m.fedavg_delta_bf16(seg.data_ptr(), gseg.data_ptr(), bseg.data_ptr(), seg.numel(), self.agg,
                                             cs)
                    self.comm.allreduce_(bseg)
                    self.m.fedavg_apply_delta(seg.data_ptr(), gseg.data_ptr(), bseg.data_ptr(), seg.numel(), cs)
            self._quantize_layer(l, self.comm_stream)
            ev = torch.cuda.Event()
            ev.record(self.comm_stream)
            self._bucket_ev[l] = ev

    def sync(self):
        """Join every pending FedAvg bucket into the compute stream."""
        for l in range(self.L):
            self._wait_bucket(l)

    def evaluate_shard(self) -> None:
        """Local evaluation of the post-step local model on the WHOLE shard (C:148, C:75-91):
        micro-batched forward passes, argmax + confusion counts on the device into
        ``self.cm`` (no host synchronisation; :meth:`metrics` reads them).  With fused evaluation
        the counts come from the next round's training forward (or :meth:`metrics`' flush)."""
        if self.fused_eval:
            self._eval_pending = True
            self.evaluated = True
            return
        self._evaluate_now()

    def _evaluate_now(self) -> None:
        self._eval_pending = False
        C = self.dims[-1]
        self._quantize()   # the GEMM operand copies of the post-step local weights
        self._local_quantized = True
        with torch.cuda.stream(self.stream):
            self.cm.zero_()
            for r0 in range(0, self.n, self.mb):
                rows = min(self.mb, self.n - r0)
                self._forward(r0, rows, keep_t=False)
                self.m.logits_confusion(self.logits.data_ptr(), self.logits.stride(0), self.y[r0:].data_ptr(), rows,
                                        C, self.cm.data_ptr(), self._s())
        self.evaluated = True

    def metrics(self) -> dict:
        """Accuracy / weighted precision, recall, F1 of the last :meth:`evaluate_shard`."""
        from .metrics import metrics_from_confusion
        if self._eval_pending:  # nobody has run the forward that would score it: run it now
            self._evaluate_now()
        self.stream.synchronize()
        C = self.dims[-1]
        return metrics_from_confusion(self.cm.cpu().numpy().reshape(C, C).astype(np.int64))

    def evaluate(self) -> float:
        self.evaluate_shard()
        return float(self.metrics()["accuracy"])

    def run_round(self, evaluate: bool = True) -> None:
        """One federated round as the reference runs it (C:145-198): local step, local evaluation
        of the post-step model on the shard (device-side, no host sync), FedAvg buckets."""
        self.local_step()
        if evaluate:
            self.evaluate_shard()
        self.aggregate()
        self.round += 1

    def loss(self) -> float:
        self.sync()
        self.stream.synchronize()
        return float(self.loss_acc.item()) / self.n

    @property
    def flops_per_round(self) -> float:
        """FLOPs a round executes: training (forward + backward, 6 n MACs) plus the local
        evaluation forward (2 n MACs) unless it is fused into the next round's training forward."""
        macs = sum(a * b for a, b in zip(self.dims[:-1], self.dims[1:]))
        return (6.0 + (2.0 if self.evaluated and not self.fused_eval else 0.0)) * self.n * macs


def run_wide_fedavg(comm, dims: Sequence[int], rows_per_client: int, rounds: int, micro_batch: int = 131072,
                    dtype: str = "bf16", lr: float = WIDE_LR, eval_every: int = 0, seed: int = 7,
                    verbose: bool = True, allreduce_dtype: str = "fp32", warmup_rounds: int = 0) -> dict:
    """BASELINE config 3 driver: every rank is one client holding ``rows_per_client``
    synthetic income-shaped rows generated on its GPU, trains the wide MLP ``dims`` with
    full-batch (micro-batched) Adam steps and averages per layer bucket every round.
    Returns the per-round loss history, evaluation accuracies and timings."""
    import time

    from ..data.synthetic import device_shard
    dev = comm.device if comm is not None else torch.device("cuda", torch.cuda.current_device())
    rank = comm.rank if comm is not None else 0
    world = comm.size if comm is not None else 1
    X, y = device_shard(rows_per_client, rank, dev, seed=seed)
    c = WideClient(X, y, dims, comm=comm if world > 1 else None, n_total=rows_per_client * world,
                   micro_batch=micro_batch, lr=lr, dtype=dtype, seed=0, allreduce_dtype=allreduce_dtype,
                   warmup_rounds=warmup_rounds)
    losses, accs, times = [], [], []
    for r in range(rounds):
        t0 = time.perf_counter()
        ev = bool(eval_every) and (r + 1) % eval_every == 0
        c.run_round(evaluate=ev)
        loss = c.loss()          # joins the round (and its FedAvg buckets)
        acc = c.metrics()["accuracy"] if ev else None
        times.append(time.perf_counter() - t0)
        losses.append(loss)
        if acc is not None:
            accs.append((r + 1, acc))
        if verbose and rank == 0:
            msg = f"Round {r + 1}: loss {loss:.5f}, {times[-1] * 1e3:.1f} ms"
            if acc is not None:
                msg += f", local accuracy {acc:.4f}"
            print(msg, flush=True)
    steady = times[1:] or times
    dt = float(np.median(steady))
    c.sync()
    from ..parallel.consistency import check_replicas
    replicas_ok = check_replicas(comm, [c.params]) if world > 1 else True
    return {"loss": losses, "accuracy": accs, "round_s": times, "median_round_s": dt,
            "replicas_consistent": replicas_ok,
            "tflops_per_client": c.flops_per_round / dt / 1e12,
            "samples_per_s_per_client": rows_per_client / dt}


def save_wide(path: str, client: WideClient) -> None:
    """Wide-client checkpoint (rank 0 writes the global weights, every rank its Adam state), as
    a round-tagged set (fedmi/ckpt/checkpoint.py ``tagged``): ``weights.r<R>.safetensors`` under the
    reference's ``model.{2i}.weight`` [out, in] / ``.bias`` keys (C:93-94),
    ``client{r}.r<R>.safetensors`` with the flat fp32 Adam moments, and -- last, after a barrier --
    ``wide_meta.json`` with the dims, the round (= StepLR epoch and Adam step; every wide client
    trains every round) and the set's file names.  A pending fused evaluation is scored first, so
    :meth:`WideClient.metrics` after the save reports the round it was requested for."""
    import os
    from ..ckpt.checkpoint import _atomic, _prune, _publish_meta, save_weights, tagged
    from ..models.mlp import flat_to_dict
    from safetensors.numpy import save_file
    if client._eval_pending:
        client._evaluate_now()
    client.sync()
    client.stream.synchronize()
    rank = client.comm.rank if client.comm is not None else 0
    multi = client.comm is not None and client.world > 1
    R = int(client.round)
    os.makedirs(path, exist_ok=True)
    m_, v_ = client.m_.cpu().numpy(), client.v_.cpu().numpy()
    cname = f"client{rank}.safetensors"
    _atomic(os.path.join(path, tagged(cname, R)),
            lambda tmp: save_file({"exp_avg": m_, "exp_avg_sq": v_}, tmp, metadata={"round": str(R)}))
    if rank == 0:
        w = flat_to_dict(client.params.cpu().numpy(), client.dims)
        _atomic(os.path.join(path, tagged("weights.safetensors", R)), lambda tmp: save_weights(tmp, w, R))
    if multi:
        client.comm.Barrier()
    if rank == 0:
        _publish_meta(path, {"format": "fedmi-wide-ckpt-2", "dims": client.dims, "round": R,
                             "files": {"weights": tagged("weights.safetensors", R),
                                       "client": tagged("client{rank}.safetensors", R)},
                             "world": client.world, "lr": client.lr, "step_size": client.step_size,
                             "gamma": client.gamma}, name="wide_meta.json")
    if multi:
        client.comm.Barrier()
    _prune(path, cname, R)
    if rank == 0:
        _prune(path, "weights.safetensors", R)


def load_wide(path: str, client: WideClient) -> int:
    """Restore :func:`save_wide` into a client of the same dims / client count; returns the round.
    A pending fused evaluation of the client's current model is scored before it is replaced."""
    import json
    import os
    from ..ckpt.checkpoint import _check_round, load_weights
    from ..models.mlp import dict_to_flat
    from safetensors.numpy import load_file
    with open(os.path.join(path, "wide_meta.json")) as f:
        meta = json.load(f)
    fmt = meta.get("format")
    if fmt not in ("fedmi-wide-ckpt-1", "fedmi-wide-ckpt-2") or list(meta["dims"]) != client.dims:
        raise ValueError(f"{path}: not a wide checkpoint for dims {client.dims}")
    if int(meta["world"]) != client.world:
        raise ValueError(f"{path}: saved with {meta['world']} clients, this run has {client.world}")
    # the optimizer schedule is part of the state: resuming a run saved at another lr / StepLR
    # (e.g. under the reference's 0.004 before WIDE_LR became the default) must not silently
    # continue at a different rate
    for key, have in (("lr", client.lr), ("step_size", client.step_size), ("gamma", client.gamma)):
        if key in meta and float(meta[key]) != float(have):
            raise ValueError(f"{path}: saved with {key}={meta[key]}, this client has {key}={have}; "
                             f"construct the client with {key}={meta[key]} to resume")
    R = int(meta["round"]) if fmt == "fedmi-wide-ckpt-2" else None
    files = meta.get("files", {"weights": "weights.safetensors", "client": "client{rank}.safetensors"})
    rank = client.comm.rank if client.comm is not None else 0
    flat = dict_to_flat(load_weights(os.path.join(path, files["weights"]), expect_round=R), client.dims)
    cp = os.path.join(path, files["client"].format(rank=rank))
    _check_round(cp, R)
    st = load_file(cp)
    if client._eval_pending:
        client._evaluate_now()
    client.sync()
    with torch.cuda.stream(client.stream):
        client.params.copy_(torch.as_tensor(flat, device=client.dev))
        client.m_.copy_(torch.as_tensor(st["exp_avg"], device=client.dev))
        client.v_.copy_(torch.as_tensor(st["exp_avg_sq"], device=client.dev))
        if client.gprev is not None:
            client.gprev.copy_(client.params)
    client._quantize()
    client.stream.synchronize()
    client.round = int(meta["round"])
    return client.round
