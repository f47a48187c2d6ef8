"""MLP classifier with the reference's module layout and a flat parameter buffer.

``MLPModel(input_size, hidden_sizes, output_size)`` builds the same
``Sequential([Linear, ReLU] * len(hidden) + [Linear])`` as the reference
(``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:12-25``), so
``named_parameters()`` keys are ``model.{2i}.weight`` / ``model.{2i}.bias`` and
checkpoints interchange with the reference's ``get_weights()`` dict (C:93-94).

MI355X-first difference: every parameter is a *view* into one contiguous fp32 buffer
(``model.flat``) in named-parameter order.  That buffer is exactly what the round engine
trains, what the FedAvg all-reduce reduces in place, and what a checkpoint stores -- no
per-tensor D2H/H2D copies (reference C:94, C:99) and no pack/unpack around the
collective.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn


def layer_dims(input_size: int, hidden_sizes: Sequence[int], output_size: int) -> List[int]:
    return [int(input_size), *[int(h) for h in hidden_sizes], int(output_size)]


def param_layout(dims: Sequence[int]) -> List[Tuple[str, Tuple[int, ...], int]]:
    """[(name, shape, offset)] in named_parameters() order, dense (no padding)."""
    out, off = [], 0
    for l in range(len(dims) - 1):
        wshape = (dims[l + 1], dims[l])
        out.append((f"model.{2 * l}.weight", wshape, off))
        off += wshape[0] * wshape[1]
        out.append((f"model.{2 * l}.bias", (dims[l + 1],), off))
        off += dims[l + 1]
    return out


def param_count(dims: Sequence[int]) -> int:
    return sum(dims[l] * dims[l + 1] + dims[l + 1] for l in range(len(dims) - 1))


class MLPModel(nn.Module):
    """Reference-compatible MLP (C:12-25) whose parameters live in ``self.flat``."""

    def __init__(self, input_size: int, hidden_sizes: Sequence[int], output_size: int,
                 device=None, dtype=torch.float32):
        super().__init__()
        layers: List[nn.Module] = []
        in_size = input_size
        for h in hidden_sizes:
            layers.append(nn.Linear(in_size, h))
            layers.append(nn.ReLU())
            in_size = h
        layers.append(nn.Linear(in_size, output_size))
        self.model = nn.Sequential(*layers)
        self.dims = layer_dims(input_size, hidden_sizes, output_size)
        self.layout = param_layout(self.dims)
        self.flat = torch.empty(param_count(self.dims), dtype=dtype, device=device)
        with torch.no_grad():
            for (name, shape, off), p in zip(self.layout, self.model.parameters()):
                n = int(np.prod(shape))
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view(shape)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.model(x)

    def rebind(self, flat: torch.Tensor) -> None:
        """Point every parameter at ``flat`` (same layout) without copying."""
        assert flat.numel() == self.flat.numel()
        self.flat = flat
        for (name, shape, off), p in zip(self.layout, self.model.parameters()):
            n = int(np.prod(shape))
            p.data = flat[off:off + n].view(shape)


def flat_to_dict(flat, dims: Sequence[int]) -> Dict[str, np.ndarray]:
    """Flat buffer -> reference ``get_weights()`` dict (C:93-94): fp32 numpy, [out,in]."""
    if isinstance(flat, torch.Tensor):
        flat = flat.detach().float().cpu().numpy()
    flat = np.asarray(flat, dtype=np.float32)
    return {name: flat[off:off + int(np.prod(shape))].reshape(shape).copy()
            for name, shape, off in param_layout(dims)}


def dict_to_flat(weights: Dict[str, np.ndarray], dims: Sequence[int]) -> np.ndarray:
    out = np.empty(param_count(dims), dtype=np.float32)
    for name, shape, off in param_layout(dims):
        w = np.asarray(weights[name], dtype=np.float32)
        if tuple(w.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {w.shape} != {shape}")
        out[off:off + w.size] = w.reshape(-1)
    return out


def sklearn_to_flat(coefs: Sequence[np.ndarray], intercepts: Sequence[np.ndarray]) -> np.ndarray:
    """sklearn ``coefs_ + intercepts_`` (coefs [in,out], S:26/S:109) -> flat buffer."""
    parts = []
    for W, b in zip(coefs, intercepts):
        parts.append(np.asarray(W, dtype=np.float32).T.reshape(-1))
        parts.append(np.asarray(b, dtype=np.float32).reshape(-1))
    return np.concatenate(parts)


def flat_to_sklearn(flat, dims: Sequence[int]):
    d = flat_to_dict(flat, dims)
    L = len(dims) - 1
    coefs = [d[f"model.{2 * l}.weight"].T.astype(np.float64) for l in range(L)]
    inter = [d[f"model.{2 * l}.bias"].astype(np.float64) for l in range(L)]
    return coefs, inter


def _ldw(K: int) -> int:
    return ((K + 15) & ~15) + 4


def _r16(n: int) -> int:
    return (n + 15) & ~15


def image_layout(dims: Sequence[int]):
    """Offsets of the padded device parameter image (fedmi/ops/csrc/fl_common.h): per layer
    W_l as [roundup16(N)][roundup16(K)+4] then b_l as [roundup16(N)], zero padded; W_l[n][k] at
    column k ^ swz(n) of row n (_image_cols)."""
    iw, ib, off = [], [], 0
    for l in range(len(dims) - 1):
        K, N = dims[l], dims[l + 1]
        iw.append(off)
        off += _r16(N) * _ldw(K)
        ib.append(off)
        off += _r16(N)
    return iw, ib, (off + 3) & ~3


def _image_cols(N: int, K: int) -> np.ndarray:
    """[N, K] image column of W[n][k]: k ^ swz(n), swz(n) = 4 for n mod 16 in [4, 12) (the fp32
    kernels' LDS chunk swizzle, fl_common.h fl_swz)."""
    n = np.arange(N)[:, None]
    return np.arange(K)[None, :] ^ (((n + 4) & 8) >> 1)


def dense_to_image(flat: np.ndarray, dims: Sequence[int]) -> np.ndarray:
    iw, ib, total = image_layout(dims)
    img = np.zeros(total, dtype=np.float32)
    flat = np.asarray(flat, dtype=np.float32)
    for l, (name, shape, off) in enumerate(param_layout(dims)[0::2]):
        N, K = shape
        W = flat[off:off + N * K].reshape(N, K)
        bo = off + N * K
        ldw = _ldw(K)
        rows = img[iw[l]:iw[l] + _r16(N) * ldw].reshape(_r16(N), ldw)
        rows[np.arange(N)[:, None], _image_cols(N, K)] = W
        img[ib[l]:ib[l] + N] = flat[bo:bo + N]
    return img


def image_to_dense(img: np.ndarray, dims: Sequence[int]) -> np.ndarray:
    iw, ib, total = image_layout(dims)
    img = np.asarray(img, dtype=np.float32)
    out = np.empty(param_count(dims), dtype=np.float32)
    for l, (name, shape, off) in enumerate(param_layout(dims)[0::2]):
        N, K = shape
        ldw = _ldw(K)
        rows = img[iw[l]:iw[l] + _r16(N) * ldw].reshape(_r16(N), ldw)
        out[off:off + N * K] = rows[np.arange(N)[:, None], _image_cols(N, K)].reshape(-1)
        out[off + N * K:off + N * K + N] = img[ib[l]:ib[l] + N]
    return out


def init_flat(dims: Sequence[int], seed: int) -> np.ndarray:
    """torch ``nn.Linear`` default init (kaiming-uniform a=sqrt(5) => U(-1/sqrt(fan_in),
    1/sqrt(fan_in)) for weight and bias), drawn from a seeded generator."""
    g = torch.Generator().manual_seed(int(seed))
    parts = []
    for l in range(len(dims) - 1):
        bound = 1.0 / np.sqrt(dims[l])
        w = (torch.rand(dims[l + 1], dims[l], generator=g, dtype=torch.float64) * 2 - 1) * bound
        b = (torch.rand(dims[l + 1], generator=g, dtype=torch.float64) * 2 - 1) * bound
        parts += [w.float().reshape(-1), b.float()]
    return torch.cat(parts).numpy()
