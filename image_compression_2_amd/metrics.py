"""PSNR exactly as the reference evaluates it (hvae_training.py:368-395): uint8 conversion
trunc(clamp(x*0.5+0.5, 0, 1)*255), then 10*log10(255^2 / MSE) in float64 (skimage 0.18 definition).
The per-image squared-error sums run in one HIP kernel (ic2_uint8_sse); the log is host arithmetic."""
from __future__ import annotations

import math

import torch

from . import _native as nv


def uint8_sse(a, b):
    """Per-image sum of squared uint8 differences -> float64 [N] (device)."""
    a = a.to(torch.float32).contiguous()
    b = b.to(torch.float32).contiguous()
    nv.require_gpu(a, b)
    assert a.shape == b.shape
    n = a.shape[0]
    out = torch.empty(n, dtype=torch.float64, device=a.device)
    scratch = torch.empty(int(nv.query("ic2_uint8_sse_scratch_doubles", n)), dtype=torch.float64, device=a.device)
    nv.call("ic2_uint8_sse", nv.ptr(a), nv.ptr(b), n, a[0].numel(), nv.ptr(out), nv.ptr(scratch), nv.stream_of(a))
    return out


def psnr_from_sums(sse_total, n_values):
    mse = float(sse_total) / float(n_values)
    return float("inf") if mse == 0 else 10.0 * math.log10(255.0 ** 2 / mse)


def psnr(a, b):
    sse = uint8_sse(a, b)
    return psnr_from_sums(sse.sum().item(), a.numel())
