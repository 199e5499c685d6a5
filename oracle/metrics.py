"""ORACLE (test infrastructure only) -- the reference's PSNR definition, restated in numpy.

uint8 conversion: ``(x * 0.5 + 0.5).clamp(0, 1)`` then ``(v * 255).astype(np.uint8)`` (truncation),
``/root/reference/hvae_training.py:368-388``; PSNR = 10 log10(255^2 / MSE) in float64 as in
skimage 0.18 ``metrics/simple_metrics.py:108-160`` (data_range 255 for uint8; read as text only).
"""
from __future__ import annotations

import numpy as np
import torch


def to_uint8(img: torch.Tensor) -> np.ndarray:
    """NCHW float in [-1, 1] -> NHWC uint8 exactly as the reference converts (float32 math, truncation)."""
    v = (img.detach().float().cpu().permute(0, 2, 3, 1) * 0.5 + 0.5).clamp(0, 1).numpy()
    return (v * 255).astype(np.uint8)


def sse_uint8(a: torch.Tensor, b: torch.Tensor) -> np.ndarray:
    """Per-image sum of squared uint8 differences (float64)."""
    ua, ub = to_uint8(a).astype(np.float64), to_uint8(b).astype(np.float64)
    return ((ua - ub) ** 2).reshape(ua.shape[0], -1).sum(1)


def psnr(a: torch.Tensor, b: torch.Tensor) -> float:
    """PSNR over the whole batch (one MSE over every pixel), data_range 255."""
    ua, ub = to_uint8(a).astype(np.float64), to_uint8(b).astype(np.float64)
    mse = np.mean((ua - ub) ** 2)
    return float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))
