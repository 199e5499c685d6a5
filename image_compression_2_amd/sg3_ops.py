"""Op-level drop-ins for StyleGAN3's ``torch_utils.ops`` (bias_act, upfirdn2d, filtered_lrelu).

Same names, argument meaning and shape rules as NVlabs/stylegan3 [SG3-public; the reference calls them
through ``G.synthesis`` at /root/reference/stylegan3_hvae_full.py:274,329].  Every op runs a
hand-written HIP kernel from libic2ops.so; ROCm tensors only (CPU tensors raise -- no fallback).
``impl`` is accepted for signature compatibility and ignored.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as nv


def _parse_scaling(s):
    if isinstance(s, int):
        s = [s, s]
    sx, sy = s
    assert sx >= 1 and sy >= 1
    return int(sx), int(sy)


def _parse_padding(padding):
    if isinstance(padding, int):
        padding = [padding, padding]
    if len(padding) == 2:
        px, py = padding
        padding = [px, px, py, py]
    return [int(p) for p in padding]


def _get_filter_size(f):
    if f is None:
        return 1, 1
    assert f.ndim in (1, 2)
    return int(f.shape[-1]), int(f.shape[0])


_ACT = {"linear": (nv.ACT_LINEAR, 0.0, 1.0), "lrelu": (nv.ACT_LRELU, 0.2, float(np.sqrt(2)))}


def bias_act(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None, impl="cuda"):
    """x + b (broadcast along ``dim``) -> act -> * gain -> clamp."""
    if act not in _ACT:
        raise NotImplementedError(f"activation {act!r} (only 'linear' and 'lrelu' are on the path)")
    x = x.contiguous()
    nv.require_gpu(x)
    code, def_alpha, def_gain = _ACT[act]
    alpha = float(alpha if alpha is not None else def_alpha)
    gain = float(gain if gain is not None else def_gain)
    clamp = float(clamp if clamp is not None else -1)
    if b is not None:
        b = b.to(torch.float32).contiguous()
        nv.require_gpu(b)
        assert b.ndim == 1 and b.shape[0] == x.shape[dim]
    outer = int(np.prod(x.shape[:dim])) if dim > 0 else 1
    inner = int(np.prod(x.shape[dim + 1:])) if dim + 1 < x.ndim else 1
    y = torch.empty_like(x)
    nv.call("ic2_bias_act", nv.ptr(x), nv.ptr(b), nv.ptr(y), nv.dtype_code(x.dtype), outer, int(x.shape[dim]), inner,
            code, alpha, gain, clamp, nv.stream_of(x))
    return y


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1, impl="cuda"):
    """Zero-insert upsample -> pad/crop -> FIR -> downsample, NCHW."""
    x = x.contiguous()
    nv.require_gpu(x)
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    n, c, h, w = x.shape
    if f is not None:
        f = f.to(device=x.device, dtype=torch.float32).contiguous()
        fw, fh = _get_filter_size(f)
        f_ndim = f.ndim
    else:
        fw, fh, f_ndim = 1, 1, 2
    assert w * upx + px0 + px1 >= fw and h * upy + py0 + py1 >= fh, "upsampled buffer smaller than the filter"
    ow = (w * upx + px0 + px1 - fw + downx) // downx
    oh = (h * upy + py0 + py1 - fh + downy) // downy
    y = torch.empty([n, c, oh, ow], dtype=x.dtype, device=x.device)
    nv.call("ic2_upfirdn2d", nv.ptr(x), nv.ptr(y), nv.dtype_code(x.dtype), n * c, h, w, oh, ow, nv.ptr(f), f_ndim,
            fh if f_ndim == 2 else 0, fw, upx, upy, downx, downy, px0, px1, py0, py1, int(bool(flip_filter)),
            float(gain), nv.stream_of(x))
    return y


def _host_taps(f):
    """1-D filter -> (ctypes float array, taps) in host memory (the fused kernel takes taps by value)."""
    if f is None:
        return None, 1
    a = f.detach().to(torch.float32).cpu().numpy() if isinstance(f, torch.Tensor) else np.asarray(f, np.float32)
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a.ctypes.data_as(ctypes.c_void_p), int(a.shape[0]), a


def filtered_lrelu(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=np.sqrt(2), slope=0.2, clamp=None,
                   flip_filter=False, impl="cuda"):
    """Fused bias -> upsample -> FIR -> lrelu*gain -> clamp -> FIR -> downsample (one HIP launch when the
    (up, down, taps) combination has a fused instance; otherwise the same four steps as separate HIP
    kernels, exactly the reference composition)."""
    x = x.contiguous()
    nv.require_gpu(x)
    px0, px1, py0, py1 = _parse_padding(padding)
    fu_w, fu_h = _get_filter_size(fu)
    fd_w, fd_h = _get_filter_size(fd)
    n, c, h, w = x.shape
    ow = (w * up + (px0 + px1) - (fu_w - 1) - (fd_w - 1) + (down - 1)) // down
    oh = (h * up + (py0 + py1) - (fu_h - 1) - (fd_h - 1) + (down - 1)) // down
    separable = (fu is None or fu.ndim == 1) and (fd is None or fd.ndim == 1)
    if b is not None:
        b = b.to(torch.float32).contiguous()
        nv.require_gpu(b)
    if separable and x.dtype in (torch.float32, torch.bfloat16):
        gu = _host_taps(fu)
        gd = _host_taps(fd)
        y = torch.empty([n, c, oh, ow], dtype=x.dtype, device=x.device)
        lib = nv.load()
        rc = lib.ic2_filtered_lrelu(nv.ptr(x), nv.ptr(y), nv.dtype_code(x.dtype), n, c, h, w, oh, ow, gu[0], gu[1], gd[0],
                                    gd[1], nv.ptr(b), int(up), int(down), px0, px1, py0, py1, float(gain), float(slope),
                                    float(clamp if clamp is not None else -1), int(bool(flip_filter)), nv.stream_of(x))
        if rc == 0:
            return y
        if rc != 2:  # anything but IC2_E_UNSUPPORTED is an error
            raise RuntimeError(f"ic2_filtered_lrelu failed: {lib.ic2_last_error().decode()}")
    # composition of the reference's four steps, each a HIP kernel
    t = bias_act(x, b)
    t = upfirdn2d(t, fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    t = bias_act(t, act="lrelu", alpha=slope, gain=gain, clamp=clamp)
    return upfirdn2d(t, fd, down=down, flip_filter=flip_filter)
