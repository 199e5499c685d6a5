"""Op-level drop-ins for StyleGAN3's ``torch_utils.ops`` (bias_act, upfirdn2d, filtered_lrelu).

Same names, argument meaning and shape rules as NVlabs/stylegan3 [SG3-public; the reference calls them
through ``G.synthesis`` at /root/reference/stylegan3_hvae_full.py:274,329].  Every op runs a
hand-written HIP kernel from libic2ops.so; ROCm tensors only (CPU tensors raise -- no fallback).
``impl`` is accepted for signature compatibility and ignored.

All three are differentiable like SG3's (its ops carry custom autograd Functions): the backward passes are
HIP kernels as well -- upfirdn2d's gradient is upfirdn2d with up/down swapped, the padding from
``upfirdn2d_adjoint_padding`` and the filter flipped; bias_act's is an elementwise mask of the saved output;
filtered_lrelu's recomputes the upsampled pre-activation and chains the two adjoint FIRs.  Filters are
constants (no gradient), as in SG3's synthesis layers.
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


def _bias_act_fwd(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None):
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


def _upfirdn2d_fwd(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
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


def _filtered_lrelu_fwd(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=np.sqrt(2), slope=0.2, clamp=None,
                        flip_filter=False):
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
    t = _bias_act_fwd(x, b)
    t = _upfirdn2d_fwd(t, fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    t = _bias_act_fwd(t, act="lrelu", alpha=slope, gain=gain, clamp=clamp)
    return _upfirdn2d_fwd(t, fd, down=down, flip_filter=flip_filter)


# ------------------------------------------------------------------------------------------------
# gradients
# ------------------------------------------------------------------------------------------------
def upfirdn2d_adjoint_padding(in_hw, out_hw, f, up=1, down=1, padding=0):
    """Padding of the adjoint upfirdn2d: for y = upfirdn2d(x, f, up, down, padding, flip, gain) [in_hw ->
    out_hw], dL/dx = upfirdn2d(dL/dy, f, up=down, down=up, padding=<this>, flip_filter=not flip, gain) --
    zero insertion and decimation swap, the FIR correlates instead of convolving, and the crop becomes a pad
    (SG3's upfirdn2d backward)."""
    ih, iw = in_hw
    oh, ow = out_hw
    fw, fh = _get_filter_size(f)
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    return [fw - px0 - 1, iw * upx - ow * downx + px0 - upx + 1,
            fh - py0 - 1, ih * upy - oh * downy + py0 - upy + 1]


def _needs_grad(*tensors):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _const_filter(f, what):
    if f is not None and f.requires_grad and torch.is_grad_enabled():
        raise nv.AutogradUnsupported(f"{what}: gradients w.r.t. the FIR filter are not implemented "
                                     "(SG3's synthesis filters are constant buffers)")


class _Upfirdn2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, f, up, down, padding, flip_filter, gain):
        y = _upfirdn2d_fwd(x, f, up, down, padding, flip_filter, gain)
        ctx.f = None if f is None else f.detach()
        ctx.meta = (tuple(x.shape[2:]), tuple(y.shape[2:]), up, down, padding, flip_filter, gain)
        return y

    @staticmethod
    def backward(ctx, dy):
        in_hw, out_hw, up, down, padding, flip_filter, gain = ctx.meta
        p = upfirdn2d_adjoint_padding(in_hw, out_hw, ctx.f, up, down, padding)
        dx = upfirdn2d(dy, ctx.f, up=down, down=up, padding=p, flip_filter=not flip_filter, gain=gain)
        assert tuple(dx.shape[2:]) == in_hw, (dx.shape, in_hw)
        return dx, None, None, None, None, None, None


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1, impl="cuda"):
    """Zero-insert upsample -> pad/crop -> FIR -> downsample, NCHW (differentiable in x)."""
    _const_filter(f, "upfirdn2d")
    if _needs_grad(x):
        return _Upfirdn2d.apply(x, f, up, down, padding, flip_filter, gain)
    return _upfirdn2d_fwd(x, f, up, down, padding, flip_filter, gain)


def bias_act_grad_mask(y, act, alpha, gain, clamp):
    """d act(z) / dz from the saved OUTPUT y = clamp(act(z) * gain): lrelu's slope follows sign(y) (gain > 0)
    and clamped elements pass no gradient."""
    code, def_alpha, def_gain = _ACT[act]
    alpha = float(alpha if alpha is not None else def_alpha)
    gain = float(gain if gain is not None else def_gain)
    m = torch.where(y > 0, gain, gain * alpha) if act == "lrelu" else torch.full_like(y, gain)
    if clamp is not None and clamp >= 0:
        m = m * (y.abs() < clamp)
    return m


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, dim, act, alpha, gain, clamp):
        y = _bias_act_fwd(x, b, dim, act, alpha, gain, clamp)
        ctx.save_for_backward(y)
        ctx.meta = (dim, act, alpha, gain, clamp, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dim, act, alpha, gain, clamp, has_b = ctx.meta
        dx = (dy.float() * bias_act_grad_mask(y.float(), act, alpha, gain, clamp)).to(y.dtype)
        db = None
        if has_b and ctx.needs_input_grad[1]:
            db = dx.float().sum(dim=[d for d in range(dx.ndim) if d != dim])
        return dx, db, None, None, None, None, None


def bias_act(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None, impl="cuda"):
    """x + b (broadcast along ``dim``) -> act -> * gain -> clamp (differentiable in x and b)."""
    if _needs_grad(x, b):
        return _BiasAct.apply(x, b, dim, act, alpha, gain, clamp)
    return _bias_act_fwd(x, b, dim, act, alpha, gain, clamp)


def filtered_lrelu_backward(z, dout, fu, fd, up, down, padding, gain, slope, clamp, flip_filter=False):
    """dL/dz of filtered_lrelu for the biased input z [N, C, H, W] f32 (NCHW): recompute the upsampled
    pre-activation U = up(z), mask the adjoint of the down FIR by lrelu'(U) * gain (zero where clamped), then
    apply the adjoint of the up FIR.  Every step is a HIP kernel (upfirdn2d) or a torch elementwise op."""
    px0, px1, py0, py1 = _parse_padding(padding)
    u = _upfirdn2d_fwd(z, fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    v = _bias_act_fwd(u, None, 1, "lrelu", slope, gain, clamp)
    m = bias_act_grad_mask(v, "lrelu", slope, gain, clamp)
    del v
    pd = upfirdn2d_adjoint_padding(u.shape[2:], dout.shape[2:], fd, 1, down, 0)
    g = _upfirdn2d_fwd(dout.float().contiguous(), fd, up=down, down=1, padding=pd, flip_filter=not flip_filter)
    assert g.shape == u.shape, (g.shape, u.shape)
    g.mul_(m)
    del m, u
    pu = upfirdn2d_adjoint_padding(z.shape[2:], g.shape[2:], fu, up, 1, [px0, px1, py0, py1])
    dz = _upfirdn2d_fwd(g, fu, up=1, down=up, padding=pu, flip_filter=not flip_filter, gain=up ** 2)
    assert dz.shape == z.shape, (dz.shape, z.shape)
    return dz


class _FilteredLRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fu, fd, b, up, down, padding, gain, slope, clamp, flip_filter):
        y = _filtered_lrelu_fwd(x, fu, fd, b, up, down, padding, gain, slope, clamp, flip_filter)
        ctx.save_for_backward(x, b)
        ctx.filters = (None if fu is None else fu.detach(), None if fd is None else fd.detach())
        ctx.meta = (up, down, padding, gain, slope, clamp, flip_filter)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        fu, fd = ctx.filters
        up, down, padding, gain, slope, clamp, flip_filter = ctx.meta
        z = x.float()
        if b is not None:
            z = z + b.float().view(1, -1, 1, 1)
        dz = filtered_lrelu_backward(z.contiguous(), dy, fu, fd, up, down, padding, gain, slope, clamp, flip_filter)
        db = dz.sum(dim=[0, 2, 3]) if b is not None and ctx.needs_input_grad[3] else None
        return dz.to(x.dtype), None, None, db, None, None, None, None, None, None, None


def filtered_lrelu(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=np.sqrt(2), slope=0.2, clamp=None,
                   flip_filter=False, impl="cuda"):
    """Fused bias -> upsample -> FIR -> lrelu*gain -> clamp -> FIR -> downsample (differentiable in x, b)."""
    _const_filter(fu, "filtered_lrelu")
    _const_filter(fd, "filtered_lrelu")
    if _needs_grad(x, b):
        return _FilteredLRelu.apply(x, fu, fd, b, up, down, padding, gain, slope, clamp, flip_filter)
    return _filtered_lrelu_fwd(x, fu, fd, b, up, down, padding, gain, slope, clamp, flip_filter)
