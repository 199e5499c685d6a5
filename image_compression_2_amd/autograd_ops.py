"""Autograd wrappers over the HIP kernels: the training path of the reference (BASELINE config C5,
``train_hvae_encoder``, /root/reference/stylegan3_hvae_full.py:655-707) backpropagates through
HVAE_VGG_Encoder (loss.backward at :693-696).  Each op's forward is the inference kernel; its backward is a
HIP kernel as well (csrc/backward.hip, or the forward implicit GEMM on transformed weights):

    conv3x3 (nn.Conv2d, :62, :175-176)   fwd ic2_conv_igemm         bwd dx: ic2_conv_igemm on flipped, transposed
                                                                     weights; dW: ic2_conv_wgrad; db: column sum
    GroupNorm -> lrelu (-> AvgPool2d)    fwd ic2_group_norm_stats +  bwd ic2_gn_lrelu_pool_bwd
    (:183-191)                               ic2_gn_lrelu_pool
    AdaptiveAvgPool2d(1) (:218)          fwd ic2_global_avg_pool    bwd ic2_gap_bwd
    NCHW -> NHWC input packing           fwd ic2_nchw_to_nhwc       bwd ic2_nhwc_to_nchw

Activations are NHWC with padded channel strides, in the module's precision (f32 parity mode / bf16);
gradients flow in the same layout and dtype; weight gradients are f32.  The projector MLPs are [N, <=512]
matrices and run as torch ops on the device.

The encoder's loss reaches it through the FROZEN StyleGAN3 synthesis network (:671-674, the generator's
parameters are frozen at :259-261), so the synthesis layers need gradients w.r.t. their input activations and
their styles only:

    modulated conv (SG3 modulated_conv2d)  fwd ic2_conv_igemm (normalised W)   bwd dx: ic2_conv_igemm on the
                                                                                 flipped, transposed W
    filtered lrelu (SG3 filtered_lrelu)    fwd ic2_flrelu_nhwc                bwd ic2_flrelu_bwd_nhwc (fused:
                                                                                 recompute up(z), adjoint FIRs)
    styles / (de)modulation / Fourier input    torch ops on [N, <= 512] rows and the 36x36 input grid
"""
from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _native as nv


def _pad_to(c_p, t):
    return t if t.shape[-1] == c_p else torch.nn.functional.pad(t, (0, c_p - t.shape[-1]))


def pack_conv_weight_adjoint(weight, cout_p, cin_p, dt):
    """[cout][cin][kh][kw] f32 -> the dgrad pack [cin_p][kh][kw][cout_p] (dt): W flipped in space and transposed in
    channels, gathered in one launch (ic2_pack_weight_adjoint)."""
    w = weight.detach().to(torch.float32).contiguous()
    cout, cin, kh, kw = w.shape
    out = torch.empty([cin_p, kh, kw, cout_p], dtype=dt, device=w.device)
    nv.call("ic2_pack_weight_adjoint", nv.ptr(w), cout, cin, kh, kw, cin_p, cout_p, nv.ptr(out), nv.dtype_code(dt),
            nv.stream_of(w))
    return out


def pack_conv_weight(weight, cin_p, cout_p, dt):
    """[cout][cin][kh][kw] f32 -> packed [cout_p][kh][kw][cin_p] (dt) on the device."""
    w = weight.detach().to(torch.float32).contiguous()
    cout, cin, kh, kw = w.shape
    out = torch.empty([cout_p, kh, kw, cin_p], dtype=dt, device=w.device)
    nv.call("ic2_pack_weight", nv.ptr(w), cout, cin, kh, kw, cout_p, cin_p, 0, 1.0, nv.ptr(out), nv.dtype_code(dt),
            None, nv.stream_of(w))
    return out


_DERIVED = None  # dict while a derived_cache() block is active


@contextlib.contextmanager
def derived_cache():
    """Inside the block, data derived from a parameter (packed and adjoint conv weights, the padded bias) is built
    once and reused: the training step runs the encoder twice on the same weights (ref :670-671), forward and
    backward.  The parameters must not change inside the block (training.train_step steps the optimizer after it;
    a fused optimizer does not bump version counters, so the cache is scoped, not versioned)."""
    global _DERIVED
    prev, _DERIVED = _DERIVED, {}
    try:
        yield
    finally:
        _DERIVED = prev


def _derived(t, key, make):
    if _DERIVED is None or not isinstance(t, torch.nn.Parameter):  # temporaries: ids and storage get reused
        return make()
    k = (id(t), t.data_ptr()) + key
    hit = _DERIVED.get(k)
    if hit is None:
        hit = _DERIVED[k] = make()
    return hit


class SplitRows(torch.autograd.Function):
    """[L, n, c] -> L contiguous [n, widths[l]] leading-column slices; the backward writes every slice's gradient
    into one zero-initialised [L, n, c] tensor (one fill and L copies, where autograd's per-slice backward would
    build L full-size zero tensors and add them)."""

    @staticmethod
    def forward(ctx, t, widths):
        ctx.shape = t.shape
        return tuple(t[i, :, :w].contiguous() for i, w in enumerate(widths))

    @staticmethod
    def backward(ctx, *grads):
        g = None
        for i, gi in enumerate(grads):
            if gi is not None:
                if g is None:
                    g = gi.new_zeros(ctx.shape)
                g[i, :, : gi.shape[1]].copy_(gi)
        return g, None


def conv_nhwc(x, wp, bias_p, cout_valid, kh, pad, dt_out=None, wino=None, grad=False):
    """Conv on NHWC x with packed weights wp [cout_p][kh][kh][cin_p].  wino: a callable returning the same weights
    packed for the Winograd kernel (U [cout_p][3][4][cin_p] f16), used where ic2_conv_wino_preferred picks it.
    grad: the output is a gradient -- an f16 output is converted IEEE (overflow -> inf, which the loss scaler must
    see) instead of saturated at +-65504 like an activation."""
    n, h, w, cin_p = x.shape
    cout_p = wp.shape[0]
    ho, wo = h + 2 * pad - kh + 1, w + 2 * pad - kh + 1
    dt_out = x.dtype if dt_out is None else dt_out
    y = torch.empty([n, ho, wo, cout_p], dtype=dt_out, device=x.device)
    odt = nv.F16_IEEE if grad and dt_out == torch.float16 else nv.dtype_code(dt_out)
    if wino is not None and nv.wino_preferred(nv.dtype_code(x.dtype), n, h, w, cin_p, cout_p, kh, kh, pad):
        nv.conv_wino(nv.ptr(x), nv.ptr(wino()), nv.ptr(y), nv.dtype_code(x.dtype), odt, n, h, w,
                     cin_p, cout_p, cout_valid, pad, ho, wo, None, nv.ptr(bias_p), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC,
                     nv.stream_of(x))
        return y
    nv.conv_igemm(nv.ptr(x), nv.ptr(wp), nv.ptr(y), nv.dtype_code(x.dtype), odt, n, h, w, cin_p,
                  cout_p, cout_valid, kh, kh, pad, ho, wo, None, nv.ptr(bias_p), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC,
                  nv.stream_of(x), x.device)
    return y


class Conv2dNHWC(torch.autograd.Function):
    """nn.Conv2d (stride 1, zero padding, k x k) on NHWC activations with padded channel strides."""

    @staticmethod
    def forward(ctx, x, weight, bias, pad, cout_p):
        cout, cin, kh, kw = weight.shape
        cin_p = x.shape[-1]
        wp = _derived(weight, ("fwd", cin_p, cout_p, x.dtype), lambda: pack_conv_weight(weight, cin_p, cout_p, x.dtype))

        def padded_bias():
            bp = torch.zeros([cout_p], dtype=torch.float32, device=x.device)
            if bias is not None:
                bp[:cout] = bias.detach().float()
            return bp
        bp = _derived(bias if bias is not None else weight, ("bias", cout_p), padded_bias)
        y = conv_nhwc(x, wp, bp, cout, kh, pad)
        ctx.save_for_backward(x, weight)
        ctx.weight = weight  # the parameter object itself: the key of its derived-data cache
        ctx.pad, ctx.has_bias = pad, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        cout, cin, kh, kw = weight.shape
        n, h, w, cin_p = x.shape
        colsum = getattr(dy, "_ic2_colsum", None)   # from the GroupNorm backward that produced dy, if unchanged
        if colsum is not None and (colsum[1] != dy._version or colsum[0].numel() < cout):
            colsum = None
        dy = dy.to(x.dtype).contiguous()
        cout_p = dy.shape[-1]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # dx = conv(dy, W flipped in space, transposed in channels), padding k - 1 - pad
            wtp = _derived(ctx.weight, ("adj", cin_p, cout_p, x.dtype),
                           lambda: pack_conv_weight_adjoint(weight, cout_p, cin_p, x.dtype))
            dx = conv_nhwc(dy, wtp, None, cin_p, kh, kh - 1 - ctx.pad, grad=True)
        if ctx.needs_input_grad[1]:
            nfl = int(nv.query("ic2_conv_wgrad_ws_floats", n, h, w, cin_p, cout_p, kh, kw, ctx.pad))
            ws = torch.empty([max(nfl, 4)], dtype=torch.float32, device=x.device)
            dw = torch.empty([cout, cin, kh, kw], dtype=torch.float32, device=x.device)   # the parameter's layout
            nv.call("ic2_conv_wgrad_oihw", nv.ptr(x), nv.ptr(dy), nv.ptr(dw), nv.dtype_code(x.dtype), n, h, w, cin_p,
                    cout_p, cout, cin, kh, kw, ctx.pad, nv.ptr(ws), nfl, nv.stream_of(x))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if colsum is not None:   # the GroupNorm backward's f64 channel sums: no pass over dy
                db = colsum[0][:cout]
            else:   # f32 accumulation straight from the 16-bit gradient (no f32 copy of dy)
                db = dy.reshape(-1, cout_p).sum(0, dtype=torch.float32)[:cout]
        return dx, dw, db, None, None


class GroupNormLReluPoolNHWC(torch.autograd.Function):
    """nn.GroupNorm(groups, c, eps) -> F.leaky_relu(slope) (-> nn.AvgPool2d(2, 2)) on NHWC."""

    @staticmethod
    def forward(ctx, y, gamma, beta, groups, eps, slope, pool, c, dt_out):
        n, h, w, c_p = y.shape
        stream = nv.stream_of(y)
        nfl = int(nv.query("ic2_group_norm_stats_floats", n, h * w, groups))
        stats = torch.empty([nfl], dtype=torch.float32, device=y.device)
        nv.call("ic2_group_norm_stats", nv.ptr(y), nv.dtype_code(y.dtype), n, h * w, c_p, c, groups, float(eps),
                nv.ptr(stats), stream)
        oh, ow = (h // 2, w // 2) if pool else (h, w)
        out = torch.empty([n, oh, ow, c_p], dtype=dt_out, device=y.device)
        g32, b32 = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
        nv.call("ic2_gn_lrelu_pool", nv.ptr(y), nv.ptr(out), nv.dtype_code(y.dtype), nv.dtype_code(dt_out), n, h, w,
                c_p, c, groups, nv.ptr(stats), nv.ptr(g32), nv.ptr(b32), float(slope), int(pool), stream)
        ctx.save_for_backward(y, stats, g32, b32)
        ctx.meta = (groups, slope, pool, c)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, stats, g32, b32 = ctx.saved_tensors
        groups, slope, pool, c = ctx.meta
        n, h, w, c_p = y.shape
        dout = dout.contiguous()
        nfl = int(nv.query("ic2_gn_lrelu_pool_bwd_floats", n, h, w, c_p, groups))
        ws = torch.empty([nfl], dtype=torch.float32, device=y.device)
        dy = torch.empty_like(y)
        dgamma = torch.empty([c], dtype=torch.float32, device=y.device)
        dbeta = torch.empty([c], dtype=torch.float32, device=y.device)
        dsum = torch.empty([c], dtype=torch.float32, device=y.device)
        nv.call("ic2_gn_lrelu_pool_bwd_db", nv.ptr(y), nv.ptr(dout), nv.ptr(dy), nv.dtype_code(y.dtype),
                nv.dtype_code(dout.dtype), nv.dtype_code(dy.dtype), n, h, w, c_p, c, groups, nv.ptr(stats),
                nv.ptr(g32), nv.ptr(b32), float(slope), int(pool), nv.ptr(dgamma), nv.ptr(dbeta), nv.ptr(dsum),
                nv.ptr(ws), nfl, nv.stream_of(y))
        # sum of dy over (n, p): the producing conv's bias gradient (Conv2dNHWC.backward reads it instead of
        # reducing dy again); stamped with dy's version so an in-place accumulation into dy invalidates it
        dy._ic2_colsum = (dsum, dy._version)
        return dy, dgamma, dbeta, None, None, None, None, None, None


class GlobalAvgPoolNHWC(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) + flatten: NHWC [n, h, w, c_p] -> [n, c] f32."""

    @staticmethod
    def forward(ctx, x, c):
        n, h, w, c_p = x.shape
        nfl = int(nv.query("ic2_global_avg_pool_floats", n, h * w, c_p, c))
        buf = torch.empty([nfl], dtype=torch.float32, device=x.device)
        nv.call("ic2_global_avg_pool", nv.ptr(x), nv.dtype_code(x.dtype), n, h * w, c_p, c, nv.ptr(buf),
                nv.stream_of(x))
        ctx.shape, ctx.dtype, ctx.c = x.shape, x.dtype, c
        return buf[: n * c].view(n, c).clone()

    @staticmethod
    def backward(ctx, dp):
        n, h, w, c_p = ctx.shape
        dp = dp.float().contiguous()
        dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=dp.device)
        nv.call("ic2_gap_bwd", nv.ptr(dp), nv.ptr(dx), nv.dtype_code(ctx.dtype), n, h * w, c_p, ctx.c,
                nv.stream_of(dp))
        return dx, None


class ToNHWC(torch.autograd.Function):
    """NCHW f32 -> NHWC (dt, channel stride c_p, zero-padded)."""

    @staticmethod
    def forward(ctx, x, dt, c_p):
        n, c, h, w = x.shape
        out = torch.empty([n, h, w, c_p], dtype=dt, device=x.device)
        nv.call("ic2_nchw_to_nhwc", nv.ptr(x), nv.ptr(out), nv.dtype_code(dt), n, c, h, w, c_p, None, nv.stream_of(x))
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty([n, c, h, w], dtype=torch.float32, device=dy.device)
        nv.call("ic2_nhwc_to_nchw", nv.ptr(dy), nv.dtype_code(dy.dtype), nv.ptr(dx), n, c, h, w, dy.shape[-1],
                nv.stream_of(dy))
        return dx, None, None


def _synth_layer_grads(L, dt, os_, y, dout, post=None):
    """Backward of one modulated synthesis layer from dL/d(filtered lrelu output) `dout`: the FLR adjoint stored
    times oscale (dL/dconv) with the per-tile sums for dL/doscale, then the dgrad implicit GEMM -> (dL/da, dL/doscale),
    a = the conv's (already input-modulated) operand.  post [n][c_p]: `dout` is the gradient of the layer output
    multiplied by `post` (the next layer's input modulation) and still has to be multiplied by it.  The FLR backward
    is linear in its input gradient per channel (the lrelu / clamp mask depends on the recomputed U only, the FIRs do
    not mix channels), so the multiply rides on its per-channel output multiplier: dc = FLRbwd(dout) * oscale * post,
    and the ydot partials (taken against that multiplier) give dL/doscale = post * sum / oscale."""
    n, h, w, c_p = y.shape
    stream = nv.stream_of(y)
    _, _, bp = L.packed(dt)
    fu, fd = L._fu, L._fd
    px0, px1, py0, py1 = L.padding
    clamp = float(L.conv_clamp) if L.conv_clamp is not None else -1.0
    dc = torch.empty([n, h, w, c_p], dtype=dt, device=y.device)
    os32 = os_.detach().float()
    mul = os32 if post is None else (os32 * post).contiguous()
    # The Winograd dgrad forms V = B^T dc with f16 adds, which overflow for opposite-sign dc values above 2^15 where
    # the direct implicit GEMM would not -- but dL/da, a sum over 9 * cout products stored f16 (IEEE), overflows first:
    # on realistic gradients both dgrads turn inf at the same loss scale (test_gpu_wino.py::
    # test_wino_dgrad_overflows_at_the_direct_gemms_scale).  Storing dc halved against 2 U would remove the V hazard
    # but costs a bit on every f16-subnormal dc value (a 2^12 loss scale's synthesis gradient: 3.06e-2 vs < 3e-2
    # relative error), so dc is stored as is.
    rc = 2
    if fu is not None and fd is not None and px0 == py0:
        nyd = int(nv.query("ic2_flrelu_bwd_ydot_floats", n, c_p, h, w, L.up_factor))
        ydot = torch.empty([nyd], dtype=torch.float32, device=y.device)
        rc = nv.load().ic2_flrelu_bwd_nhwc_ex(
            nv.ptr(y), nv.dtype_code(y.dtype), nv.ptr(dout), nv.dtype_code(dout.dtype), nv.ptr(dc),
            nv.dtype_code(dt), n, c_p, h, w, dout.shape[1], dout.shape[2], fu.ctypes.data_as(ctypes.c_void_p),
            fu.shape[0], fd.ctypes.data_as(ctypes.c_void_p), fd.shape[0], L.up_factor, L.down_factor, px0, px1,
            py0, py1, float(L.act_gain), 0.2, clamp, 0, nv.ptr(mul), nv.ptr(bp), nv.ptr(ydot), nyd, stream)
        if rc not in (0, 2):
            raise RuntimeError(f"ic2_flrelu_bwd_nhwc_ex failed: {nv.load().ic2_last_error().decode()}")
    if rc == 0:   # dL/doscale = sum over tiles of the ydot partials / oscale (0 where oscale is 0), one launch
        d_os = nv.colsum_div(ydot, n, c_p, os32)
        if post is not None:
            d_os = d_os * post
    else:   # no fused instance for this geometry: the composed HIP path + torch epilogue
        if post is not None:
            dout = (dout.float() * post[:, None, None, :]).to(dout.dtype)
        gy = _flrelu_backward_composed(y, dout, L)
        dc.copy_(gy * os_[:, None, None, :])
        yd = (gy * (y.float() - bp)).sum(dim=(1, 2))
        d_os = torch.where(os_ != 0, yd / torch.where(os_ != 0, os_, torch.ones_like(os_)), torch.zeros_like(os_))
    # dL/da: the implicit GEMM on the adjoint weights (valid conv: the forward padded by k - 1), or the Winograd kernel
    # where ic2_conv_wino_preferred picks it; f16 stored IEEE (a gradient: overflow -> inf for the loss scaler)
    da = conv_nhwc(dc, L.packed_adjoint(dt), None, L.in_channels, L.conv_kernel, 0,
                   wino=L.packed_adjoint_wino if dt == torch.float16 else None, grad=True)
    return da, d_os


def _synth_conv_fwd(layer, a, os_, dt, y):
    """The modulated conv of the training forward: y = conv(a, W_norm) * oscale + bias, NHWC (f16 operands: the
    Winograd kernel where ic2_conv_wino_preferred picks it, as inference's conv_nhwc)."""
    n, s_in = a.shape[0], a.shape[1]
    k = layer.conv_kernel
    pad = k - 1
    conv = y.shape[1]
    wp, _, bp = layer.packed(dt)
    if dt == torch.float16 and nv.wino_preferred(nv.F16, n, s_in, s_in, layer.cin_p, layer.cout_p, k, k, pad):
        nv.conv_wino(nv.ptr(a), nv.ptr(layer.packed_wino()), nv.ptr(y), nv.F16, nv.dtype_code(y.dtype), n, s_in, s_in,
                     layer.cin_p, layer.cout_p, layer.out_channels, pad, conv, conv, nv.ptr(os_), nv.ptr(bp), 0, 0.0,
                     1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(a))
        return
    nv.conv_igemm(nv.ptr(a), nv.ptr(wp), nv.ptr(y), nv.dtype_code(dt), nv.dtype_code(y.dtype), n, s_in, s_in,
                  layer.cin_p, layer.cout_p, layer.out_channels, k, k, pad, conv, conv, nv.ptr(os_), nv.ptr(bp), 0,
                  0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(a), a.device)


class SynthLayerScaledNHWC(torch.autograd.Function):
    """A modulated synthesis layer on the network's training path, taking its input already modulated and
    returning its output modulated for the NEXT layer (SG3 SynthesisLayer.forward chained):
        y = conv(a, W_norm) * oscale + bias  ->  out = filtered_lrelu(y) * xs_next
    The next layer's input modulation rides on this layer's FLR store (its post-scale row, as in inference), so the
    separate ic2_scale_nhwc pass over every activation is gone.  Backward: dL/d(lrelu out) = g * xs_next and
    dL/dxs_next = sum_p g * out / xs_next (ic2_scale_bwd_nhwc on the stored, modulated out; 0 where xs_next = 0, where
    out is 0 too), then _synth_layer_grads; the gradient w.r.t. `a` is dL/da itself."""

    @staticmethod
    def forward(ctx, a, os_, xs_next, layer, dt):
        n, s_in = a.shape[0], a.shape[1]
        a = a.contiguous()
        assert xs_next.shape == (n, layer.cout_p), (xs_next.shape, layer.cout_p)
        k = layer.conv_kernel
        pad = k - 1
        conv = s_in + 2 * pad - k + 1
        ydt = torch.float16 if dt == torch.bfloat16 else dt
        y = torch.empty([n, conv, conv, layer.cout_p], dtype=ydt, device=a.device)
        _synth_conv_fwd(layer, a, os_, dt, y)
        xs32 = xs_next.detach().float().contiguous()
        out = layer.flrelu_nhwc(y, dt, post_scale=xs32)
        ctx.save_for_backward(a, os_, xs32, y, out)
        ctx.layer, ctx.dt = layer, dt
        return out

    @staticmethod
    def backward(ctx, g):
        a, os_, xs, y, out = ctx.saved_tensors
        L, dt = ctx.layer, ctx.dt
        g = g.to(out.dtype).contiguous()
        n, ho, wo, c_p = out.shape
        npart = int(nv.query("ic2_scale_bwd_part_floats", n, ho * wo, c_p))
        part = torch.empty([npart], dtype=torch.float32, device=out.device)
        # the sums for d xs_next only: g * xs_next itself rides on the FLR backward's output multiplier (post=)
        nv.call("ic2_scale_bwd_nhwc", nv.ptr(g), nv.ptr(out), nv.ptr(xs), None, nv.dtype_code(out.dtype), n,
                ho * wo, c_p, nv.ptr(part), npart, nv.stream_of(out))
        d_xs = nv.colsum_div(part, n, c_p, xs)   # sum_p g * out / xs_next, 0 where xs_next = 0
        da, d_os = _synth_layer_grads(L, dt, os_, y, g, post=xs)
        return da, d_os, d_xs, None, None


class ScaleNHWC(torch.autograd.Function):
    """a = x * xscale[n][c] on NHWC (ic2_scale_nhwc), differentiable in x and xscale (ic2_scale_bwd_nhwc: the per-pixel
    sums of d xscale reduce in f32 per chunk, so an f16 activation with a loss-scaled gradient does not overflow the
    way an f16 torch reduction over 256^2 pixels does)."""

    @staticmethod
    def forward(ctx, x, xs):
        x = x.contiguous()
        n, h, w, c_p = x.shape
        xs32 = xs.detach().float().contiguous()
        a = torch.empty_like(x)
        nv.call("ic2_scale_nhwc", nv.ptr(x), nv.ptr(xs32), nv.ptr(a), nv.dtype_code(x.dtype), n, h * w, c_p,
                nv.stream_of(x))
        ctx.save_for_backward(x, xs32)
        return a

    @staticmethod
    def backward(ctx, da):
        x, xs = ctx.saved_tensors
        n, h, w, c_p = x.shape
        da = da.to(x.dtype).contiguous()
        npart = int(nv.query("ic2_scale_bwd_part_floats", n, h * w, c_p))
        part = torch.empty([npart], dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        nv.call("ic2_scale_bwd_nhwc", nv.ptr(da), nv.ptr(x), nv.ptr(xs), nv.ptr(dx), nv.dtype_code(x.dtype), n, h * w,
                c_p, nv.ptr(part), npart, nv.stream_of(x))
        return dx, nv.colsum_div(part, n, c_p)


class FrozenConvNHWC(torch.autograd.Function):
    """Conv with constant, pre-packed weights (the modulated conv of a frozen SG3 layer, whose per-sample
    modulation is applied outside as xscale / oscale): output f32, gradient w.r.t. the input only.
    wp [cout_p][k][k][cin_p] and wt = the flipped, channel-transposed pack [cin_p][k][k][cout_p]."""

    @staticmethod
    def forward(ctx, x, wp, wt, k, pad, cout, cin):
        y = conv_nhwc(x, wp, None, cout, k, pad, dt_out=torch.float32)
        ctx.wt, ctx.meta = wt, (k, pad, cin, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        k, pad, cin, dt = ctx.meta
        dx = conv_nhwc(dy.to(dt).contiguous(), ctx.wt, None, cin, k, k - 1 - pad, grad=True)
        return dx, None, None, None, None, None, None


def _flr_chunk(n, c, hu, wu):
    """Samples per backward chunk: keep the recomputed upsampled planes (f32, ~3 live copies) near 2 GiB."""
    per = max(1, c * hu * wu * 4 * 3)
    return max(1, min(n, (2 << 30) // per))


class FilteredLReluNHWC(torch.autograd.Function):
    """SG3 filtered_lrelu on NHWC activations with the layer's filters, padding, gain sqrt(2), slope 0.2 and
    clamp (SynthesisLayer.forward).  y arrives in f32; in bf16 mode it is saturated to the f16 range and stored
    as f16 for the MFMA forward kernel (the inference epilogue's semantics), and that f16 copy is what the
    backward recomputes from.  Forward: the fused HIP kernel.  Backward: ic2_flrelu_bwd_nhwc (one fused HIP
    kernel: U recompute, adjoint down-FIR, lrelu'/clamp mask, adjoint up-FIR; f32 gradient) for the StyleGAN3-T
    geometries, otherwise per chunk of samples through sg3_ops.filtered_lrelu_backward (HIP upfirdn2d)."""

    @staticmethod
    def forward(ctx, y, layer, dt_out):
        if dt_out == torch.bfloat16:
            y = y.clamp(-65504.0, 65504.0).to(torch.float16)
        else:
            y = y.contiguous()
        out = layer.flrelu_nhwc(y, dt_out)
        ctx.save_for_backward(y)
        ctx.layer = layer
        return out

    @staticmethod
    def backward(ctx, dout):
        (y,) = ctx.saved_tensors
        L = ctx.layer
        dout = dout.contiguous()
        n, h, w, c_p = y.shape
        fu, fd = L._fu, L._fd
        px0, px1, py0, py1 = L.padding
        clamp = float(L.conv_clamp) if L.conv_clamp is not None else -1.0
        if fu is not None and fd is not None and px0 == py0:
            dy = torch.empty([n, h, w, c_p], dtype=torch.float32, device=y.device)
            rc = nv.load().ic2_flrelu_bwd_nhwc(
                nv.ptr(y), nv.dtype_code(y.dtype), nv.ptr(dout), nv.dtype_code(dout.dtype), nv.ptr(dy), n, c_p, h, w,
                dout.shape[1], dout.shape[2], fu.ctypes.data_as(ctypes.c_void_p), fu.shape[0],
                fd.ctypes.data_as(ctypes.c_void_p), fd.shape[0], L.up_factor, L.down_factor, px0, px1, py0, py1,
                float(L.act_gain), 0.2, clamp, 0, nv.stream_of(y))
            if rc == 0:
                return dy, None, None
            if rc != 2:   # anything but IC2_E_UNSUPPORTED is an error
                raise RuntimeError(f"ic2_flrelu_bwd_nhwc failed: {nv.load().ic2_last_error().decode()}")
        return _flrelu_backward_composed(y, dout, L), None, None


def _flrelu_backward_composed(y, dout, L):
    from . import sg3_ops
    n, h, w, c_p = y.shape
    c = L.out_channels
    dy = torch.zeros([n, h, w, c_p], dtype=torch.float32, device=y.device)
    hu = h * L.up_factor + L.padding[2] + L.padding[3] - (L.up_taps - 1)
    wu = w * L.up_factor + L.padding[0] + L.padding[1] - (L.up_taps - 1)
    step = _flr_chunk(n, c, hu, wu)
    clamp = float(L.conv_clamp) if L.conv_clamp is not None else None
    for i in range(0, n, step):
        z = y[i:i + step, :, :, :c].permute(0, 3, 1, 2).float().contiguous()
        g = dout[i:i + step, :, :, :c].permute(0, 3, 1, 2).float().contiguous()
        dz = sg3_ops.filtered_lrelu_backward(z, g, L.up_filter, L.down_filter, L.up_factor, L.down_factor,
                                             L.padding, L.act_gain, 0.2, clamp)
        dy[i:i + step, :, :, :c] = dz.permute(0, 2, 3, 1)
    return dy


class SynthLayerNHWC(torch.autograd.Function):
    """One non-ToRGB synthesis layer on the autograd path, w.r.t. its input activation and its (de)modulation
    coefficients (SG3 SynthesisLayer.forward with frozen weights):
        a = x * xscale[n][i]  ->  y = conv(a, W_norm) * oscale[n][o] + bias  ->  out = filtered_lrelu(y)
    Forward = the inference kernels (ic2_conv_igemm with oscale / bias / f16-saturating epilogue in bf16 mode,
    ic2_flrelu_nhwc).  Backward, three HIP launches:
        ic2_flrelu_bwd_nhwc_ex  dL/dy (FLR adjoint), stored times oscale (= dL/dconv, the dgrad operand) and the
                                per-tile sums of dL/dy * (y - bias) -> dL/doscale = sum / oscale
        ic2_conv_igemm          dL/da = conv(dL/dconv, flipped / transposed W)
        ic2_scale_bwd_nhwc      dL/dx = dL/da * xscale, dL/dxscale = sum_p dL/da * x"""

    @staticmethod
    def forward(ctx, x, xs, os_, layer, dt):
        n, s_in = x.shape[0], x.shape[1]
        x = x.contiguous()
        xs32 = xs.detach().float().contiguous()
        assert xs32.shape == (n, x.shape[3]), (xs32.shape, x.shape)
        a = torch.empty_like(x)
        nv.call("ic2_scale_nhwc", nv.ptr(x), nv.ptr(xs32), nv.ptr(a), nv.dtype_code(x.dtype), n, s_in * s_in,
                x.shape[3], nv.stream_of(x))
        k = layer.conv_kernel
        pad = k - 1
        conv = s_in + 2 * pad - k + 1
        ydt = torch.float16 if dt == torch.bfloat16 else dt
        y = torch.empty([n, conv, conv, layer.cout_p], dtype=ydt, device=x.device)
        _synth_conv_fwd(layer, a, os_, dt, y)
        del a
        out = layer.flrelu_nhwc(y, dt)
        ctx.save_for_backward(x, xs, os_, y)
        ctx.layer, ctx.dt = layer, dt
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xs, os_, y = ctx.saved_tensors
        da, d_os = _synth_layer_grads(ctx.layer, ctx.dt, os_, y, dout.contiguous())
        n, hi, wi, cin_p = x.shape
        npart = int(nv.query("ic2_scale_bwd_part_floats", n, hi * wi, cin_p))
        part = torch.empty([npart], dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        nv.call("ic2_scale_bwd_nhwc", nv.ptr(da), nv.ptr(x), nv.ptr(xs), nv.ptr(dx), nv.dtype_code(x.dtype), n, hi * wi,
                cin_p, nv.ptr(part), npart, nv.stream_of(y))
        d_xs = nv.colsum_div(part, n, cin_p)
        return dx, d_xs, d_os, None, None
