"""Drop-in for /root/reference/stylegan3_hvae_full.py's hot-path classes, MI355X-native.

Same class names, constructor arguments, module tree / state-dict keys and parameter-construction
order as the reference (so ``torch.manual_seed(s)`` + construction draws identical weights and the
reference's checkpoints load).  The forward passes run in libic2ops HIP kernels:

  HVAE_VGG_Encoder.forward  (ref :105-167)   NHWC, MFMA implicit-GEMM 3x3 convs, deterministic GroupNorm,
                                             fused GN-apply + lrelu + 2x2 avg-pool, GAP, FCs, reparam
  StyleGAN3Compressor.compress (ref :295-318) bit-exact uniform quantizer kernel
  StyleGAN3Compressor.decompress / forward    generator.synthesis (networks_stylegan3) + bilinear resize

Behaviour kept on purpose: the fine projector's fc1 is re-created with fresh
``nn.Linear`` weights (CPU RNG) whenever the pooled width differs from ``in_channels`` (ref :225-230);
reparameterisation noise is drawn with ``torch.randn_like`` on the device in the reference's order.
Not kept: the debug prints of every forward.  ``precision`` ('fp32' parity | 'bf16' throughput) is an
opt-in extension.
"""
from __future__ import annotations

import math
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from PIL import Image

from . import _native as nv
from . import autograd_ops as ao


def _version_key(*tensors):
    return tuple((t.data_ptr(), t._version, t.device) for t in tensors)


class _Act:
    """NHWC activation handle: tensor [n, h, w, c_p] + logical channel count.  x3: split bf16 (ic2ops.h
    IC2_BF16X3), the tensor holds 2 * c_p bf16 channels [hi | lo] per pixel (the convs' K runs over [hi | hi | lo]).
    h2: plain f16, consumed by the split-weight convs (IC2_F16X2: K runs over [x | x] against [w_hi | w_lo])."""
    __slots__ = ("t", "n", "h", "w", "c", "c_p", "x3", "h2")

    def __init__(self, t, c, x3=False, h2=False):
        self.t = t
        self.n, self.h, self.w, cp = t.shape
        self.c_p = cp // 2 if x3 else cp
        self.c = c
        self.x3 = x3
        self.h2 = h2

    @property
    def split(self):
        return self.x3 or self.h2

    @property
    def k_p(self):
        """Channel stride the conv's GEMM sees (the tripled / doubled one in the split modes)."""
        return 3 * self.c_p if self.x3 else 2 * self.c_p if self.h2 else self.c_p

    @property
    def code(self):
        return nv.BF16X3 if self.x3 else nv.F16X2 if self.h2 else nv.dtype_code(self.t.dtype)


def _packed(conv: nn.Conv2d, x: _Act, dt, cache: dict, stream):
    cout, cin, kh, kw = conv.weight.shape
    assert conv.stride == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and cin == x.c
    x3, h2 = bool(getattr(x, "x3", False)), bool(getattr(x, "h2", False))
    key = (dt, x3, h2, _version_key(conv.weight, conv.bias))
    hit = cache.get(id(conv))
    if hit is None or hit[0] != key:
        w = conv.weight.detach().to(torch.float32).contiguous()
        cout_p, cin_p = nv.pad32(cout), x.c_p
        # split modes: [cout_p][kh][kw][3 * cin_p] = [hi | lo | hi] against the activation's [hi | hi | lo]; f16
        # [cout_p][kh][kw][2 * cin_p] = [hi | lo] against [x | x], the weights times 2^s (max |w| 2^s in [2^12, 2^13):
        # the low halves of all but the ~2^-15-smallest weights stay f16 normals), the conv output times 2^-s (exact)
        mul = 1.0
        if h2:
            wp = torch.empty([cout_p, kh, kw, 2 * cin_p], dtype=torch.float16, device=w.device)
            m = float(w.abs().max().item())
            sh = 13 - math.frexp(m)[1] if m > 0 else 0
            mul = math.ldexp(1.0, -sh)
        else:
            wp = torch.empty([cout_p, kh, kw, 3 * cin_p if x3 else cin_p], dtype=dt, device=w.device)
        nv.call("ic2_pack_weight", nv.ptr(w), cout, cin, kh, kw, cout_p, cin_p, 0, 1.0 / mul, nv.ptr(wp),
                nv.BF16X3 if x3 else nv.F16X2 if h2 else nv.dtype_code(dt), None, stream)
        bp = torch.zeros([cout_p], dtype=torch.float32, device=w.device)
        if conv.bias is not None:
            bp[:cout] = conv.bias.detach().float() / mul
        hit = (key, (wp, bp), mul)
        cache[id(conv)] = hit
    return hit[1]


def _out_mul(conv: nn.Conv2d, cache: dict):
    """The output multiplier of conv's cached packing (2^-s for split-weight f16 weights packed times 2^s, else 1)."""
    return cache[id(conv)][2]


def _conv_flops(n, ho, wo, cout, cin, kh, kw):
    """Algorithmic FLOPs of an nn.Conv2d launch (unpadded channels): what the reference computes."""
    return 2 * n * ho * wo * cout * cin * kh * kw


def _conv(conv: nn.Conv2d, x: _Act, dt, cache: dict, stream):
    """nn.Conv2d (3x3 or k x k, stride 1, 'same' padding) + bias on MFMA (plain activations; the split ones go through
    _conv_gn)."""
    assert not x.split, "split activations are consumed by _conv_gn"
    cout, cin, kh, kw = conv.weight.shape
    pad = conv.padding[0]
    wp, bp = _packed(conv, x, dt, cache, stream)
    cout_p = wp.shape[0]
    ho, wo = x.h + 2 * pad - kh + 1, x.w + 2 * pad - kw + 1
    y = torch.empty([x.n, ho, wo, cout_p], dtype=dt, device=x.t.device)
    nv.note_flops(_conv_flops(x.n, ho, wo, cout, cin, kh, kw))
    nv.conv_igemm(nv.ptr(x.t), nv.ptr(wp), nv.ptr(y), nv.dtype_code(x.t.dtype), nv.dtype_code(dt), x.n, x.h, x.w,
                  x.c_p, cout_p, cout, kh, kw, pad, ho, wo, None, nv.ptr(bp), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, stream,
                  x.t.device)
    return _Act(y, cout)


# knob IC2_FROM_RGB_DIRECT=0 (IC2_DEV=1) keeps the packing + implicit-GEMM from_rgb (A/B switch)
_FROM_RGB_DIRECT = nv.knob("IC2_FROM_RGB_DIRECT", 1) != 0
# knob IC2_SPLIT_F16_BLOCKS: in the split ('bf16x3') mode the first K blocks' convs take f16 activations against
# split f16 weights (IC2_F16X2, two f16 MFMAs per product instead of three bf16 ones): K = 3 (blocks 0-2,
# the 1024^2 .. 256^2 levels at C4) by default, 0 = every conv split bf16.  Measured (profiles/r5_split_f16_blocks.txt):
# K 0 / 2 / 3 -> C4 316 / 340 / 346 img/s, C2 1426 / 1451 / 1461 (f32 conv outputs), C2 index mismatches 18 / 37 / 34
# of 262144; with f16 conv outputs (default) K = 3 -> C4 371-378, C2 1482-1520, 63 mismatches
_SPLIT_F16_BLOCKS = nv.knob("IC2_SPLIT_F16_BLOCKS", 3)
# knob IC2_GN_IN_FUSE=1 applies norm1 + lrelu inside conv2's halo-conv staging instead of materialising it.  Bit-identical
# but measured level on MI355X (C2 1438.0 -> 1439.4, C4 415.5 -> 415.9 img/s, same box: the saved pass is paid back in
# the heavier staging of the 64-channel halo conv), so off by default
_GN_IN_FUSE = nv.knob("IC2_GN_IN_FUSE", 0) == 1


def _from_rgb(conv: nn.Conv2d, x, dt, cache: dict, stream, split=False, h2=False):
    """from_rgb on the NCHW f32 image: in bf16 mode one direct kernel (ic2_from_rgb_conv: no 32-channel packed copy
    of the image), else the packing + implicit GEMM.  split: the encoder's bf16x3 mode -- exact f32 arithmetic, the
    output stored split for the next conv (ic2_from_rgb_conv_x3, or an f32 conv + split packing); h2: rounded once to
    f16 instead, the input of a split-weight f16 conv (ic2_from_rgb_conv_f16)."""
    cout, cin, kh, kw = conv.weight.shape
    if split:
        n, _, hh, ww = x.shape
        cout_p = nv.pad32(cout)
        bp = torch.zeros([cout_p], dtype=torch.float32, device=x.device)
        bp[:cout] = conv.bias.detach().float()
        direct = cin <= 4 and kh == 3 and kw == 3 and conv.padding[0] == 1 and cout_p in (32, 64, 128)
        if h2 and direct:
            y = torch.empty([n, hh, ww, cout_p], dtype=torch.float16, device=x.device)
            wf = conv.weight.detach().to(torch.float32).contiguous()
            nv.note_flops(_conv_flops(n, hh, ww, cout, cin, 3, 3))
            nv.call("ic2_from_rgb_conv_f16", nv.ptr(x), cin, nv.ptr(wf), cout, nv.ptr(bp), nv.ptr(y), n, hh, ww,
                    cout_p, stream)
            return _Act(y, cout, h2=True)
        y = torch.empty([n, hh, ww, 2 * cout_p], dtype=torch.bfloat16, device=x.device)
        if direct:
            wf = conv.weight.detach().to(torch.float32).contiguous()
            nv.note_flops(_conv_flops(n, hh, ww, cout, cin, 3, 3))
            nv.call("ic2_from_rgb_conv_x3", nv.ptr(x), cin, nv.ptr(wf), cout, nv.ptr(bp), nv.ptr(y), n, hh, ww, cout_p,
                    stream)
        else:
            xf = _to_nhwc(x, torch.float32, stream)
            wp, bq = _packed(conv, xf, torch.float32, cache, stream)
            pad = conv.padding[0]
            ho, wo = hh + 2 * pad - kh + 1, ww + 2 * pad - kw + 1
            yf = torch.empty([n, cout, ho, wo], dtype=torch.float32, device=x.device)
            nv.note_flops(_conv_flops(n, ho, wo, cout, cin, kh, kw))
            nv.conv_igemm(nv.ptr(xf.t), nv.ptr(wp), nv.ptr(yf), nv.F32, nv.F32, n, hh, ww, xf.c_p, cout_p, cout, kh, kw,
                          pad, ho, wo, None, nv.ptr(bq), 0, 0.0, 1.0, -1.0, 1.0, nv.NCHW, stream, x.device)
            y = torch.empty([n, ho, wo, 2 * cout_p], dtype=torch.bfloat16, device=x.device)
            nv.call("ic2_nchw_to_nhwc", nv.ptr(yf), nv.ptr(y), nv.BF16X3, n, cout, ho, wo, cout_p, None, stream)
        return _Act(y, cout, x3=True)
    if (dt == torch.bfloat16 and cin <= 4 and kh == 3 and kw == 3 and conv.padding[0] == 1
            and nv.pad32(cout) in (32, 64) and _FROM_RGB_DIRECT):
        n, _, hh, ww = x.shape
        fake = types.SimpleNamespace(c=cin, c_p=nv.pad32(cin))
        wp, bp = _packed(conv, fake, dt, cache, stream)
        y = torch.empty([n, hh, ww, wp.shape[0]], dtype=dt, device=x.device)
        nv.note_flops(_conv_flops(n, hh, ww, cout, cin, kh, kw))
        nv.call("ic2_from_rgb_conv", nv.ptr(x), cin, nv.ptr(wp), fake.c_p, nv.ptr(bp), nv.ptr(y), n, hh, ww,
                wp.shape[0], stream)
        return _Act(y, cout)
    return _conv(conv, _to_nhwc(x, dt, stream), dt, cache, stream)


def _conv_gn(conv: nn.Conv2d, norm: nn.GroupNorm, x: _Act, dt, cache: dict, stream, fuse=-1, in_gn=None):
    """conv (+ bias) and the GroupNorm statistics of its output in one call (ic2_conv3x3_gn_fwd: fused into the
    halo conv's epilogue where that kernel runs the layer).  in_gn = (affine table, slope): the previous GroupNorm +
    lrelu applied to x while the halo conv stages it (ic2_conv3x3_gnin_gn_fwd).  -> (y, stats)."""
    cout, cin, kh, kw = conv.weight.shape
    pad = conv.padding[0]
    wp, bp = _packed(conv, x, dt, cache, stream)
    cout_p = wp.shape[0]
    ho, wo = x.h + 2 * pad - kh + 1, x.w + 2 * pad - kw + 1
    # split-weight f16: the conv output stored f16 (its consumer, the f16 GroupNorm output, rounds there anyway)
    ydt = torch.float16 if x.h2 else torch.float32
    if x.split and bool(nv.query("ic2_conv3x3_gn_fuses", x.code, x.n, x.h, x.w, x.k_p, cout_p, cout, kh, kw, pad,
                                 norm.num_groups, int(fuse))):
        # split bf16 / split-weight f16, 64- / 128-wide layers: the 4-wave halo GEMM writes the output and the
        # statistics in one launch
        y = torch.empty([x.n, ho, wo, cout_p], dtype=ydt, device=x.t.device)
        nfl = int(nv.query("ic2_conv3x3_gn_stats_floats", x.code, x.n, x.h, x.w, x.k_p, cout_p, kh, kw, pad,
                           norm.num_groups))
        stats = torch.empty([nfl], dtype=torch.float32, device=x.t.device)
        nv.note_flops(_conv_flops(x.n, ho, wo, cout, cin, kh, kw))
        if x.h2:
            nv.call("ic2_conv3x3_gn_fwd_scaled", nv.ptr(x.t), nv.ptr(wp), nv.ptr(y), x.code, x.n, x.h, x.w, x.k_p,
                    cout_p, cout, kh, kw, pad, nv.ptr(bp), _out_mul(conv, cache), norm.num_groups, float(norm.eps),
                    nv.ptr(stats), nfl, None, 0, int(fuse), stream)
        else:
            nv.call("ic2_conv3x3_gn_fwd", nv.ptr(x.t), nv.ptr(wp), nv.ptr(y), x.code, x.n, x.h, x.w, x.k_p, cout_p,
                    cout, kh, kw, pad, nv.ptr(bp), norm.num_groups, float(norm.eps), nv.ptr(stats), nfl, None, 0,
                    int(fuse), stream)
        return _Act(y, cout), stats
    if x.split:
        # split bf16: one bf16 implicit GEMM over the tripled K (its input [hi | lo] read as [hi | hi | lo]), f32 out,
        # GroupNorm statistics on the f32 values (split-weight f16: the f16 GEMM over the doubled K)
        y = torch.empty([x.n, ho, wo, cout_p], dtype=ydt, device=x.t.device)
        nv.note_flops(_conv_flops(x.n, ho, wo, cout, cin, kh, kw))
        nv.conv_igemm(nv.ptr(x.t), nv.ptr(wp), nv.ptr(y), x.code, nv.dtype_code(ydt), x.n, x.h, x.w, x.k_p, cout_p,
                      cout, kh, kw, pad, ho, wo, None, nv.ptr(bp), 0, 0.0, 1.0, -1.0, _out_mul(conv, cache), nv.NHWC,
                      stream, x.t.device)
        ya = _Act(y, cout)
        nfl = int(nv.query("ic2_group_norm_stats_floats", ya.n, ya.h * ya.w, norm.num_groups))
        stats = torch.empty([nfl], dtype=torch.float32, device=y.device)
        nv.call("ic2_group_norm_stats", nv.ptr(y), nv.dtype_code(ydt), ya.n, ya.h * ya.w, ya.c_p, ya.c,
                norm.num_groups, float(norm.eps), nv.ptr(stats), stream)
        return ya, stats
    if dt == torch.float16:
        # f16 (the training precision's inference forward): the conv, then the separate statistics pass (the fused
        # statistics epilogue is bf16 halo-conv code)
        ya = _conv(conv, x, dt, cache, stream)
        nfl = int(nv.query("ic2_group_norm_stats_floats", ya.n, ya.h * ya.w, norm.num_groups))
        stats = torch.empty([nfl], dtype=torch.float32, device=ya.t.device)
        nv.call("ic2_group_norm_stats", nv.ptr(ya.t), nv.F16, ya.n, ya.h * ya.w, ya.c_p, ya.c, norm.num_groups,
                float(norm.eps), nv.ptr(stats), stream)
        return ya, stats
    dc = nv.dtype_code(dt)
    y = torch.empty([x.n, ho, wo, cout_p], dtype=dt, device=x.t.device)
    nfl = int(nv.query("ic2_conv3x3_gn_stats_floats", dc, x.n, x.h, x.w, x.c_p, cout_p, kh, kw, pad, norm.num_groups))
    stats = torch.empty([nfl], dtype=torch.float32, device=x.t.device)
    nbytes = int(nv.query("ic2_conv_igemm_ws_bytes", dc, x.n, x.h, x.w, x.c_p, cout_p, kh, kw, pad))
    ws = torch.empty([max(nbytes, 16) // 4], dtype=torch.float32, device=x.t.device) if nbytes > 0 else None
    nv.note_flops(_conv_flops(x.n, ho, wo, cout, cin, kh, kw))
    if in_gn is not None:
        nv.call("ic2_conv3x3_gnin_gn_fwd", nv.ptr(x.t), nv.ptr(in_gn[0]), float(in_gn[1]), nv.ptr(wp), nv.ptr(y), dc,
                x.n, x.h, x.w, x.c_p, cout_p, cout, kh, kw, pad, nv.ptr(bp), norm.num_groups, float(norm.eps),
                nv.ptr(stats), nfl, nv.ptr(ws), nbytes, int(fuse), stream)
    else:
        nv.call("ic2_conv3x3_gn_fwd", nv.ptr(x.t), nv.ptr(wp), nv.ptr(y), dc, x.n, x.h, x.w, x.c_p, cout_p, cout, kh,
                kw, pad, nv.ptr(bp), norm.num_groups, float(norm.eps), nv.ptr(stats), nfl, nv.ptr(ws), nbytes,
                int(fuse), stream)
    return _Act(y, cout), stats


def _gn_in_fusable(conv: nn.Conv2d, y: _Act, dt):
    """Can conv consume lrelu(GroupNorm(y)) through ic2_conv3x3_gnin_gn_fwd (the halo conv runs the shape)?"""
    cout, cin, kh, kw = conv.weight.shape
    return (_GN_IN_FUSE and dt == torch.bfloat16 and y.t.dtype == torch.bfloat16 and
            bool(nv.query("ic2_conv3x3_gnin_supported", nv.BF16, y.n, y.h, y.w, y.c_p, nv.pad32(cout), kh, kw,
                          conv.padding[0])))


def _gn_affine_table(norm: nn.GroupNorm, y: _Act, stats, stream):
    table = torch.empty([y.n, y.c_p, 4], dtype=torch.float32, device=y.t.device)
    nv.call("ic2_gn_affine_table", nv.ptr(stats), nv.ptr(norm.weight), nv.ptr(norm.bias), y.n, y.c, y.c_p,
            norm.num_groups, nv.ptr(table), stream)
    return table


def _group_norm_lrelu(norm: nn.GroupNorm, y: _Act, pool: bool, dt, stream, slope=0.2, stats=None, split=False,
                      h2=False):
    """nn.GroupNorm -> F.leaky_relu(0.2) (-> AvgPool2d(2, 2)); `stats` from _conv_gn, else computed here.
    split: f32 arithmetic, output stored split bf16 (the next conv's operand in bf16x3 mode); with h2 rounded once to
    f16 instead (the operand of a split-weight f16 conv)."""
    groups = norm.num_groups
    if stats is None:
        nfl = int(nv.query("ic2_group_norm_stats_floats", y.n, y.h * y.w, groups))
        stats = torch.empty([nfl], dtype=torch.float32, device=y.t.device)
        nv.call("ic2_group_norm_stats", nv.ptr(y.t), nv.dtype_code(y.t.dtype), y.n, y.h * y.w, y.c_p, y.c, groups,
                float(norm.eps), nv.ptr(stats), stream)
    oh, ow = (y.h // 2, y.w // 2) if pool else (y.h, y.w)
    if split and h2:
        out = torch.empty([y.n, oh, ow, y.c_p], dtype=torch.float16, device=y.t.device)
        code = nv.F16
    else:
        out = torch.empty([y.n, oh, ow, 2 * y.c_p if split else y.c_p], dtype=dt, device=y.t.device)
        code = nv.BF16X3 if split else nv.dtype_code(dt)
    nv.call("ic2_gn_lrelu_pool", nv.ptr(y.t), nv.ptr(out), nv.dtype_code(y.t.dtype), code, y.n, y.h, y.w, y.c_p, y.c,
            groups, nv.ptr(stats), nv.ptr(norm.weight), nv.ptr(norm.bias), float(slope), int(pool), stream)
    return _Act(out, y.c, x3=split and not h2, h2=split and h2)


def _gap(x: _Act, stream):
    nfl = int(nv.query("ic2_global_avg_pool_floats", x.n, x.h * x.w, x.c_p, x.c))
    buf = torch.empty([nfl], dtype=torch.float32, device=x.t.device)
    nv.call("ic2_global_avg_pool", nv.ptr(x.t), nv.F16 if x.h2 else x.code, x.n, x.h * x.w, x.c_p, x.c, nv.ptr(buf),
            stream)
    return buf[: x.n * x.c].view(x.n, x.c)


def _linear(lin: nn.Linear, x, stream, act=False, slope=0.2):
    n = x.shape[0]
    y = torch.empty([n, lin.out_features], dtype=torch.float32, device=x.device)
    nv.call("ic2_fc", nv.ptr(x), x.shape[1], nv.ptr(lin.weight), nv.ptr(lin.bias), nv.ptr(y), n, lin.in_features,
            lin.out_features, 1.0, 1.0, nv.ACT_LRELU if act else nv.ACT_LINEAR, float(slope), 1.0, stream)
    return y


def _to_nhwc(x, dt, stream, c_p=None):
    n, c, h, w = x.shape
    c_p = nv.pad32(c) if c_p is None else c_p
    out = torch.empty([n, h, w, c_p], dtype=dt, device=x.device)
    nv.call("ic2_nchw_to_nhwc", nv.ptr(x), nv.ptr(out), nv.dtype_code(dt), n, c, h, w, c_p, None, stream)
    return _Act(out, c)


def _to_nchw(x: _Act, stream):
    y = torch.empty([x.n, x.c, x.h, x.w], dtype=torch.float32, device=x.t.device)
    nv.call("ic2_nhwc_to_nchw", nv.ptr(x.t), nv.dtype_code(x.t.dtype), nv.ptr(y), x.n, x.c, x.h, x.w, x.c_p, stream)
    return y


def _check_input(x):
    x = x.to(torch.float32).contiguous()
    nv.require_gpu(x)
    return x


# ================================================================================================
class HVAE_VGG_Encoder(nn.Module):
    """Full VGG-style HVAE encoder (ref ``stylegan3_hvae_full.py:29-167``)."""

    def __init__(self, img_resolution=1024, img_channels=3, w_dim=512, num_ws=16, block_split=(5, 12),
                 channel_base=32768, channel_max=512, use_fp16=False, precision="fp32", fix_fine_projector=False):
        """Extensions (not in the reference), both opt-in:
        precision: 'fp32' (parity, exact-f32 MFMA), 'bf16' (bf16 storage and MFMA), 'bf16x3' (split bf16: three bf16
            MFMA terms per product, f32 storage -- latents at fp32 level, the 8-bit indices of the fp32 reference;
            DESIGN.md (c)), 'f16' (f16 storage and MFMA: the training precision of BASELINE config 5, used with a
            loss scaler as the reference's fp16 autocast + GradScaler, stylegan3_hvae_full.py:487,669,693-696).
        fix_fine_projector: the reference builds the fine projector's fc1 for 64 inputs, receives 128 and re-creates
            fc1 with fresh random weights on every call (:225-230, SURVEY.md 5 bug 1).  True builds fc1 for the
            pooled width once, right after the reference's construction (so every other weight is still drawn as the
            reference draws it) and keeps it: slots 12-15 become deterministic and trainable, and data-parallel ranks
            agree without broadcasting fc1."""
        super().__init__()
        self.img_resolution = img_resolution
        self.img_channels = img_channels
        self.w_dim = w_dim
        self.num_ws = num_ws
        self.block_split = block_split
        self.use_fp16 = use_fp16
        self.precision = precision
        nv.encoder_dtype(precision)
        self.num_layers = int(np.log2(img_resolution))
        channels = {}
        for res in range(self.num_layers + 1):
            channels[res] = min(channel_max, channel_base // (2 ** (self.num_layers - res)))
        self.from_rgb = nn.Conv2d(img_channels, channels[0], kernel_size=3, padding=1)
        self.blocks = nn.ModuleList()
        for i in range(self.num_layers):
            in_channels = channels[i]
            out_channels = channels[i + 1] if i < self.num_layers - 1 else channels[i]
            self.blocks.append(VGGBlock(in_channels, out_channels))
        self.hierarchy_blocks = {"fine": 1, "medium": 4, "global": self.num_layers - 1}
        self.num_ws_global = block_split[0]
        self.num_ws_medium = block_split[1] - block_split[0]
        self.num_ws_fine = num_ws - block_split[1]
        self.global_projector = HierarchyProjector(channels[self.hierarchy_blocks["global"]], w_dim, self.num_ws_global)
        self.medium_projector = HierarchyProjector(channels[self.hierarchy_blocks["medium"]], w_dim, self.num_ws_medium)
        self.fine_projector = HierarchyProjector(channels[self.hierarchy_blocks["fine"]], w_dim, self.num_ws_fine)
        self.fix_fine_projector = fix_fine_projector
        if fix_fine_projector:
            # the width the fine projector actually pools: the output of block `fine` (channels[fine + 1])
            for proj, key in ((self.global_projector, "global"), (self.medium_projector, "medium"),
                              (self.fine_projector, "fine")):
                blk = self.hierarchy_blocks[key]
                width = channels[blk + 1] if blk < self.num_layers - 1 else channels[blk]
                if width != proj.in_channels:
                    proj.fc1 = nn.Linear(width, 256)
                    proj.in_channels = width
        self._cache = {}

    def set_precision(self, precision):
        nv.encoder_dtype(precision)
        self.precision = precision
        return self

    def features_nhwc(self, x, dt, stream, split=False):
        """from_rgb + blocks with the reference's 1x1 break; returns {'fine','medium','global'} -> _Act."""
        nh2 = _SPLIT_F16_BLOCKS if split else 0
        h = _from_rgb(self.from_rgb, x, dt, self._cache, stream, split=split, h2=nh2 > 0)
        feats = {}
        for i, block in enumerate(self.blocks):
            if h.h <= 1 or h.w <= 1:
                break
            h = block.run_nhwc(h, dt, self._cache, stream, h2=i < nh2, h2_next=i + 1 < nh2)
            if i == self.hierarchy_blocks["fine"]:
                feats["fine"] = h
            elif i == self.hierarchy_blocks["medium"]:
                feats["medium"] = h
        feats["global"] = h
        feats.setdefault("fine", h)
        feats.setdefault("medium", h)
        return feats

    def forward(self, x):
        """x [N, C, H, W] f32 in [-1, 1] -> (w_plus, means, logvars), each [N, num_ws, w_dim] f32.
        With grad mode on and a parameter or x requiring grad (the reference's training loop, :655-707) the same
        HIP kernels run under autograd (autograd_ops: HIP backward kernels); otherwise the inference path."""
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return self.forward_train(x)
        x = _check_input(x)
        dt, split = nv.encoder_dtype(self.precision)
        stream = nv.stream_of(x)
        feats = self.features_nhwc(x, dt, stream, split=split)
        n = x.shape[0]
        outs = [torch.empty([n, self.num_ws, self.w_dim], dtype=torch.float32, device=x.device) for _ in range(3)]
        off = 0
        for proj, key in ((self.global_projector, "global"), (self.medium_projector, "medium"),
                          (self.fine_projector, "fine")):
            proj.run_pooled(_gap(feats[key], stream), outs, off, self.num_ws, stream)
            off += proj.num_ws
        return tuple(outs)


    def forward_train(self, x):
        """Autograd path: NHWC activations in the module's precision, HIP forward + backward kernels per op
        ('bf16x3', an inference precision, trains in bf16)."""
        return self.heads_train(self.trunk_train(x))

    def trunk_train(self, x):
        """The autograd path's trunk: from_rgb, the blocks (with the reference's 1x1 break) and the global average
        pools of the three hierarchy features -> {'global', 'medium', 'fine'}: pooled [N, C] f32.  No randomness:
        two calls on the same input and weights give the same values, so a caller that needs the encoder twice on one
        batch (the reference's training step, :669 and :678) can run it once and the heads twice."""
        x = x.to(torch.float32)
        nv.require_gpu(x.contiguous())
        dt, _ = nv.encoder_dtype(self.precision)
        h = ao.ToNHWC.apply(x.contiguous(), dt, nv.pad32(x.shape[1]))
        h = ao.Conv2dNHWC.apply(h, self.from_rgb.weight, self.from_rgb.bias, self.from_rgb.padding[0],
                                nv.pad32(self.from_rgb.out_channels))
        c = self.from_rgb.out_channels
        feats = {}
        for i, block in enumerate(self.blocks):
            if h.shape[1] <= 1 or h.shape[2] <= 1:
                break
            h, c = block.forward_train_nhwc(h, dt)
            if i == self.hierarchy_blocks["fine"]:
                feats["fine"] = (h, c)
            elif i == self.hierarchy_blocks["medium"]:
                feats["medium"] = (h, c)
        feats["global"] = (h, c)
        feats.setdefault("fine", (h, c))
        feats.setdefault("medium", (h, c))
        return {key: ao.GlobalAvgPoolNHWC.apply(*feats[key]) for key in ("global", "medium", "fine")}

    def heads_train(self, pooled):
        """The three projectors on trunk_train's pooled features, in the reference's order (global, medium, fine:
        :160-167), each with its fc1 quirk and reparameterisation draw -> (w_plus, means, logvars)."""
        outs = []
        for proj, key in ((self.global_projector, "global"), (self.medium_projector, "medium"),
                          (self.fine_projector, "fine")):
            outs.append(proj.forward_pooled_train(pooled[key]))
        return tuple(torch.cat([o[k] for o in outs], dim=1) for k in range(3))


class VGGBlock(nn.Module):
    """conv3x3 -> GroupNorm -> lrelu(0.2), twice, then AvgPool2d(2) (ref ``:170-191``)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1)
        self.conv2 = nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1)
        self.norm1 = nn.GroupNorm(num_groups=min(32, out_channels), num_channels=out_channels)
        self.norm2 = nn.GroupNorm(num_groups=min(32, out_channels), num_channels=out_channels)
        self.pool = nn.AvgPool2d(kernel_size=2, stride=2)
        self._cache = {}

    def run_nhwc(self, x: _Act, dt, cache, stream, h2=False, h2_next=False):
        """Inference path.  Split mode (x.split): h2 = this block's conv2 takes its input in f16 against split f16
        weights, h2_next = so does the next block's conv1 (the pooled output stored f16); else split bf16."""
        split = x.split
        y, st = _conv_gn(self.conv1, self.norm1, x, dt, cache, stream)
        if not split and _gn_in_fusable(self.conv2, y, dt):
            # norm1 + lrelu applied while conv2's halo conv stages its input: lrelu(norm1(y)) never reaches HBM
            y, st = _conv_gn(self.conv2, self.norm2, y, dt, cache, stream,
                             in_gn=(_gn_affine_table(self.norm1, y, st, stream), 0.2))
        else:
            h = _group_norm_lrelu(self.norm1, y, False, dt, stream, stats=st, split=split, h2=h2)
            y, st = _conv_gn(self.conv2, self.norm2, h, dt, cache, stream)
        pool = y.h > 1 and y.w > 1
        return _group_norm_lrelu(self.norm2, y, pool, dt, stream, stats=st, split=split, h2=h2_next)

    def forward_train_nhwc(self, h, dt):
        """Autograd path of run_nhwc: (NHWC activation, valid channels) -> the same after the block."""
        y = ao.Conv2dNHWC.apply(h, self.conv1.weight, self.conv1.bias, 1, nv.pad32(self.conv1.out_channels))
        c = self.conv1.out_channels
        h = ao.GroupNormLReluPoolNHWC.apply(y, self.norm1.weight, self.norm1.bias, self.norm1.num_groups,
                                            self.norm1.eps, 0.2, False, c, dt)
        y = ao.Conv2dNHWC.apply(h, self.conv2.weight, self.conv2.bias, 1, nv.pad32(self.conv2.out_channels))
        pool = y.shape[1] > 1 and y.shape[2] > 1
        h = ao.GroupNormLReluPoolNHWC.apply(y, self.norm2.weight, self.norm2.bias, self.norm2.num_groups,
                                            self.norm2.eps, 0.2, pool, c, dt)
        return h, c

    def forward(self, x):
        xin = x
        x = _check_input(x)
        stream = nv.stream_of(x)
        y = _to_nchw(self.run_nhwc(_to_nhwc(x, torch.float32, stream), torch.float32, self._cache, stream), stream)
        return nv.refuse_backward("VGGBlock.forward", y, (xin,), (self,))


def _fresh_linear(in_features, out_features, device):
    """nn.Linear(in_features, out_features) initialised on the CPU generator exactly as the reference's
    per-call re-creation (:225-230) and moved to `device` without a host sync: the parameters go through pinned
    memory with non_blocking copies (a pageable copy would block the host until the stream drained, leaving the
    GPU idle while the host then issues the synthesis launches one by one)."""
    lin = nn.Linear(in_features, out_features)
    if device.type == "cuda":
        with torch.no_grad():
            for prm in lin.parameters():
                prm.data = prm.data.pin_memory().to(device, non_blocking=True)
    return lin


class HierarchyProjector(nn.Module):
    """GAP -> fc1 -> lrelu -> fc2 -> (mean, logvar) -> reparameterise (ref ``:194-247``)."""

    def __init__(self, in_channels, w_dim, num_ws):
        super().__init__()
        self.w_dim = w_dim
        self.num_ws = num_ws
        self.in_channels = in_channels
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Linear(in_channels, 256)
        self.act = nn.LeakyReLU(0.2)
        self.fc2 = nn.Linear(256, num_ws * w_dim * 2)

    fc1_hook = None   # callable(fc1) run after each re-creation (training.train_step: broadcast from rank 0)

    def refresh_fc1(self, in_features, device):
        """Reference quirk (:225-230): a fresh nn.Linear(in_features, 256) on EVERY call whose pooled width differs
        from in_channels, drawn from the CPU generator; then the hook (data-parallel consistency)."""
        self.fc1 = _fresh_linear(in_features, 256, device)
        if self.fc1_hook is not None:
            self.fc1_hook(self.fc1)

    def run_pooled(self, pooled, outs, off, ws_total, stream):
        """pooled [N, C] f32 -> writes slots [off, off + num_ws) of (w, mean, logvar)."""
        n, in_features = pooled.shape
        if in_features != self.in_channels:
            self.refresh_fc1(in_features, pooled.device)
        h = _linear(self.fc1, pooled, stream, act=True, slope=self.act.negative_slope)
        p = _linear(self.fc2, h, stream)
        # torch.randn_like(std) on the device, in the reference's order (global, medium, fine)
        eps = torch.randn([n, self.num_ws, self.w_dim], dtype=torch.float32, device=pooled.device)
        w_out, m_out, lv_out = outs
        nv.call("ic2_reparameterize", nv.ptr(p), nv.ptr(eps), n, self.num_ws, self.w_dim, ws_total, off, nv.ptr(w_out),
                nv.ptr(m_out), nv.ptr(lv_out), stream)

    def forward_pooled_train(self, pooled):
        """Autograd path of run_pooled (torch ops on [N, <= 512] rows): -> (w, mean, logvar)."""
        n, in_features = pooled.shape
        if in_features != self.in_channels:
            self.refresh_fc1(in_features, pooled.device)
        h = F.leaky_relu(F.linear(pooled, self.fc1.weight, self.fc1.bias), self.act.negative_slope)
        p = F.linear(h, self.fc2.weight, self.fc2.bias).view(n, self.num_ws, self.w_dim * 2)
        mean, logvar = torch.chunk(p, 2, dim=2)
        std = torch.exp(0.5 * logvar)
        eps = torch.randn([n, self.num_ws, self.w_dim], dtype=torch.float32, device=pooled.device)
        return mean + eps * std, mean, logvar

    def forward(self, x):
        xin = x
        x = _check_input(x)
        stream = nv.stream_of(x)
        n = x.shape[0]
        pooled = _gap(_to_nhwc(x, torch.float32, stream), stream).contiguous()
        outs = [torch.empty([n, self.num_ws, self.w_dim], dtype=torch.float32, device=x.device) for _ in range(3)]
        self.run_pooled(pooled, outs, 0, self.num_ws, stream)
        return nv.refuse_backward("HierarchyProjector.forward", tuple(outs), (xin,), (self,))


# ================================================================================================
def quantize_uniform(w, bits=8, return_indices=False):
    """The compress() quantizer (ref ``:313-316``) as one bit-exact HIP kernel."""
    w = w.to(torch.float32).contiguous()
    nv.require_gpu(w)
    q = torch.empty_like(w)
    idx = torch.empty(w.shape, dtype=torch.int32, device=w.device) if return_indices else None
    if w.data_ptr() % 16 or q.data_ptr() % 16:
        raise RuntimeError("quantize_uniform needs 16-byte aligned tensors")
    nv.call("ic2_quantize_uniform", nv.ptr(w), w.numel(), int(bits), nv.ptr(q), nv.ptr(idx), nv.stream_of(w))
    return (q, idx) if return_indices else q


def _resize_fwd(img, size):
    img = img.to(torch.float32).contiguous()
    nv.require_gpu(img)
    n, c, h, w = img.shape
    oh, ow = size
    out = torch.empty([n, c, oh, ow], dtype=torch.float32, device=img.device)
    nv.call("ic2_resize_bilinear", nv.ptr(img), nv.ptr(out), n * c, h, w, oh, ow, nv.stream_of(img))
    return out


class _ResizeBilinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, size):
        ctx.in_size = tuple(img.shape)
        return _resize_fwd(img, size)

    @staticmethod
    def backward(ctx, dy):
        # the adjoint of the 4-tap bilinear gather is a scatter-add: torch's own upsample backward on the device
        dx = torch.ops.aten.upsample_bilinear2d_backward(dy.contiguous(), list(dy.shape[2:]), list(ctx.in_size),
                                                         False, None, None)
        return dx, None


def resize_bilinear(img, size):
    """F.interpolate(img, size, mode='bilinear', align_corners=False) (ref ``:277-279``); differentiable (the
    compressor's training forward resizes the synthesized image back to the training resolution)."""
    if torch.is_grad_enabled() and img.requires_grad:
        return _ResizeBilinear.apply(img, tuple(size))
    return _resize_fwd(img, size)


class StyleGAN3Compressor(nn.Module):
    """Encoder + frozen StyleGAN3 generator codec (ref ``:250-380``)."""

    def __init__(self, encoder, generator, training_resolution=None):
        super().__init__()
        self.encoder = encoder
        self.generator = generator
        self.training_resolution = training_resolution
        for param in generator.parameters():
            param.requires_grad = False

    def forward(self, x, noise_mode="const"):
        w_plus, _, _ = self.encoder(x)
        img = self.generator.synthesis(w_plus, noise_mode=noise_mode)
        if self.training_resolution is not None and img.shape[2] != x.shape[2]:
            img = resize_bilinear(img, (x.shape[2], x.shape[3]))
        return img, w_plus

    def encode(self, x, deterministic=False):
        w_plus, means, _ = self.encoder(x)
        return means if deterministic else w_plus

    def compress(self, x, quantization_bits=8, deterministic=True):
        # an inference API whose output is rounded (zero gradient in the reference too): run without a graph
        with torch.no_grad():
            if deterministic:
                _, w_plus, _ = self.encoder(x)
            else:
                w_plus, _, _ = self.encoder(x)
            return quantize_uniform(w_plus, quantization_bits)

    def decompress(self, w_plus, noise_mode="const"):
        return self.generator.synthesis(w_plus, noise_mode=noise_mode)

    def save_compressed(self, x, filename, quantization_bits=8, deterministic=True):
        """Same .npz container as the reference (keys w, resolution, bits, orig_size, comp_size,
        compression_ratio; ref ``:331-361``)."""
        w_quantized = self.compress(x, quantization_bits, deterministic)
        w_quantized_np = w_quantized.detach().cpu().numpy()
        orig_size = x.numel() * 4
        comp_size = w_quantized.numel() * (quantization_bits / 8)
        np.savez_compressed(filename, w=w_quantized_np, resolution=x.shape[2:4], bits=quantization_bits,
                            orig_size=orig_size, comp_size=comp_size, compression_ratio=orig_size / comp_size)
        return orig_size, comp_size, orig_size / comp_size

    def load_compressed(self, filename, noise_mode="const"):
        data = np.load(filename)  # allow_pickle=False (default): plain arrays only
        w_quantized = torch.tensor(data["w"]).to(next(self.generator.parameters()).device)
        with torch.no_grad():
            img = self.decompress(w_quantized, noise_mode=noise_mode)
        return img, data["compression_ratio"]


def save_tensor_as_image(tensor, filename):
    """Tensor [C, H, W] in [-1, 1] -> PNG, exactly as the reference (no clamp; ref ``:923-932``)."""
    img = tensor.detach().cpu().numpy()
    img = ((img.transpose(1, 2, 0) + 1.0) * 127.5).astype(np.uint8)
    Image.fromarray(img).save(filename)
