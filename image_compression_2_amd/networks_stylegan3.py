"""MI355X-native StyleGAN3-T generator: the ``G_ema`` duck type the reference decodes with.

The reference unpickles NVlabs' ``G_ema`` (/root/reference/stylegan3_hvae_full.py:454-455) and calls
``G.synthesis(ws, noise_mode=...)`` (``:274, :329``; ``gumbel_softmax_compression.py:193, 262``),
``G.mapping`` / ``G.mapping.w_avg`` (``:557, :626``), ``G(z, c)`` (``:561``), ``G.parameters()``
(``:262``) and ``.z_dim/.w_dim/.num_ws/.img_resolution/.img_channels`` (``:459-468``).  This module
provides the same module tree (state-dict keys ``synthesis.L0_36_512.affine.weight`` ...), the same
seeded parameter construction order, and a forward that runs entirely in libic2ops HIP kernels:

    per layer:  styles = FC(w)                        ic2_fc
                xscale / oscale (mod / demod)         ic2_modconv_prep
                y = oscale * conv(W_norm, x) + bias   ic2_conv_igemm   (MFMA, NHWC)
                x = filtered_lrelu(y) * xscale_next   ic2_flrelu_nhwc  (fused FIR, NHWC)

``precision='bf16'`` stores activations and weights in bf16 (fp32 accumulate; the conv output that feeds
the filtered lrelu is f16, whose FIR runs on MFMA with f16 operands and fp32 accumulation);
``precision='f16'`` is the same pipeline with f16 activations and weights throughout (11-bit significands: about
20 dB more synthesis SNR than bf16 at the same MFMA rate; outputs saturate at +-65504, far above conv_clamp);
inference only (the autograd path trains in bf16).  ``precision='fp32'`` (default) is the parity mode (exact-fp32 MFMA).

With grad mode on and ``ws`` requiring grad (the reference's encoder training backpropagates through the
frozen generator, :669-696) ``SynthesisNetwork.forward`` takes the autograd path ``forward_train``: the same
conv / filtered-lrelu kernels with HIP backward passes (autograd_ops), gradients w.r.t. ws only.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import scipy.signal
import torch
import torch.nn.functional as F

from . import _native as nv
from . import autograd_ops as ao
from . import sg3_ops

# conv -> filtered lrelu hand-off in the channel-blocked NHWC16 layout (bf16 mode); knob IC2_FLR_BLOCKED=0 (IC2_DEV=1):
# plain NHWC
_FLR_BLOCKED = nv.knob("IC2_FLR_BLOCKED", 1) != 0
# longest row (w_dim, cin) of ic2_modconv_prep_batched's LDS-staged small GEMM (synth_ops.hip kSmK)
_MOD_BATCH_MAX = 512


def _train_mode(module, *tensors):
    """Autograd path wanted: grad mode on, an input requires grad and the module's weights are frozen (the
    reference trains its encoder through a frozen G, stylegan3_hvae_full.py:259-261).  With unfrozen weights the
    inference path runs and its output refuses backward (_refuse): gradients w.r.t. the generator's weights are
    not implemented."""
    if not torch.is_grad_enabled():
        return False
    if any(p.requires_grad for p in module.parameters()):
        return False
    return any(t is not None and t.requires_grad for t in tensors)


def _refuse(module, out, *tensors):
    return nv.refuse_backward(type(module).__name__ + ".forward", out, tensors, (module,))


def _version_key(*tensors):
    return tuple((t.data_ptr(), t._version, t.device) for t in tensors)


# ------------------------------------------------------------------------------------------------
class FullyConnectedLayer(torch.nn.Module):
    """[SG3-public] y = x @ (W * lr/sqrt(in))^T + b * lr, optional lrelu (bias_act)."""

    def __init__(self, in_features, out_features, activation="linear", bias=True, lr_multiplier=1, weight_init=1,
                 bias_init=0):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.activation = activation
        self.weight = torch.nn.Parameter(torch.randn([out_features, in_features]) * (weight_init / lr_multiplier))
        bias_init = np.broadcast_to(np.asarray(bias_init, dtype=np.float32), [out_features])
        self.bias = torch.nn.Parameter(torch.from_numpy(bias_init / lr_multiplier)) if bias else None
        self.weight_gain = lr_multiplier / np.sqrt(in_features)
        self.bias_gain = lr_multiplier

    def run(self, x, out=None, ldx=None, n=None):
        """x: f32 [n, ldx] rows (only the first in_features of each row are read)."""
        n = x.shape[0] if n is None else n
        ldx = self.in_features if ldx is None else ldx
        if out is None:
            out = torch.empty([n, self.out_features], dtype=torch.float32, device=x.device)
        act = nv.ACT_LRELU if self.activation == "lrelu" else nv.ACT_LINEAR
        nv.call("ic2_fc", nv.ptr(x), ldx, nv.ptr(self.weight), nv.ptr(self.bias), nv.ptr(out), n, self.in_features,
                self.out_features, float(self.weight_gain), float(self.bias_gain), act, 0.2,
                float(np.sqrt(2)) if act == nv.ACT_LRELU else 1.0, nv.stream_of(x))
        return out

    def forward(self, x):
        xin = x
        x = x.to(torch.float32).contiguous()
        nv.require_gpu(x)
        if self.activation not in ("linear", "lrelu"):
            raise NotImplementedError(self.activation)
        return _refuse(self, self.run(x), xin)

    def extra_repr(self):
        return f"in_features={self.in_features:d}, out_features={self.out_features:d}, activation={self.activation:s}"


# ------------------------------------------------------------------------------------------------
class MappingNetwork(torch.nn.Module):
    """[SG3-public] z -> w (2 lrelu FCs, lr 0.01), w_avg, truncation.  Not on the encode->decode path
    (SURVEY.md 2 #9); provided for the Generator duck type (``G.mapping``, ``G.mapping.w_avg``)."""

    def __init__(self, z_dim, c_dim, w_dim, num_ws, num_layers=2, lr_multiplier=0.01, w_avg_beta=0.998):
        super().__init__()
        if c_dim:
            raise NotImplementedError("conditional mapping (c_dim > 0) is not on the path")
        self.z_dim, self.c_dim, self.w_dim, self.num_ws = z_dim, c_dim, w_dim, num_ws
        self.num_layers, self.w_avg_beta = num_layers, w_avg_beta
        features = [z_dim] + [w_dim] * num_layers
        for idx, in_f, out_f in zip(range(num_layers), features[:-1], features[1:]):
            setattr(self, f"fc{idx}", FullyConnectedLayer(in_f, out_f, activation="lrelu", lr_multiplier=lr_multiplier))
        self.register_buffer("w_avg", torch.zeros([w_dim]))

    def forward(self, z, c=None, truncation_psi=1, truncation_cutoff=None, update_emas=False):
        if update_emas:
            raise NotImplementedError("update_emas is a training feature (out of scope)")
        x = z.to(torch.float32).contiguous()
        nv.require_gpu(x)
        x = x * (x.square().mean(1, keepdim=True) + 1e-8).rsqrt()
        for idx in range(self.num_layers):
            x = getattr(self, f"fc{idx}").run(x.contiguous())
        x = x.unsqueeze(1).repeat([1, self.num_ws, 1])
        if truncation_psi != 1:
            cut = self.num_ws if truncation_cutoff is None else truncation_cutoff
            x[:, :cut] = self.w_avg.lerp(x[:, :cut], truncation_psi)
        return _refuse(self, x, z)


# ------------------------------------------------------------------------------------------------
class SynthesisInput(torch.nn.Module):
    """[SG3-public] Fourier-feature input; buffers/params drawn in SG3's order."""

    def __init__(self, w_dim, channels, size, sampling_rate, bandwidth):
        super().__init__()
        self.w_dim = w_dim
        self.channels = channels
        self.size = np.broadcast_to(np.asarray(size), [2])
        self.sampling_rate = sampling_rate
        self.bandwidth = bandwidth
        freqs = torch.randn([self.channels, 2])
        radii = freqs.square().sum(dim=1, keepdim=True).sqrt()
        freqs /= radii * radii.square().exp().pow(0.25)
        freqs *= bandwidth
        phases = torch.rand([self.channels]) - 0.5
        self.weight = torch.nn.Parameter(torch.randn([self.channels, self.channels]))
        self.affine = FullyConnectedLayer(w_dim, 4, weight_init=0, bias_init=[1, 0, 0, 0])
        self.register_buffer("transform", torch.eye(3, 3))
        self.register_buffer("freqs", freqs)
        self.register_buffer("phases", phases)
        self._cache = {}

    def packed_weight(self, dt):
        key = (dt, _version_key(self.weight))
        hit = self._cache.get(dt)
        if hit is not None and hit[0] == key:
            return hit[1]
        C, cp = self.channels, nv.pad_synth(self.channels)
        w = self.weight.detach().to(torch.float32).contiguous()
        out = torch.empty([cp, cp], dtype=dt, device=w.device)
        nv.call("ic2_pack_weight", nv.ptr(w), C, C, 1, 1, cp, cp, 0, float(1 / np.sqrt(C)), nv.ptr(out),
                nv.dtype_code(dt), None, nv.stream_of(w))
        self._cache[dt] = (key, out)
        return out

    def run_nhwc(self, ws, ldx, n, dt, post_scale):
        """Features -> NHWC [n, S, S, c_p] (dt), scaled by the first layer's xscale (post_scale)."""
        C, cp, S = self.channels, nv.pad_synth(self.channels), int(self.size[0])
        dev = ws.device
        t = self.affine.run(ws, ldx=ldx, n=n)
        feats = torch.empty([n, S, S, cp], dtype=dt, device=dev)
        nv.call("ic2_synth_input_features", nv.ptr(t), nv.ptr(self.freqs), nv.ptr(self.phases), nv.ptr(self.transform),
                n, C, cp, S, float(self.sampling_rate), float(self.bandwidth), nv.ptr(feats), nv.dtype_code(dt),
                nv.stream_of(ws))
        out = torch.empty([n, S, S, cp], dtype=dt, device=dev)
        w = self.packed_weight(dt)
        nv.note_flops(2 * n * S * S * C * C)
        nv.conv_igemm(nv.ptr(feats), nv.ptr(w), nv.ptr(out), nv.dtype_code(dt), nv.dtype_code(dt), n, S, S, cp, cp, C,
                      1, 1, 0, S, S, nv.ptr(post_scale), None, 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(ws),
                      feats.device)
        return out

    def _train_grid(self, device):
        """The sampling grid of the Fourier features (constant): built once per device.  Built on every call, its
        host-side theta was a blocking host-to-device copy that drained the stream once per training step."""
        g = getattr(self, "_grid_cache", None)
        if g is None or g.device != device:
            S = int(self.size[0])
            theta = torch.tensor([[0.5 * S / self.sampling_rate, 0, 0], [0, 0.5 * S / self.sampling_rate, 0]],
                                 dtype=torch.float32)
            g = F.affine_grid(theta.unsqueeze(0), [1, 1, S, S], align_corners=False).to(device)
            self._grid_cache = g
        return g

    def forward_train_nhwc(self, w, dt=torch.float32):
        """Autograd path: w [n, w_dim] -> NHWC [n, S, S, C] features (dt), as torch ops (SG3
        SynthesisInput.forward: affine -> rotation/translation of the Fourier frequencies -> sin features with
        the bandwidth taper -> 1x1 mix by weight / sqrt(C); the grid is 36 x 36 and the rows are <= 512 wide).
        A 16-bit dt runs the 1x1 mix (n * 1296 x 512 x 512, and its input gradient) on 16-bit operands, as the
        reference's fp16 autocast does; in f32 the library GEMMs took 0.9 ms of the C5 step."""
        A = self.affine
        t = F.linear(w, A.weight * float(A.weight_gain), A.bias * float(A.bias_gain))
        t = t / t[:, :2].norm(dim=1, keepdim=True)
        zero, one = torch.zeros_like(t[:, 0]), torch.ones_like(t[:, 0])
        m_r = torch.stack([torch.stack([t[:, 0], -t[:, 1], zero], 1), torch.stack([t[:, 1], t[:, 0], zero], 1),
                           torch.stack([zero, zero, one], 1)], 1)
        m_t = torch.stack([torch.stack([one, zero, -t[:, 2]], 1), torch.stack([zero, one, -t[:, 3]], 1),
                           torch.stack([zero, zero, one], 1)], 1)
        transforms = m_r @ m_t @ self.transform.float().unsqueeze(0)
        freqs = self.freqs.float().unsqueeze(0)
        phases = self.phases.float().unsqueeze(0) + (freqs @ transforms[:, :2, 2:]).squeeze(2)
        freqs = freqs @ transforms[:, :2, :2]
        amplitudes = (1 - (freqs.norm(dim=2) - self.bandwidth) / (self.sampling_rate / 2 - self.bandwidth)).clamp(0, 1)
        grids = self._train_grid(w.device)  # [1, S, S, 2]
        # grid . freq as two broadcast products (a K = 2 batched matmul here, and its backward over the 36 x 36 grid,
        # ran as two ~0.45 ms library GEMMs per C5 step)
        x = grids[0, :, :, 0, None] * freqs[:, None, None, :, 0] + grids[0, :, :, 1, None] * freqs[:, None, None, :, 1]
        x = torch.sin((x + phases[:, None, None, :]) * (np.pi * 2)) * amplitudes[:, None, None, :]
        wt = (self.weight.float() / np.sqrt(self.channels)).t()
        return x @ wt if dt == torch.float32 else x.to(dt) @ wt.to(dt)

    def forward(self, w):
        if _train_mode(self, w):
            return self.forward_train_nhwc(w.to(torch.float32)).permute(0, 3, 1, 2).contiguous()
        w_in = w
        w = w.to(torch.float32).contiguous()
        nv.require_gpu(w)
        n, S, C, cp = w.shape[0], int(self.size[0]), self.channels, nv.pad_synth(self.channels)
        x = self.run_nhwc(w, self.w_dim, n, torch.float32, None)
        y = torch.empty([n, C, S, S], dtype=torch.float32, device=w.device)
        nv.call("ic2_nhwc_to_nchw", nv.ptr(x), nv.F32, nv.ptr(y), n, C, S, S, cp, nv.stream_of(w))
        return _refuse(self, y, w_in)

    def extra_repr(self):
        return (f"w_dim={self.w_dim:d}, channels={self.channels:d}, size={list(self.size)}, "
                f"sampling_rate={self.sampling_rate:g}, bandwidth={self.bandwidth:g}")


# ------------------------------------------------------------------------------------------------
class SynthesisLayer(torch.nn.Module):
    """[SG3-public] modulated conv + filtered lrelu; same constructor and derived hyper-parameters."""

    def __init__(self, w_dim, is_torgb, is_critically_sampled, use_fp16, in_channels, out_channels, in_size, out_size,
                 in_sampling_rate, out_sampling_rate, in_cutoff, out_cutoff, in_half_width, out_half_width,
                 conv_kernel=3, filter_size=6, lrelu_upsampling=2, use_radial_filters=False, conv_clamp=256,
                 magnitude_ema_beta=0.999):
        super().__init__()
        if use_radial_filters and not is_critically_sampled and not is_torgb:
            raise NotImplementedError("radial (StyleGAN3-R) filters are not on the path: StyleGAN3-T only")
        self.w_dim = w_dim
        self.is_torgb = is_torgb
        self.is_critically_sampled = is_critically_sampled
        self.use_fp16 = use_fp16
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.in_size = np.broadcast_to(np.asarray(in_size), [2])
        self.out_size = np.broadcast_to(np.asarray(out_size), [2])
        self.in_sampling_rate = in_sampling_rate
        self.out_sampling_rate = out_sampling_rate
        self.tmp_sampling_rate = max(in_sampling_rate, out_sampling_rate) * (1 if is_torgb else lrelu_upsampling)
        self.in_cutoff = in_cutoff
        self.out_cutoff = out_cutoff
        self.in_half_width = in_half_width
        self.out_half_width = out_half_width
        self.conv_kernel = 1 if is_torgb else conv_kernel
        self.conv_clamp = conv_clamp
        self.magnitude_ema_beta = magnitude_ema_beta

        self.affine = FullyConnectedLayer(self.w_dim, self.in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn([self.out_channels, self.in_channels, self.conv_kernel,
                                                      self.conv_kernel]))
        self.bias = torch.nn.Parameter(torch.zeros([self.out_channels]))
        self.register_buffer("magnitude_ema", torch.ones([]))

        self.up_factor = int(np.rint(self.tmp_sampling_rate / self.in_sampling_rate))
        assert self.in_sampling_rate * self.up_factor == self.tmp_sampling_rate
        self.up_taps = filter_size * self.up_factor if self.up_factor > 1 and not self.is_torgb else 1
        self.register_buffer("up_filter", self.design_lowpass_filter(
            numtaps=self.up_taps, cutoff=self.in_cutoff, width=self.in_half_width * 2, fs=self.tmp_sampling_rate))
        self.down_factor = int(np.rint(self.tmp_sampling_rate / self.out_sampling_rate))
        assert self.out_sampling_rate * self.down_factor == self.tmp_sampling_rate
        self.down_taps = filter_size * self.down_factor if self.down_factor > 1 and not self.is_torgb else 1
        self.down_radial = use_radial_filters and not self.is_critically_sampled
        self.register_buffer("down_filter", self.design_lowpass_filter(
            numtaps=self.down_taps, cutoff=self.out_cutoff, width=self.out_half_width * 2, fs=self.tmp_sampling_rate))

        pad_total = (self.out_size - 1) * self.down_factor + 1
        pad_total -= (self.in_size + self.conv_kernel - 1) * self.up_factor
        pad_total += self.up_taps + self.down_taps - 2
        pad_lo = (pad_total + self.up_factor) // 2
        pad_hi = pad_total - pad_lo
        self.padding = [int(pad_lo[0]), int(pad_hi[0]), int(pad_lo[1]), int(pad_hi[1])]

        # filtered_lrelu gain (SG3 default sqrt(2) for the lrelu layers; ToRGB runs linear, gain 1)
        self.act_gain = 1.0 if self.is_torgb else float(np.sqrt(2))
        # host copies of the (constant) FIR taps: the fused kernel takes them by value
        self._fu = None if self.up_filter is None else np.ascontiguousarray(self.up_filter.numpy(), np.float32)
        self._fd = None if self.down_filter is None else np.ascontiguousarray(self.down_filter.numpy(), np.float32)
        self._cache = {}
        self._ig_cache = None

    # ---- constants -------------------------------------------------------------------------
    @property
    def cin_p(self):
        return nv.pad_synth(self.in_channels)

    @property
    def cout_p(self):
        return nv.pad_synth(self.out_channels)

    def input_gain(self):
        key = _version_key(self.magnitude_ema)
        if self._ig_cache is None or self._ig_cache[0] != key:
            self._ig_cache = (key, float(self.magnitude_ema.detach().float().rsqrt().cpu()))
        return self._ig_cache[1]

    def packed(self, dt):
        """(W packed [cout_p][k][k][cin_p] dt, wsq [cout][cin] f32, bias_p [cout_p] f32) per weight version."""
        key = (dt, _version_key(self.weight, self.bias))
        hit = self._cache.get(dt)
        if hit is not None and hit[0] == key:
            return hit[1]
        w = self.weight.detach().to(torch.float32).contiguous()
        k = self.conv_kernel
        wp = torch.empty([self.cout_p, k, k, self.cin_p], dtype=dt, device=w.device)
        wsq = torch.empty([self.out_channels, self.in_channels], dtype=torch.float32, device=w.device)
        nv.call("ic2_pack_weight", nv.ptr(w), self.out_channels, self.in_channels, k, k, self.cout_p, self.cin_p,
                int(not self.is_torgb), 1.0, nv.ptr(wp), nv.dtype_code(dt), nv.ptr(wsq), nv.stream_of(w))
        bp = torch.zeros([self.cout_p], dtype=torch.float32, device=w.device)
        bp[: self.out_channels] = self.bias.detach().float()
        val = (wp, wsq, bp)
        self._cache[dt] = (key, val)
        return val

    def mod_record(self, dt, ws_off, styles, xs, os_):
        """This layer's ic2_modconv_prep_batched record (16 int64, see include/ic2ops.h)."""
        _, wsq, _ = self.packed(dt)
        fc = self.affine
        style_gain = float(1 / np.sqrt(self.in_channels * (self.conv_kernel ** 2))) if self.is_torgb else 1.0
        f32 = lambda v: int(np.float32(v).view(np.uint32))  # noqa: E731
        dp = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        return [dp(fc.weight), dp(fc.bias), dp(wsq), dp(styles), dp(xs), dp(os_), ws_off, self.in_channels, self.cin_p,
                self.out_channels, self.cout_p, int(not self.is_torgb), f32(fc.weight_gain), f32(fc.bias_gain),
                f32(style_gain), f32(self.input_gain())]

    def batchable(self):
        """Fits ic2_modconv_prep_batched's LDS-staged small GEMM (rows of <= 512: w_dim and cin)."""
        return self.in_channels <= _MOD_BATCH_MAX and self.affine.in_features <= _MOD_BATCH_MAX

    def scales(self, ws, ldx, n, dt, unbatched=False):
        """Runs the affine FC and the (de)modulation prep: -> (xscale [n][cin_p], oscale [n][cout_p]).
        The same kernels as SynthesisNetwork.scales_batched (a one-layer batch), so both give identical bits; a
        layer wider than that kernel's rows (channel_max > 512) -- or unbatched=True -- takes the
        per-layer kernels ic2_fc + ic2_modconv_prep (no width cap)."""
        dev = ws.device
        styles = torch.empty([n, self.in_channels], dtype=torch.float32, device=dev)
        xs = torch.empty([n, self.cin_p], dtype=torch.float32, device=dev)
        os_ = torch.empty([n, self.cout_p], dtype=torch.float32, device=dev)
        if unbatched or not self.batchable():
            _, wsq, _ = self.packed(dt)
            fc = self.affine
            stream = nv.stream_of(ws)
            nv.call("ic2_fc", nv.ptr(ws), ldx, nv.ptr(fc.weight), nv.ptr(fc.bias), nv.ptr(styles), n, fc.in_features,
                    self.in_channels, float(fc.weight_gain), float(fc.bias_gain), nv.ACT_LINEAR, 0.0, 1.0, stream)
            style_gain = float(1 / np.sqrt(self.in_channels * (self.conv_kernel ** 2))) if self.is_torgb else 1.0
            nv.call("ic2_modconv_prep", nv.ptr(styles), nv.ptr(wsq), n, self.in_channels, self.out_channels,
                    self.cin_p, self.cout_p, int(not self.is_torgb), style_gain, float(self.input_gain()), nv.ptr(xs),
                    nv.ptr(os_), None, stream)
            return xs, os_
        rec = np.asarray([self.mod_record(dt, 0, styles, xs, os_)], dtype=np.int64)
        nv.call("ic2_modconv_prep_batched", nv.ptr(ws), ldx, n, self.affine.in_features, 1,
                rec.ctypes.data_as(ctypes.c_void_p), nv.stream_of(ws))
        return xs, os_

    # ---- NHWC pipeline step ------------------------------------------------------------------
    def run_nhwc(self, x, n, dt, oscale, post_scale, final_scale=None):
        """x: NHWC [n, in, in, cin_p] already scaled by this layer's xscale.  Returns NHWC output scaled by
        post_scale (next layer's xscale), or -- for ToRGB -- the final NCHW f32 image * final_scale."""
        s_in = int(self.in_size[0])
        k = self.conv_kernel
        pad = k - 1
        conv = s_in + 2 * pad - k + 1
        wp, _, bp = self.packed(dt)
        stream = nv.stream_of(x)
        nv.note_flops(2 * n * conv * conv * self.out_channels * self.in_channels * k * k)
        if self.is_torgb:
            assert self.up_factor == 1 and self.down_factor == 1 and self.padding == [0, 0, 0, 0]
            out = torch.empty([n, self.out_channels, conv, conv], dtype=torch.float32, device=x.device)
            clamp = float(self.conv_clamp) if self.conv_clamp is not None else -1.0
            nv.conv_igemm(nv.ptr(x), nv.ptr(wp), nv.ptr(out), nv.dtype_code(dt), nv.F32, n, s_in, s_in, self.cin_p,
                          self.cout_p, self.out_channels, k, k, pad, conv, conv, nv.ptr(oscale), nv.ptr(bp),
                          nv.ACT_LRELU, 1.0, 1.0, clamp, float(1.0 if final_scale is None else final_scale), nv.NCHW,
                          stream, x.device)
            return out
        y, blocked = self.conv_nhwc(x, n, dt, oscale)
        return self.flrelu_nhwc(y, dt, post_scale, blocked=blocked)

    def conv_nhwc(self, x, n, dt, oscale):
        """The modulated conv of a non-ToRGB layer: -> (conv output y, blocked layout?) for flrelu_nhwc."""
        s_in = int(self.in_size[0])
        k = self.conv_kernel
        pad = k - 1
        conv = s_in + 2 * pad - k + 1
        wp, _, bp = self.packed(dt)
        stream = nv.stream_of(x)
        # bf16 / f16 mode: the conv output feeds the MFMA filtered-lrelu, whose operands are f16 -> store it as f16, in
        # the channel-blocked layout [n][cout_p/16][conv][conv][16] the fused kernel's 16-channel tiles read as
        # contiguous rows (IC2_FLR_BLOCKED=0: plain NHWC)
        ydt = torch.float16 if dt in (torch.bfloat16, torch.float16) else dt
        blocked = ydt == torch.float16 and _FLR_BLOCKED
        if blocked:
            y = torch.empty([n, self.cout_p // 16, conv, conv, 16], dtype=ydt, device=x.device)
        else:
            y = torch.empty([n, conv, conv, self.cout_p], dtype=ydt, device=x.device)
        layout = nv.NHWC16 if blocked else nv.NHWC
        if nv.wino_preferred(nv.dtype_code(dt), n, s_in, s_in, self.cin_p, self.cout_p, k, k, pad):
            # f16, >= 256 channels: the fused Winograd F(2,3)-along-x kernel (2/3 of the MFMA work, wino.hip)
            nv.conv_wino(nv.ptr(x), nv.ptr(self.packed_wino()), nv.ptr(y), nv.F16, nv.dtype_code(ydt), n, s_in, s_in,
                         self.cin_p, self.cout_p, self.out_channels, pad, conv, conv, nv.ptr(oscale), nv.ptr(bp), 0,
                         0.0, 1.0, -1.0, 1.0, layout, stream)
        else:
            nv.conv_igemm(nv.ptr(x), nv.ptr(wp), nv.ptr(y), nv.dtype_code(dt), nv.dtype_code(ydt), n, s_in, s_in,
                          self.cin_p, self.cout_p, self.out_channels, k, k, pad, conv, conv, nv.ptr(oscale),
                          nv.ptr(bp), 0, 0.0, 1.0, -1.0, 1.0, layout, stream, x.device)
        return y, blocked

    def packed_wino(self):
        """Winograd F(2,3)-along-x weights U [cout_p][3][4][cin_p] f16 of the pre-normalised W, per weight version
        (ic2_pack_weight_wino, from the f32 master weights: one rounding)."""
        key = _version_key(self.weight)
        hit = self._cache.get("wino")
        if hit is not None and hit[0] == key:
            return hit[1]
        w = self.weight.detach().to(torch.float32).contiguous()
        u = torch.empty([self.cout_p, 3, 4, self.cin_p], dtype=torch.float16, device=w.device)
        nv.call("ic2_pack_weight_wino", nv.ptr(w), self.out_channels, self.in_channels, self.cout_p, self.cin_p,
                int(not self.is_torgb), 1.0, nv.ptr(u), nv.F16, nv.stream_of(w))
        self._cache["wino"] = (key, u)
        return u

    def flrelu_nhwc(self, y, dt_out, post_scale=None, blocked=False):
        """The layer's filtered lrelu on the conv output y NHWC [n, conv, conv, cout_p] (f32, or f16 for the
        MFMA kernel; blocked: f16/bf16 [n, cout_p/16, conv, conv, 16]) -> NHWC [n, out, out, cout_p] dt_out, times
        post_scale [n][cout_p] when given."""
        n, conv = y.shape[0], y.shape[2 if blocked else 1]
        s_out = int(self.out_size[0])
        out = torch.empty([n, s_out, s_out, self.cout_p], dtype=dt_out, device=y.device)
        fu = self._fu
        fd = self._fd
        px0, px1, py0, py1 = self.padding
        clamp = float(self.conv_clamp) if self.conv_clamp is not None else -1.0
        nv.call("ic2_flrelu_nhwc16" if blocked else "ic2_flrelu_nhwc", nv.ptr(y), nv.ptr(out), nv.dtype_code(y.dtype),
                nv.dtype_code(dt_out), n,
                self.cout_p, conv, conv, s_out, s_out, None if fu is None else fu.ctypes.data_as(ctypes.c_void_p),
                1 if fu is None else fu.shape[0], None if fd is None else fd.ctypes.data_as(ctypes.c_void_p),
                1 if fd is None else fd.shape[0], None, self.up_factor, self.down_factor, px0, px1, py0, py1,
                float(self.act_gain), 0.2, clamp, 0, nv.ptr(post_scale), nv.stream_of(y))
        return out

    # ---- autograd path: gradients w.r.t. the input activation and w (weights frozen) ----------------------
    def packed_adjoint(self, dt):
        """The dgrad weights: normalised W flipped in space, transposed in channels, packed
        [cin_p][k][k][cout_p] (dt) -- the forward igemm on these is the modulated conv's adjoint."""
        key = (dt, _version_key(self.weight))
        hit = self._cache.get(("adj", dt))
        if hit is not None and hit[0] == key:
            return hit[1]
        w = self.weight.detach().to(torch.float32)
        if not self.is_torgb:
            w = w * w.square().mean(dim=[1, 2, 3], keepdim=True).rsqrt()
        wt = ao.pack_conv_weight(w.transpose(0, 1).flip(2, 3), self.cout_p, self.cin_p, dt)
        self._cache[("adj", dt)] = (key, wt)
        return wt

    def packed_adjoint_wino(self, scale=1.0):
        """packed_adjoint for the Winograd kernel: U [cin_p][3][4][cout_p] f16 of the normalised W flipped in space
        and transposed in channels (ic2_pack_weight_wino on the f32 adjoint, no further normalisation), times `scale`."""
        key = (_version_key(self.weight), scale)
        hit = self._cache.get(("adj_wino", scale))
        if hit is not None and hit[0] == key:
            return hit[1]
        w = self.weight.detach().to(torch.float32)
        if not self.is_torgb:
            w = w * w.square().mean(dim=[1, 2, 3], keepdim=True).rsqrt()
        wa = w.transpose(0, 1).flip(2, 3).contiguous()
        u = torch.empty([self.cin_p, 3, 4, self.cout_p], dtype=torch.float16, device=w.device)
        nv.call("ic2_pack_weight_wino", nv.ptr(wa), self.in_channels, self.out_channels, self.cin_p, self.cout_p, 0,
                float(scale), nv.ptr(u), nv.F16, nv.stream_of(wa))
        self._cache[("adj_wino", scale)] = (key, u)
        return u

    def modulation_train(self, w):
        """Differentiable (xscale [n][cin_p], oscale [n][cout_p]) f32 from w [n, w_dim]: the same math as
        ic2_modconv_prep (styles = affine(w); demodulated layers: s * rsqrt(mean s^2) over the whole batch,
        oscale = input_gain * rsqrt(sum_i s_i^2 wsq[o, i] + 1e-8); ToRGB: s / sqrt(cin k^2), oscale =
        input_gain), as torch ops on [n, <= 512] rows."""
        A = self.affine
        styles = F.linear(w, A.weight * float(A.weight_gain), A.bias * float(A.bias_gain))
        ig = self.input_gain()
        if self.is_torgb:
            s = styles * float(1 / np.sqrt(self.in_channels * (self.conv_kernel ** 2)))
            d = torch.full([w.shape[0], self.out_channels], ig, dtype=torch.float32, device=w.device)
        else:
            s = styles * styles.square().mean().rsqrt()
            _, wsq, _ = self.packed(torch.float32)
            d = (s.square() @ wsq.t() + 1e-8).rsqrt() * ig
        return F.pad(s, (0, self.cin_p - self.in_channels)), F.pad(d, (0, self.cout_p - self.out_channels))

    def forward_train_nhwc(self, x, w, dt, final_scale=None):
        """Autograd step: x NHWC [n, in, in, cin_p] (dt, NOT yet scaled by xscale), w [n, w_dim] f32 ->
        NHWC [n, out, out, cout_p] dt, or for ToRGB the NCHW f32 image * final_scale."""
        xs, os_ = self.modulation_train(w)
        if not self.is_torgb:
            return ao.SynthLayerNHWC.apply(x.contiguous(), xs.contiguous(), os_.contiguous(), self, dt)
        # ToRGB (1x1, 3 channels, linear + clamp): input modulation and frozen conv as HIP kernels (the d xscale
        # reduction in f32), the rest as torch ops
        return self.torgb_train_nhwc(ao.ScaleNHWC.apply(x, xs), os_, dt, final_scale)

    def torgb_train_nhwc(self, a, os_, dt, final_scale=None):
        """ToRGB's autograd step on its already-modulated input a NHWC [n, s, s, cin_p] -> NCHW f32 image."""
        wp, _, bp = self.packed(dt)
        c = ao.FrozenConvNHWC.apply(a, wp, self.packed_adjoint(dt), 1, 0, self.out_channels, self.in_channels)
        y = c * os_[:, None, None, :] + bp
        if self.conv_clamp is not None:
            y = y.clamp(-float(self.conv_clamp), float(self.conv_clamp))
        img = y[..., : self.out_channels].permute(0, 3, 1, 2)
        return img if final_scale is None else img * float(final_scale)

    def forward(self, x, w, noise_mode="random", force_fp32=False, update_emas=False):
        """Layer-level API (NCHW f32 in/out), as SG3's SynthesisLayer.forward."""
        assert noise_mode in ("random", "const", "none")
        if update_emas:
            raise NotImplementedError("update_emas is a training feature (out of scope)")
        if _train_mode(self, x, w):
            return self.forward_train(x, w)
        x_in, w_in = x, w
        x = x.to(torch.float32).contiguous()
        w = w.to(torch.float32).contiguous()
        nv.require_gpu(x, w)
        n = x.shape[0]
        assert list(x.shape) == [n, self.in_channels, int(self.in_size[1]), int(self.in_size[0])], x.shape
        dt = torch.float32
        xs, os_ = self.scales(w, self.w_dim, n, dt)
        s_in = int(self.in_size[0])
        xn = torch.empty([n, s_in, s_in, self.cin_p], dtype=dt, device=x.device)
        nv.call("ic2_nchw_to_nhwc", nv.ptr(x), nv.ptr(xn), nv.F32, n, self.in_channels, s_in, s_in, self.cin_p,
                nv.ptr(xs), nv.stream_of(x))
        out = self.run_nhwc(xn, n, dt, os_, None)
        if self.is_torgb:
            return _refuse(self, out, x_in, w_in)
        s_out = int(self.out_size[0])
        y = torch.empty([n, self.out_channels, s_out, s_out], dtype=torch.float32, device=x.device)
        nv.call("ic2_nhwc_to_nchw", nv.ptr(out), nv.F32, nv.ptr(y), n, self.out_channels, s_out, s_out, self.cout_p,
                nv.stream_of(x))
        return _refuse(self, y, x_in, w_in)

    def forward_train(self, x, w):
        """Layer-level autograd path (NCHW f32 in/out), fp32."""
        x = x.to(torch.float32)
        w = w.to(torch.float32)
        nv.require_gpu(x.contiguous(), w.contiguous())
        xn = F.pad(x.permute(0, 2, 3, 1), (0, self.cin_p - self.in_channels)).contiguous()
        out = self.forward_train_nhwc(xn, w, torch.float32)
        if self.is_torgb:
            return out
        return out[..., : self.out_channels].permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def design_lowpass_filter(numtaps, cutoff, width, fs, radial=False):
        assert numtaps >= 1
        if numtaps == 1:
            return None
        if radial:
            raise NotImplementedError("radial filters (StyleGAN3-R) are not on the path")
        f = scipy.signal.firwin(numtaps=numtaps, cutoff=cutoff, width=width, fs=fs)
        return torch.as_tensor(f, dtype=torch.float32)

    def extra_repr(self):
        return "\n".join([
            f"w_dim={self.w_dim:d}, is_torgb={self.is_torgb},",
            f"is_critically_sampled={self.is_critically_sampled}, use_fp16={self.use_fp16},",
            f"in_sampling_rate={self.in_sampling_rate:g}, out_sampling_rate={self.out_sampling_rate:g},",
            f"in_cutoff={self.in_cutoff:g}, out_cutoff={self.out_cutoff:g},",
            f"in_half_width={self.in_half_width:g}, out_half_width={self.out_half_width:g},",
            f"in_size={list(self.in_size)}, out_size={list(self.out_size)},",
            f"in_channels={self.in_channels:d}, out_channels={self.out_channels:d}"])


# ------------------------------------------------------------------------------------------------
class SynthesisNetwork(torch.nn.Module):
    """[SG3-public] ws [N, num_ws, w_dim] -> image [N, 3, R, R] f32, entirely in HIP kernels."""

    def __init__(self, w_dim, img_resolution, img_channels, channel_base=32768, channel_max=512, num_layers=14,
                 num_critical=2, first_cutoff=2, first_stopband=2 ** 2.1, last_stopband_rel=2 ** 0.3, margin_size=10,
                 output_scale=0.25, num_fp16_res=4, precision="fp32", **layer_kwargs):
        super().__init__()
        self.w_dim = w_dim
        self.num_ws = num_layers + 2
        self.img_resolution = img_resolution
        self.img_channels = img_channels
        self.num_layers = num_layers
        self.num_critical = num_critical
        self.margin_size = margin_size
        self.output_scale = output_scale
        self.num_fp16_res = num_fp16_res
        self.precision = precision
        nv.torch_dtype(precision)
        self.train_f16 = False   # autograd path in f16 (loss-scaled training, training.train_step(scaler=...))

        last_cutoff = self.img_resolution / 2
        last_stopband = last_cutoff * last_stopband_rel
        exponents = np.minimum(np.arange(self.num_layers + 1) / (self.num_layers - self.num_critical), 1)
        cutoffs = first_cutoff * (last_cutoff / first_cutoff) ** exponents
        stopbands = first_stopband * (last_stopband / first_stopband) ** exponents
        sampling_rates = np.exp2(np.ceil(np.log2(np.minimum(stopbands * 2, self.img_resolution))))
        half_widths = np.maximum(stopbands, sampling_rates / 2) - cutoffs
        sizes = sampling_rates + self.margin_size * 2
        sizes[-2:] = self.img_resolution
        channels = np.rint(np.minimum((channel_base / 2) / cutoffs, channel_max))
        channels[-1] = self.img_channels

        self.input = SynthesisInput(w_dim=self.w_dim, channels=int(channels[0]), size=int(sizes[0]),
                                    sampling_rate=sampling_rates[0], bandwidth=cutoffs[0])
        self.layer_names = []
        for idx in range(self.num_layers + 1):
            prev = max(idx - 1, 0)
            is_torgb = idx == self.num_layers
            is_critically_sampled = idx >= self.num_layers - self.num_critical
            use_fp16 = sampling_rates[idx] * (2 ** self.num_fp16_res) > self.img_resolution
            layer = SynthesisLayer(
                w_dim=self.w_dim, is_torgb=is_torgb, is_critically_sampled=is_critically_sampled, use_fp16=use_fp16,
                in_channels=int(channels[prev]), out_channels=int(channels[idx]), in_size=int(sizes[prev]),
                out_size=int(sizes[idx]), in_sampling_rate=int(sampling_rates[prev]),
                out_sampling_rate=int(sampling_rates[idx]), in_cutoff=cutoffs[prev], out_cutoff=cutoffs[idx],
                in_half_width=half_widths[prev], out_half_width=half_widths[idx], **layer_kwargs)
            name = f"L{idx}_{layer.out_size[0]}_{layer.out_channels}"
            setattr(self, name, layer)
            self.layer_names.append(name)

    def layers(self):
        return [getattr(self, name) for name in self.layer_names]

    def forward(self, ws, noise_mode="const", force_fp32=False, update_emas=False, **layer_kwargs):
        """noise_mode is accepted and ignored exactly like SG3 (the T generator has no noise inputs)."""
        assert noise_mode in ("random", "const", "none")
        if update_emas:
            raise NotImplementedError("update_emas is a training feature (out of scope)")
        assert ws.ndim == 3 and ws.shape[1] == self.num_ws and ws.shape[2] == self.w_dim, ws.shape
        dt = torch.float32 if force_fp32 else nv.torch_dtype(self.precision)
        if _train_mode(self, ws):
            # 'f16' trains in f16 only when the caller scales its loss (train_f16: the reference's fp16 autocast +
            # GradScaler, stylegan3_hvae_full.py:487,693-696; unscaled gradients underflow f16), else in bf16
            tdt = dt if dt != torch.float16 or self.train_f16 else torch.bfloat16
            return self.forward_train(ws, tdt)
        ws_in = ws
        ws = ws.to(torch.float32).contiguous()
        nv.require_gpu(ws)
        n = ws.shape[0]
        ldx = self.num_ws * self.w_dim
        layers = self.layers()
        # all per-layer modulation coefficients first (each step needs the next layer's xscale): one batched
        # affine FC + (de)modulation prep for every layer (three launches, bit-identical to L.scales per layer)
        sc = self.scales_batched(ws, ldx, n, dt)
        x = self.input.run_nhwc(ws, ldx, n, dt, sc[0][0])
        for i, L in enumerate(layers):
            post = sc[i + 1][0] if i + 1 < len(layers) else None
            x = L.run_nhwc(x, n, dt, sc[i][1], post, final_scale=self.output_scale if L.is_torgb else None)
        return _refuse(self, x, ws_in)

    def scales_batched(self, ws, ldx, n, dt):
        """[(xscale [n][cin_p], oscale [n][cout_p]) per layer] through ic2_modconv_prep_batched (per layer when a
        layer is wider than its rows allow)."""
        layers = self.layers()
        if not all(L.batchable() for L in layers):
            flat = ws.view(-1)
            return [L.scales(flat[(i + 1) * self.w_dim:], ldx, n, dt) for i, L in enumerate(layers)]
        sizes = [(n * L.in_channels + 3) // 4 * 4 + n * L.cin_p + n * L.cout_p for L in layers]
        buf = torch.empty([sum(sizes)], dtype=torch.float32, device=ws.device)
        rec = np.zeros([len(layers), 16], dtype=np.int64)
        out, off = [], 0
        for i, L in enumerate(layers):
            ns = (n * L.in_channels + 3) // 4 * 4
            styles = buf[off:off + ns]
            xs = buf[off + ns:off + ns + n * L.cin_p].view(n, L.cin_p)
            os_ = buf[off + ns + n * L.cin_p:off + sizes[i]].view(n, L.cout_p)
            off += sizes[i]
            rec[i] = L.mod_record(dt, (i + 1) * self.w_dim, styles, xs, os_)
            out.append((xs, os_))
        nv.call("ic2_modconv_prep_batched", nv.ptr(ws), ldx, n, self.w_dim, len(layers),
                rec.ctypes.data_as(ctypes.c_void_p), nv.stream_of(ws))
        return out

    def _train_mod_pack(self, convs, device):
        """Frozen constants of the batched training modulation of the modulated (non-ToRGB) layers, zero-padded to
        the widest layer: affine weights / biases times their gains [L, cm, w_dim] / [L, cm], |W|^2 rows [L, om, cm],
        input channel counts [L], and input gain x valid-output mask [L, 1, om].  Rebuilt when any weight changes."""
        key = (device,) + tuple(k for L in convs for k in _version_key(L.affine.weight, L.affine.bias, L.weight,
                                                                        L.magnitude_ema))
        hit = getattr(self, "_mod_pack_cache", None)
        if hit is not None and hit[0] == key:
            return hit[1]
        nl = len(convs)
        cm, om = max(L.cin_p for L in convs), max(L.cout_p for L in convs)
        wst = torch.zeros([nl, cm, self.w_dim], dtype=torch.float32, device=device)
        bst = torch.zeros([nl, cm], dtype=torch.float32, device=device)
        wsq = torch.zeros([nl, om, cm], dtype=torch.float32, device=device)
        igm = torch.zeros([nl, 1, om], dtype=torch.float32, device=device)
        with torch.no_grad():
            for i, L in enumerate(convs):
                A = L.affine
                wst[i, : L.in_channels] = A.weight.float() * float(A.weight_gain)
                bst[i, : L.in_channels] = A.bias.float() * float(A.bias_gain)
                wsq[i, : L.out_channels, : L.in_channels] = L.packed(torch.float32)[1]
                igm[i, 0, : L.out_channels] = L.input_gain()
        cin = torch.tensor([float(L.in_channels) for L in convs], dtype=torch.float32).to(device)
        pack = (wst, bst, wsq, igm, cin)
        self._mod_pack_cache = (key, pack)
        return pack

    def forward_train(self, ws, dt):
        """Autograd path w.r.t. ws (the reference's encoder training, stylegan3_hvae_full.py:669-696): input
        features and the (de)modulation of all layers as batched torch ops on small tensors, the convs and filtered
        lrelus as HIP kernels with HIP backward passes (autograd_ops).  The generator's weights stay frozen.
        The modulated layers' styles and demodulation coefficients come from one batched GEMM each over the stacked
        (zero-padded) layers: the same math as SynthesisLayer.modulation_train per layer, in ~10 launches instead
        of ~14 per layer (and as many fewer in the backward)."""
        ws = ws.to(torch.float32)
        nv.require_gpu(ws.contiguous())
        C = self.input.channels
        x = self.input.forward_train_nhwc(ws[:, 0], dt)
        layers = self.layers()
        x = F.pad(x, (0, layers[0].cin_p - C)).to(dt)
        convs = [L for L in layers if not L.is_torgb]
        assert all(not L.is_torgb for L in layers[: len(convs)]), "modulated layers first, ToRGB last"
        wst, bst, wsq, igm, cin = self._train_mod_pack(convs, ws.device)
        n = ws.shape[0]
        wl = ws[:, 1: 1 + len(convs)].transpose(0, 1)                       # [L, n, w_dim]
        st = torch.baddbmm(bst.unsqueeze(1), wl, wst.transpose(1, 2))       # styles [L, n, cm], 0 past cin
        s = st * (st.square().sum(dim=(1, 2)) / (cin * n)).rsqrt()[:, None, None]
        d = (torch.bmm(s.square(), wsq.transpose(1, 2)) + 1e-8).rsqrt() * igm  # [L, n, om], 0 past cout
        xss = ao.SplitRows.apply(s, tuple(L.cin_p for L in convs))
        oss = ao.SplitRows.apply(d, tuple(L.cout_p for L in convs))
        # each layer's input modulation rides on the previous layer's filtered-lrelu store (its post-scale row); the
        # first layer's on a scale pass, the ToRGB's on the last modulated layer's store
        rgb = layers[len(convs)]
        xs_rgb, os_rgb = rgb.modulation_train(ws[:, len(convs) + 1])
        x = ao.ScaleNHWC.apply(x, xss[0])
        for i, L in enumerate(convs):
            xs_next = xss[i + 1] if i + 1 < len(convs) else xs_rgb
            x = ao.SynthLayerScaledNHWC.apply(x, oss[i], xs_next, L, dt)
        return rgb.torgb_train_nhwc(x, os_rgb, dt, final_scale=self.output_scale)

    def extra_repr(self):
        return "\n".join([
            f"w_dim={self.w_dim:d}, num_ws={self.num_ws:d},",
            f"img_resolution={self.img_resolution:d}, img_channels={self.img_channels:d},",
            f"num_layers={self.num_layers:d}, num_critical={self.num_critical:d},",
            f"margin_size={self.margin_size:d}, num_fp16_res={self.num_fp16_res:d}, precision={self.precision}"])


# ------------------------------------------------------------------------------------------------
class Generator(torch.nn.Module):
    """[SG3-public] Generator(z_dim, c_dim, w_dim, img_resolution, img_channels): synthesis built first,
    then mapping (SG3's construction order, so a seeded build draws the same parameters)."""

    def __init__(self, z_dim=512, c_dim=0, w_dim=512, img_resolution=256, img_channels=3, mapping_kwargs={},
                 precision="fp32", **synthesis_kwargs):
        super().__init__()
        self.z_dim = z_dim
        self.c_dim = c_dim
        self.w_dim = w_dim
        self.img_resolution = img_resolution
        self.img_channels = img_channels
        self.synthesis = SynthesisNetwork(w_dim=w_dim, img_resolution=img_resolution, img_channels=img_channels,
                                          precision=precision, **synthesis_kwargs)
        self.num_ws = self.synthesis.num_ws
        self.mapping = MappingNetwork(z_dim=z_dim, c_dim=c_dim, w_dim=w_dim, num_ws=self.num_ws, **mapping_kwargs)

    @property
    def precision(self):
        return self.synthesis.precision

    def set_precision(self, precision):
        nv.torch_dtype(precision)
        self.synthesis.precision = precision
        return self

    def forward(self, z, c=None, truncation_psi=1, truncation_cutoff=None, update_emas=False, **synthesis_kwargs):
        ws = self.mapping(z, c, truncation_psi=truncation_psi, truncation_cutoff=truncation_cutoff,
                          update_emas=update_emas)
        return self.synthesis(ws, update_emas=update_emas, **synthesis_kwargs)


def make_generator(img_resolution=256, seed=None, precision="fp32", device="cuda", **kw):
    """Seeded StyleGAN3-T generator (random init -- no pretrained weights are available offline)."""
    if seed is not None:
        torch.manual_seed(seed)
    G = Generator(z_dim=512, c_dim=0, w_dim=512, img_resolution=img_resolution, img_channels=3, precision=precision, **kw)
    return G.to(device).eval().requires_grad_(False)
