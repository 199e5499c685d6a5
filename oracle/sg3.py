"""ORACLE (test infrastructure only) -- CPU restatement of StyleGAN3 synthesis.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The product path (``image_compression_2_amd``) never calls it.

Third-party algorithm (NOT in /root/reference): NVlabs/stylegan3, cloned at unpinned HEAD by the
reference (``README.md:47``; ``sys.path.insert(0, 'stylegan3')`` at ``stylegan3_hvae_full.py:8-13``).
Its source is absent from this container, so this file restates the *published* design of
``training/networks_stylegan3.py`` (SynthesisNetwork / SynthesisInput / SynthesisLayer /
modulated_conv2d / FullyConnectedLayer / MappingNetwork) and the reference ("_ref") paths of
``torch_utils/ops/{upfirdn2d,bias_act,filtered_lrelu}.py``.

Reference call sites this stands in for: ``stylegan3_hvae_full.py:274`` (forward), ``:329``
(decompress), ``gumbel_softmax_compression.py:193,262``.

PARITY STATUS: synthesis parity is UNPINNED by the reference (it ships no SG3 code, weights or
fixtures -- SURVEY.md 8(c)).  This restatement is pinned by known-answer tests instead
(impulse responses, identity filters, 4-op composition, layer-name table L0_36_512 .. L14_1024_3).

Everything here is plain fp32/fp64 PyTorch on the CPU; ``dtype`` selects the arithmetic type.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.signal
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------------------
# bias_act (restates torch_utils/ops/bias_act.py::_bias_act_ref)  [SG3-public]
# ----------------------------------------------------------------------------------------------
_ACT_DEFAULTS = {"linear": (0.0, 1.0), "lrelu": (0.2, math.sqrt(2))}


def bias_act(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None):
    """x + b (along ``dim``) -> activation -> * gain -> clamp(+-clamp)."""
    def_alpha, def_gain = _ACT_DEFAULTS[act]
    alpha = float(alpha if alpha is not None else def_alpha)
    gain = float(gain if gain is not None else def_gain)
    clamp = float(clamp if clamp is not None else -1)
    if b is not None:
        x = x + b.reshape([-1 if i == dim else 1 for i in range(x.ndim)])
    if act == "lrelu":
        x = F.leaky_relu(x, alpha)
    if gain != 1:
        x = x * gain
    if clamp >= 0:
        x = x.clamp(-clamp, clamp)
    return x


# ----------------------------------------------------------------------------------------------
# upfirdn2d (restates torch_utils/ops/upfirdn2d.py::_upfirdn2d_ref)  [SG3-public]
# ----------------------------------------------------------------------------------------------
def _parse_padding(padding):
    if isinstance(padding, int):
        padding = [padding, padding]
    if len(padding) == 2:
        px, py = padding
        padding = [px, px, py, py]
    return [int(p) for p in padding]


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
    """Zero-insert upsample -> pad/crop -> FIR (flipped unless flip_filter) -> keep every down-th."""
    if f is None:
        f = torch.ones([1, 1], dtype=torch.float32)
    n, c, h, w = x.shape
    px0, px1, py0, py1 = _parse_padding(padding)
    # zero insertion
    x = x.reshape([n, c, h, 1, w, 1])
    x = F.pad(x, [0, up - 1, 0, 0, 0, up - 1])
    x = x.reshape([n, c, h * up, w * up])
    # pad or crop (negative padding crops)
    x = F.pad(x, [max(px0, 0), max(px1, 0), max(py0, 0), max(py1, 0)])
    x = x[:, :, max(-py0, 0): x.shape[2] - max(-py1, 0), max(-px0, 0): x.shape[3] - max(-px1, 0)]
    # filter: gain ** (ndim/2) so a separable 1-D filter applied twice carries the full gain
    f = (f * (gain ** (f.ndim / 2))).to(x.dtype)
    if not flip_filter:
        f = f.flip(list(range(f.ndim)))
    f = f[None, None].repeat([c, 1] + [1] * f.ndim)
    if f.ndim == 4:
        x = F.conv2d(x, f, groups=c)
    else:
        x = F.conv2d(x, f.unsqueeze(2), groups=c)   # horizontal pass
        x = F.conv2d(x, f.unsqueeze(3), groups=c)   # vertical pass
    return x[:, :, ::down, ::down]


# ----------------------------------------------------------------------------------------------
# filtered_lrelu (restates torch_utils/ops/filtered_lrelu.py::_filtered_lrelu_ref)  [SG3-public]
# ----------------------------------------------------------------------------------------------
def filtered_lrelu(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=math.sqrt(2),
                   slope=0.2, clamp=None, flip_filter=False):
    """bias -> upfirdn2d(fu, up, pad, gain=up^2) -> lrelu*gain, clamp -> upfirdn2d(fd, down)."""
    px0, px1, py0, py1 = _parse_padding(padding)
    x = bias_act(x, b)
    x = upfirdn2d(x, fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    x = bias_act(x, act="lrelu", alpha=slope, gain=gain, clamp=clamp)
    x = upfirdn2d(x, fd, down=down, flip_filter=flip_filter)
    return x


def filtered_lrelu_out_size(in_h, in_w, fu_taps, fd_taps, up, down, padding):
    px0, px1, py0, py1 = _parse_padding(padding)
    ow = (in_w * up + (px0 + px1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) // down
    oh = (in_h * up + (py0 + py1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) // down
    return oh, ow


# ----------------------------------------------------------------------------------------------
# modulated_conv2d (restates training/networks_stylegan3.py::modulated_conv2d)  [SG3-public]
# ----------------------------------------------------------------------------------------------
def modulated_conv2d(x, w, s, demodulate=True, padding=0, input_gain=None):
    """Grouped-conv definition: per-sample modulated (+demodulated) weights, groups = batch."""
    batch = x.shape[0]
    out_c, in_c, kh, kw = w.shape
    if demodulate:
        w = w * w.square().mean([1, 2, 3], keepdim=True).rsqrt()
        s = s * s.square().mean().rsqrt()          # batch-global pre-normalisation
    w = w.unsqueeze(0) * s.unsqueeze(1).unsqueeze(3).unsqueeze(4)        # [N,O,I,k,k]
    if demodulate:
        d = (w.square().sum(dim=[2, 3, 4]) + 1e-8).rsqrt()                # [N,O]
        w = w * d.unsqueeze(2).unsqueeze(3).unsqueeze(4)
    if input_gain is not None:
        ig = torch.as_tensor(input_gain, dtype=w.dtype).expand(batch, in_c)
        w = w * ig.unsqueeze(1).unsqueeze(3).unsqueeze(4)
    x = x.reshape(1, -1, *x.shape[2:])
    w = w.reshape(-1, in_c, kh, kw)
    x = F.conv2d(x, w.to(x.dtype), padding=padding, groups=batch)
    return x.reshape(batch, -1, *x.shape[2:])


def fully_connected(x, weight, bias, lr_multiplier=1.0, activation="linear"):
    """FullyConnectedLayer.forward: x @ (W * lr/sqrt(in))^T + b * lr."""
    w = weight.to(x.dtype) * (lr_multiplier / math.sqrt(weight.shape[1]))
    b = bias.to(x.dtype) * lr_multiplier if bias is not None else None
    if activation == "linear" and b is not None:
        return torch.addmm(b.unsqueeze(0), x, w.t())
    x = x.matmul(w.t())
    return bias_act(x, b, act=activation)


# ----------------------------------------------------------------------------------------------
# Layer table (restates SynthesisNetwork.__init__ / SynthesisLayer.__init__)  [SG3-public]
# ----------------------------------------------------------------------------------------------
def design_lowpass_filter(numtaps, cutoff, width, fs):
    """Separable Kaiser low-pass via scipy.signal.firwin; numtaps == 1 -> identity (None)."""
    if numtaps == 1:
        return None
    f = scipy.signal.firwin(numtaps=numtaps, cutoff=cutoff, width=width, fs=fs)
    return torch.as_tensor(f, dtype=torch.float32)


def layer_table(img_resolution, img_channels=3, channel_base=32768, channel_max=512, num_layers=14,
                num_critical=2, first_cutoff=2, first_stopband=2 ** 2.1, last_stopband_rel=2 ** 0.3,
                margin_size=10, conv_kernel=3, filter_size=6, lrelu_upsampling=2):
    """Returns (input_spec, [layer_spec]) with every derived SG3-T hyper-parameter."""
    last_cutoff = img_resolution / 2
    last_stopband = last_cutoff * last_stopband_rel
    exponents = np.minimum(np.arange(num_layers + 1) / (num_layers - num_critical), 1)
    cutoffs = first_cutoff * (last_cutoff / first_cutoff) ** exponents
    stopbands = first_stopband * (last_stopband / first_stopband) ** exponents
    sampling_rates = np.exp2(np.ceil(np.log2(np.minimum(stopbands * 2, img_resolution))))
    half_widths = np.maximum(stopbands, sampling_rates / 2) - cutoffs
    sizes = sampling_rates + margin_size * 2
    sizes[-2:] = img_resolution
    channels = np.rint(np.minimum((channel_base / 2) / cutoffs, channel_max))
    channels[-1] = img_channels
    inp = dict(channels=int(channels[0]), size=int(sizes[0]), sampling_rate=float(sampling_rates[0]),
               bandwidth=float(cutoffs[0]))
    layers = []
    for idx in range(num_layers + 1):
        prev = max(idx - 1, 0)
        is_torgb = idx == num_layers
        L = dict(idx=idx, is_torgb=is_torgb, is_critically_sampled=idx >= num_layers - num_critical,
                 in_channels=int(channels[prev]), out_channels=int(channels[idx]),
                 in_size=int(sizes[prev]), out_size=int(sizes[idx]),
                 in_sampling_rate=int(sampling_rates[prev]), out_sampling_rate=int(sampling_rates[idx]),
                 in_cutoff=float(cutoffs[prev]), out_cutoff=float(cutoffs[idx]),
                 in_half_width=float(half_widths[prev]), out_half_width=float(half_widths[idx]))
        tmp_sr = max(L["in_sampling_rate"], L["out_sampling_rate"]) * (1 if is_torgb else lrelu_upsampling)
        k = 1 if is_torgb else conv_kernel
        up = int(np.rint(tmp_sr / L["in_sampling_rate"]))
        down = int(np.rint(tmp_sr / L["out_sampling_rate"]))
        up_taps = filter_size * up if up > 1 and not is_torgb else 1
        down_taps = filter_size * down if down > 1 and not is_torgb else 1
        pad_total = (L["out_size"] - 1) * down + 1
        pad_total -= (L["in_size"] + k - 1) * up
        pad_total += up_taps + down_taps - 2
        pad_lo = (pad_total + up) // 2
        pad_hi = pad_total - pad_lo
        L.update(tmp_sampling_rate=tmp_sr, conv_kernel=k, up=up, down=down, up_taps=up_taps,
                 down_taps=down_taps, padding=[int(pad_lo), int(pad_hi), int(pad_lo), int(pad_hi)],
                 name=f"L{idx}_{L['out_size']}_{L['out_channels']}",
                 up_filter=design_lowpass_filter(up_taps, L["in_cutoff"], L["in_half_width"] * 2, tmp_sr),
                 down_filter=design_lowpass_filter(down_taps, L["out_cutoff"], L["out_half_width"] * 2, tmp_sr))
        layers.append(L)
    return inp, layers


# ----------------------------------------------------------------------------------------------
# Seeded parameters with the public construction order (Generator: synthesis first, then mapping)
# ----------------------------------------------------------------------------------------------
def init_params(img_resolution, w_dim=512, z_dim=512, seed=None, **kw):
    """State dict keyed like SG3's G_ema (``synthesis.*``, ``mapping.*``), drawn in SG3's order."""
    if seed is not None:
        torch.manual_seed(seed)
    inp, layers = layer_table(img_resolution, **kw)
    sd = {}
    C, bw = inp["channels"], inp["bandwidth"]
    freqs = torch.randn([C, 2])
    radii = freqs.square().sum(dim=1, keepdim=True).sqrt()
    freqs /= radii * radii.square().exp().pow(0.25)
    freqs *= bw
    phases = torch.rand([C]) - 0.5
    sd["synthesis.input.weight"] = torch.randn([C, C])
    sd["synthesis.input.affine.weight"] = torch.randn([4, w_dim]) * 0.0
    sd["synthesis.input.affine.bias"] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    sd["synthesis.input.transform"] = torch.eye(3, 3)
    sd["synthesis.input.freqs"] = freqs
    sd["synthesis.input.phases"] = phases
    for L in layers:
        p = f"synthesis.{L['name']}."
        sd[p + "affine.weight"] = torch.randn([L["in_channels"], w_dim])
        sd[p + "affine.bias"] = torch.ones([L["in_channels"]])
        sd[p + "weight"] = torch.randn([L["out_channels"], L["in_channels"], L["conv_kernel"], L["conv_kernel"]])
        sd[p + "bias"] = torch.zeros([L["out_channels"]])
        sd[p + "magnitude_ema"] = torch.ones([])
        if L["up_filter"] is not None:
            sd[p + "up_filter"] = L["up_filter"]
        if L["down_filter"] is not None:
            sd[p + "down_filter"] = L["down_filter"]
    lr = 0.01
    for i in range(2):
        sd[f"mapping.fc{i}.weight"] = torch.randn([w_dim, z_dim if i == 0 else w_dim]) * (1 / lr)
        sd[f"mapping.fc{i}.bias"] = torch.zeros([w_dim])
    sd["mapping.w_avg"] = torch.zeros([w_dim])
    return sd


# ----------------------------------------------------------------------------------------------
# Forward passes
# ----------------------------------------------------------------------------------------------
def synthesis_input(sd, inp, w, dtype=torch.float32):
    """SynthesisInput.forward: affine -> rot/trans of Fourier freqs -> sin features -> @ W/sqrt(C)."""
    p = "synthesis.input."
    w = w.to(dtype)
    N = w.shape[0]
    freqs = sd[p + "freqs"].to(dtype).unsqueeze(0)
    phases = sd[p + "phases"].to(dtype).unsqueeze(0)
    transforms = sd[p + "transform"].to(dtype).unsqueeze(0)
    t = fully_connected(w, sd[p + "affine.weight"].to(dtype), sd[p + "affine.bias"].to(dtype))
    t = t / t[:, :2].norm(dim=1, keepdim=True)
    m_r = torch.eye(3, dtype=dtype).unsqueeze(0).repeat([N, 1, 1])
    m_r[:, 0, 0] = t[:, 0]
    m_r[:, 0, 1] = -t[:, 1]
    m_r[:, 1, 0] = t[:, 1]
    m_r[:, 1, 1] = t[:, 0]
    m_t = torch.eye(3, dtype=dtype).unsqueeze(0).repeat([N, 1, 1])
    m_t[:, 0, 2] = -t[:, 2]
    m_t[:, 1, 2] = -t[:, 3]
    transforms = m_r @ m_t @ transforms
    phases = phases + (freqs @ transforms[:, :2, 2:]).squeeze(2)
    freqs = freqs @ transforms[:, :2, :2]
    sr, bw, size = inp["sampling_rate"], inp["bandwidth"], inp["size"]
    amplitudes = (1 - (freqs.norm(dim=2) - bw) / (sr / 2 - bw)).clamp(0, 1)
    theta = torch.eye(2, 3, dtype=dtype)
    theta[0, 0] = 0.5 * size / sr
    theta[1, 1] = 0.5 * size / sr
    grids = F.affine_grid(theta.unsqueeze(0), [1, 1, size, size], align_corners=False)
    x = (grids.unsqueeze(3) @ freqs.permute(0, 2, 1).unsqueeze(1).unsqueeze(2)).squeeze(3)
    x = x + phases.unsqueeze(1).unsqueeze(2)
    x = torch.sin(x * (np.pi * 2))
    x = x * amplitudes.unsqueeze(1).unsqueeze(2)
    weight = sd[p + "weight"].to(dtype) / np.sqrt(inp["channels"])
    x = x @ weight.t()
    return x.permute(0, 3, 1, 2)


def synthesis_layer(sd, L, x, w, dtype=torch.float32):
    """SynthesisLayer.forward (noise_mode is ignored by SG3: the layer has no noise input)."""
    p = f"synthesis.{L['name']}."
    input_gain = sd[p + "magnitude_ema"].to(dtype).rsqrt()
    styles = fully_connected(w.to(dtype), sd[p + "affine.weight"].to(dtype), sd[p + "affine.bias"].to(dtype))
    if L["is_torgb"]:
        styles = styles * (1 / np.sqrt(L["in_channels"] * (L["conv_kernel"] ** 2)))
    x = modulated_conv2d(x.to(dtype), sd[p + "weight"].to(dtype), styles, demodulate=not L["is_torgb"],
                         padding=L["conv_kernel"] - 1, input_gain=input_gain)
    gain = 1 if L["is_torgb"] else np.sqrt(2)
    slope = 1 if L["is_torgb"] else 0.2
    fu = sd.get(p + "up_filter")
    fd = sd.get(p + "down_filter")
    return filtered_lrelu(x, fu=None if fu is None else fu.to(dtype), fd=None if fd is None else fd.to(dtype),
                          b=sd[p + "bias"].to(dtype), up=L["up"], down=L["down"], padding=L["padding"],
                          gain=gain, slope=slope, clamp=256)


def synthesis_forward(sd, img_resolution, ws, dtype=torch.float32, output_scale=0.25, return_all=False, **kw):
    """SynthesisNetwork.forward: ws.unbind(1) -> input(ws[0]) -> L0..L14(ws[1..]) -> * 0.25."""
    inp, layers = layer_table(img_resolution, **kw)
    assert ws.ndim == 3 and ws.shape[1] == len(layers) + 1, ws.shape
    ws = ws.to(dtype).unbind(dim=1)
    x = synthesis_input(sd, inp, ws[0], dtype)
    acts = [x]
    for L, w in zip(layers, ws[1:]):
        x = synthesis_layer(sd, L, x, w, dtype)
        acts.append(x)
    x = x * output_scale
    return (x, acts) if return_all else x


def mapping_forward(sd, z, truncation_psi=1.0, num_ws=16):
    """MappingNetwork.forward (c_dim = 0): normalise z, 2 lrelu FCs (lr 0.01), broadcast, truncate."""
    x = z.to(torch.float32)
    x = x * (x.square().mean(1, keepdim=True) + 1e-8).rsqrt()
    for i in range(2):
        x = fully_connected(x, sd[f"mapping.fc{i}.weight"], sd[f"mapping.fc{i}.bias"], lr_multiplier=0.01,
                            activation="lrelu")
    x = x.unsqueeze(1).repeat([1, num_ws, 1])
    if truncation_psi != 1:
        x = sd["mapping.w_avg"].lerp(x, truncation_psi)
    return x
