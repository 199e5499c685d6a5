"""ORACLE (test infrastructure only) -- CPU restatement of the reference's HVAE encoder and quantizers.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker; the product path never calls it.

Restates /root/reference/stylegan3_hvae_full.py and gumbel_softmax_compression.py as pure functions
over a state_dict (keys identical to the reference modules', so a product encoder's state_dict
plugs straight in).  PINNED by the golden vectors in ``tests/golden/`` that
``tests/golden/make_golden.py`` captured from the reference's own code in the build container.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def encoder_channels(img_resolution=1024, channel_base=32768, channel_max=512):
    """``stylegan3_hvae_full.py:54-59``: num_layers = log2(res); channels[r] = min(max, base // 2^(L-r))."""
    num_layers = int(math.log2(img_resolution))
    ch = {r: min(channel_max, channel_base // (2 ** (num_layers - r))) for r in range(num_layers + 1)}
    return num_layers, ch


def vgg_block(sd, prefix, x):
    """``VGGBlock.forward`` (``stylegan3_hvae_full.py:183-191``)."""
    c = sd[prefix + "conv1.weight"].shape[0]
    groups = min(32, c)
    x = F.conv2d(x, sd[prefix + "conv1.weight"], sd[prefix + "conv1.bias"], padding=1)
    x = F.leaky_relu(F.group_norm(x, groups, sd[prefix + "norm1.weight"], sd[prefix + "norm1.bias"], 1e-5), 0.2)
    x = F.conv2d(x, sd[prefix + "conv2.weight"], sd[prefix + "conv2.bias"], padding=1)
    x = F.leaky_relu(F.group_norm(x, groups, sd[prefix + "norm2.weight"], sd[prefix + "norm2.bias"], 1e-5), 0.2)
    if x.shape[2] > 1 and x.shape[3] > 1:
        x = F.avg_pool2d(x, 2, 2)
    return x


def projector(sd, prefix, x, num_ws, w_dim=512, fc1=None, eps=None):
    """``HierarchyProjector.forward`` (``stylegan3_hvae_full.py:211-247``).

    ``fc1``: optional (weight, bias) that replaces the stored fc1 -- the reference re-creates fc1 with
    fresh random weights whenever the pooled width differs from ``in_channels`` (``:225-230``); the
    caller passes the weights the product actually drew.  ``eps``: the reparameterisation noise;
    None -> zeros (returns w == mean)."""
    n = x.shape[0]
    x = F.adaptive_avg_pool2d(x, 1).view(n, -1)
    w1, b1 = fc1 if fc1 is not None else (sd[prefix + "fc1.weight"], sd[prefix + "fc1.bias"])
    assert w1.shape[1] == x.shape[1], "fc1 width mismatch: pass the re-created fc1 (reference quirk)"
    x = F.leaky_relu(F.linear(x, w1, b1), 0.2)
    p = F.linear(x, sd[prefix + "fc2.weight"], sd[prefix + "fc2.bias"]).view(n, num_ws, w_dim * 2)
    mean, logvar = torch.chunk(p, 2, dim=2)
    std = torch.exp(0.5 * logvar)
    if eps is None:
        eps = torch.zeros_like(std)
    return mean + eps * std, mean, logvar


def encoder_forward(sd, x, num_ws=16, block_split=(5, 12), w_dim=512, fine_fc1=None, eps=None,
                    return_features=False):
    """``HVAE_VGG_Encoder.forward`` (``stylegan3_hvae_full.py:105-167``).

    eps: optional dict {'global','medium','fine'} of noise tensors.  Returns (w_plus, means, logvars)."""
    nblocks = len({k.split(".")[1] for k in sd if k.startswith("blocks.")})
    num_layers = nblocks
    hier = {"fine": 1, "medium": 4, "global": num_layers - 1}
    feats = {}
    x = F.conv2d(x, sd["from_rgb.weight"], sd["from_rgb.bias"], padding=1)
    for i in range(nblocks):
        if x.shape[2] <= 1 or x.shape[3] <= 1:
            break
        x = vgg_block(sd, f"blocks.{i}.", x)
        if i == hier["fine"]:
            feats["fine"] = x
        elif i == hier["medium"]:
            feats["medium"] = x
    feats["global"] = x
    feats.setdefault("fine", x)
    feats.setdefault("medium", x)
    n_g = block_split[0]
    n_m = block_split[1] - block_split[0]
    n_f = num_ws - block_split[1]
    eps = eps or {}
    g = projector(sd, "global_projector.", feats["global"], n_g, w_dim, eps=eps.get("global"))
    m = projector(sd, "medium_projector.", feats["medium"], n_m, w_dim, eps=eps.get("medium"))
    f = projector(sd, "fine_projector.", feats["fine"], n_f, w_dim, fc1=fine_fc1, eps=eps.get("fine"))
    out = tuple(torch.cat([g[i], m[i], f[i]], dim=1) for i in range(3))
    return (out, feats) if return_features else out


# ----------------------------------------------------------------------------------------------
# Quantizers
# ----------------------------------------------------------------------------------------------
def quantize_uniform(w, bits=8):
    """``StyleGAN3Compressor.compress`` quantizer, ``stylegan3_hvae_full.py:313-316``, fp32 op order as
    written; torch.round = half-to-even; no clamp."""
    scale = (2 ** bits) - 1
    w_scaled = (w + 1) * 0.5
    q = torch.round(w_scaled * scale) / scale
    return q * 2 - 1


def uniform_indices(w, bits=8):
    """Integer index of the uniform code: round(((w+1)*0.5)*S) (the numerator at ``:315``)."""
    scale = (2 ** bits) - 1
    return torch.round(((w + 1) * 0.5) * scale).to(torch.int64)


def codebook(n_embeddings=256):
    """``gumbel_softmax_compression.py:49-52``."""
    return torch.linspace(-1, 1, n_embeddings).float()


def codebook_argmin(z, n_embeddings=256):
    """``GumbelSoftmaxDiscretization.forward`` indices (``:93,:97,:118``): argmin |z - c_k|, first index
    on ties, fp32 distances."""
    cb = codebook(n_embeddings)
    d = torch.abs(z.reshape(-1, 1).float() - cb.reshape(1, -1))
    return torch.argmin(d, dim=1)


def codebook_lookup(codes, n_embeddings=256):
    """``GumbelSoftmaxCompressor.decompress`` lookup (``gumbel_softmax_compression.py:258``)."""
    return codebook(n_embeddings)[codes.reshape(-1)].reshape(codes.shape)


def gumbel_noise(seed, m, k=256):
    """The noise ``F.gumbel_softmax`` draws inside ``GumbelSoftmaxDiscretization.forward``
    (``gumbel_softmax_compression.py:103-108``) right after ``torch.manual_seed(seed)``: the forward
    consumes no CPU RNG before it; the draw is ``-empty_like(logits).exponential_().log()`` on [m, k]."""
    g = torch.Generator().manual_seed(seed)
    return -torch.empty(m, k).exponential_(generator=g).log()


def gumbel_forward(z, noise, tau, hard, n_embeddings=256):
    """``GumbelSoftmaxDiscretization.forward`` (``gumbel_softmax_compression.py:73-129``) with the Gumbel
    noise given: distances (``:97``), ``F.gumbel_softmax`` (``:103-108``, torch's own op order: (logits +
    g) / tau, softmax, straight-through one-hot at the argmax when hard), disc = soft @ codebook
    (``:112``), argmin indices (``:118``), perplexity of soft.mean(0) (``:126-127``)."""
    cb = codebook(n_embeddings)
    d = torch.abs(z.reshape(-1, 1).float() - cb.reshape(1, -1))
    logits = -d
    y = ((logits + noise) / tau).softmax(1)
    if hard:
        y = torch.zeros_like(logits).scatter_(1, y.max(1, keepdim=True)[1], 1.0) - y + y
    disc = torch.matmul(y, cb.reshape(-1, 1)).reshape(z.shape)
    idx = torch.argmin(d, dim=1)
    avg = y.mean(0)
    perplexity = torch.exp(-torch.sum(avg * torch.log(avg + 1e-10)))
    return disc, perplexity, idx


def perplexity_from_hist(hist):
    """Perplexity of hard one-hot assignments: p = hist / total; exp(-sum p log(p + 1e-10))
    (``gumbel_softmax_compression.py:126-127`` evaluated on the hard one-hot)."""
    p = hist.double() / hist.sum().double()
    return torch.exp(-torch.sum(p * torch.log(p + 1e-10)))
