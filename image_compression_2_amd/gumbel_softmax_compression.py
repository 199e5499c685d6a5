"""Drop-in for /root/reference/gumbel_softmax_compression.py's codec classes, MI355X-native.

GumbelSoftmaxDiscretization keeps the reference's buffers/parameters (``codebook`` = linspace(-1, 1, K),
``log_temperature``, ``usage``) and signatures; its forward is ONE fused HIP kernel
(``ic2_gumbel_softmax_quantize``) instead of the reference's chain of [N*8192, K] fp32 tensors.
Indices are bit-exact (fp32 |z - c| argmin, first index on ties, ref :97, :118).  The Gumbel noise
comes from an in-kernel Philox stream whose seed is drawn on the device generator (as ``F.gumbel_softmax`` draws on
z's device): the same distribution as the reference's noise, not the same stream (the reference's noisy outputs are
RNG-dependent anyway), and torch's CPU stream -- which the encoder's fine projector re-creates
fc1 from -- advances exactly as the reference's.  The device generator's offset advances by a different amount than
the reference's [N*8192, K] exponential_ draw (only later device draws, e.g. the reparameterisation noise of w_plus,
see that); compress()/decompress() are deterministic and bit-exact, and compress() skips the noise entirely (its
indices are the exact argmin) while still counting `usage` in training mode as the reference's does.
Forward is inference-only: it runs in grad mode, but a backward through the kernel raises (training is out of
scope).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _native as nv
from .stylegan3_hvae_full import HVAE_VGG_Encoder, StyleGAN3Compressor, save_tensor_as_image, resize_bilinear  # noqa: F401


def codebook_argmin(z, codebook, hist=False):
    """Exact argmin_k |z - codebook[k]| -> int64 indices (+ uint32 usage histogram)."""
    z = z.to(torch.float32).contiguous()
    nv.require_gpu(z, codebook)
    idx = torch.empty(z.numel(), dtype=torch.int64, device=z.device)
    h = torch.zeros(codebook.numel(), dtype=torch.int32, device=z.device) if hist else None
    nv.call("ic2_quantize_codebook_argmin", nv.ptr(z), z.numel(), nv.ptr(codebook), codebook.numel(), nv.ptr(idx), None,
            nv.ptr(h), nv.stream_of(z))
    return (idx, h) if hist else idx


def codebook_lookup(codes, codebook):
    """codebook[codes] -> (f32 values, int32 flag); flag != 0 when some code lies outside [0, K)."""
    codes = codes.to(torch.int64).contiguous()
    nv.require_gpu(codes, codebook)
    out = torch.empty(codes.shape, dtype=torch.float32, device=codes.device)
    flag = torch.zeros(1, dtype=torch.int32, device=codes.device)
    nv.call("ic2_codebook_lookup", nv.ptr(codes), codes.numel(), nv.ptr(codebook), codebook.numel(), nv.ptr(out),
            nv.ptr(flag), nv.stream_of(codes))
    return out, flag


def check_codes(flag, k):
    """The reference's ``codebook[flat_codes]`` (gumbel_softmax_compression.py:258) raises on a code outside
    [0, K); the lookup kernel raises the same way through its flag (one small sync on a path that syncs)."""
    if int(flag.item()) != 0:
        raise IndexError(f"code out of range for a codebook of {k} entries")


class GumbelSoftmaxDiscretization(nn.Module):
    """Codebook quantizer (ref ``gumbel_softmax_compression.py:26-137``)."""

    def __init__(self, latent_dim=512, n_embeddings=256, temperature=1.0, straight_through=True, learnable_temp=True):
        super().__init__()
        self.latent_dim = latent_dim
        self.n_embeddings = n_embeddings
        self.initial_temp = temperature
        self.straight_through = straight_through
        self.register_buffer("codebook", torch.linspace(-1, 1, n_embeddings).float())
        if learnable_temp:
            self.log_temperature = nn.Parameter(torch.ones(1) * np.log(temperature))
        else:
            self.register_buffer("log_temperature", torch.ones(1) * np.log(temperature))
        self.register_buffer("usage", torch.zeros(n_embeddings))

    @property
    def temperature(self):
        return torch.exp(self.log_temperature)

    def update_temp(self, anneal_rate=0.00003, min_temp=0.5):
        with torch.no_grad():
            self.log_temperature.clamp_(min=np.log(min_temp))
            self.log_temperature -= anneal_rate

    def forward(self, z, hard=None, gumbel_noise=None):
        """-> (discretized [B, num_ws, w_dim], perplexity scalar, encoding_indices [B*num_ws*w_dim]).
        ``gumbel_noise`` (optional [B*num_ws*w_dim, K] f32) replaces the in-kernel noise (testing)."""
        batch_size, num_ws, w_dim = z.shape
        if hard is None:
            hard = not self.training
        z_in = z
        z = z.to(torch.float32).contiguous()
        nv.require_gpu(z)
        m = z.numel()
        k = self.n_embeddings
        disc = torch.empty(m, dtype=torch.float32, device=z.device)
        idx = torch.empty(m, dtype=torch.int64, device=z.device)
        psum = torch.zeros(k, dtype=torch.float32, device=z.device)
        if gumbel_noise is not None:
            gumbel_noise = gumbel_noise.to(torch.float32).contiguous()
            assert gumbel_noise.shape == (m, k)
        # the Philox seed is drawn on the DEVICE generator (F.gumbel_softmax draws its noise on z's device, ref
        # :103-108) and read by the kernel from device memory: no host sync, and torch's CPU stream -- from which the
        # fine projector re-creates fc1 on every encoder call (stylegan3_hvae_full.py:225-230) -- advances exactly as
        # the reference's does
        seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=z.device)
        nv.call("ic2_gumbel_softmax_quantize_dseed", nv.ptr(z), m, nv.ptr(self.codebook), k,
                nv.ptr(self.log_temperature.detach()), 1.0, int(bool(hard)), nv.ptr(seed), 0, nv.ptr(gumbel_noise),
                nv.ptr(disc), nv.ptr(idx), nv.ptr(psum), nv.stream_of(z))
        if self.training:
            hist = torch.zeros(k, dtype=torch.int32, device=z.device)
            nv.call("ic2_quantize_codebook_argmin", nv.ptr(z), m, nv.ptr(self.codebook), k, nv.ptr(idx), None,
                    nv.ptr(hist), nv.stream_of(z))
            self.usage += hist.to(self.usage.dtype)
        avg_probs = psum / m
        perplexity = torch.exp(-torch.sum(avg_probs * torch.log(avg_probs + 1e-10)))
        # inference in grad mode works; a backward through the fused kernel raises (training is out of scope)
        return nv.refuse_backward("GumbelSoftmaxDiscretization.forward", (disc.view(batch_size, num_ws, w_dim),
                                  perplexity, idx), (z_in, self.log_temperature))

    def get_code_usage(self):
        total = self.usage.sum().float()
        if total > 0:
            return self.usage / total
        return self.usage


class GumbelSoftmaxCompressor(nn.Module):
    """Encoder + codebook quantizer + frozen generator (ref ``gumbel_softmax_compression.py:140-319``)."""

    def __init__(self, encoder, generator, n_embeddings=256, temperature=1.0, straight_through=True,
                 training_resolution=None):
        super().__init__()
        self.encoder = encoder
        self.generator = generator
        self.training_resolution = training_resolution
        self.discretization = GumbelSoftmaxDiscretization(latent_dim=encoder.w_dim, n_embeddings=n_embeddings,
                                                          temperature=temperature, straight_through=straight_through)
        for param in generator.parameters():
            param.requires_grad = False

    def forward(self, x, noise_mode="const"):
        w_plus, means, _ = self.encoder(x)
        w_discrete, perplexity, _ = self.discretization(means)
        img = self.generator.synthesis(w_discrete, noise_mode=noise_mode)
        if self.training_resolution is not None and img.shape[2] != x.shape[2]:
            img = resize_bilinear(img, (x.shape[2], x.shape[3]))
        return img, w_plus, w_discrete, perplexity

    def encode(self, x, deterministic=True):
        w_plus, means, _ = self.encoder(x)
        if deterministic:
            w_discrete, _, _ = self.discretization(means, hard=True)
        else:
            w_discrete, _, _ = self.discretization(w_plus, hard=True)
        return w_discrete

    def compress(self, x, discrete_bits=8):
        """-> int64 codes [B, num_ws, w_dim] on the CPU (ref :213-235); exact argmin kernel."""
        return self.compress_codes(x, discrete_bits).cpu()

    def compress_codes(self, x, discrete_bits=8):
        """compress() with the codes left on the device (extension): the reference's indices (argmin |means - c|,
        first index on ties, gumbel_softmax_compression.py:229) without its device -> host copy (:235)."""
        with torch.no_grad():
            w_plus, means, _ = self.encoder(x)
            disc = self.discretization
            if disc.training:
                # the reference's compress runs discretization(means, hard=True), which in training mode adds the
                # batch's argmin indices to `usage` (:121-123); the indices are the same exact argmin
                indices, hist = codebook_argmin(means, disc.codebook, hist=True)
                disc.usage += hist.to(disc.usage.dtype)
            else:
                indices = codebook_argmin(means, disc.codebook)
            batch_size, num_ws, w_dim = w_plus.shape
            return indices.reshape(batch_size, num_ws, w_dim)

    def decompress(self, codes, noise_mode="const"):
        with torch.no_grad():
            device = self.discretization.codebook.device
            codes = codes.to(device)
            w_discrete, flag = codebook_lookup(codes, self.discretization.codebook)
            check_codes(flag, self.discretization.n_embeddings)
            return self.generator.synthesis(w_discrete, noise_mode=noise_mode)

    def save_compressed(self, x, filename, discrete_bits=8):
        """Same .npz container as the reference (keys codes, n_embeddings, resolution, orig_size, comp_size,
        compression_ratio; ref :266-297)."""
        codes = self.compress(x, discrete_bits=discrete_bits)
        codes_np = codes.numpy()
        orig_size = x.numel() * 4
        comp_size = codes_np.size * (np.log2(self.discretization.n_embeddings) / 8)
        np.savez_compressed(filename, codes=codes_np, n_embeddings=self.discretization.n_embeddings,
                            resolution=x.shape[2:4], orig_size=orig_size, comp_size=comp_size,
                            compression_ratio=orig_size / comp_size)
        return orig_size, comp_size, orig_size / comp_size

    def load_compressed(self, filename, noise_mode="const"):
        data = np.load(filename)  # allow_pickle=False (default): plain arrays only
        if "n_embeddings" in data.files and int(data["n_embeddings"]) != self.discretization.n_embeddings:
            raise ValueError(f"container was written with n_embeddings={int(data['n_embeddings'])}, this "
                             f"compressor's codebook has {self.discretization.n_embeddings}")
        codes = torch.from_numpy(data["codes"])
        img = self.decompress(codes, noise_mode=noise_mode)
        return img, data["compression_ratio"]
