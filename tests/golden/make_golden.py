"""Generates the golden fixtures in tests/golden/ by running the REFERENCE's own code on the CPU.

Runs only in the build container (needs /root/reference; never on the GPU box).  The reference
imports third-party modules that are absent offline and unused by the hot-path classes
(torch_utils, dnnlib, lpips, torchvision -- SURVEY.md 8(c)); they are stubbed as empty modules.
Nothing from the reference is copied: the fixtures are inputs + outputs only (.npz / .pt tensors).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import io
import os
import sys
import tempfile
import types
import contextlib

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    for name in ["torch_utils", "torch_utils.misc", "dnnlib", "lpips", "torchvision", "torchvision.transforms"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["torch_utils"].misc = sys.modules["torch_utils.misc"]
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.path.insert(0, REF)
    import stylegan3_hvae_full as ref_full          # noqa: E402
    import gumbel_softmax_compression as ref_gumbel  # noqa: E402
    return ref_full, ref_gumbel


class StubEncoder(torch.nn.Module):
    """Returns fixed latents so the reference compress() exercises only its quantizer."""
    def __init__(self, means):
        super().__init__()
        self.means = means
        self.w_dim = means.shape[-1]

    def forward(self, x):
        return self.means, self.means, torch.zeros_like(self.means)


class StubGenerator(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1))


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


def sd_to_np(sd):
    return {k: v.detach().cpu().numpy() for k, v in sd.items()}


def adversarial_uniform(bits):
    """Exact half-steps of the uniform grid (w = 2(k+0.5)/S - 1) and their +-1 ulp neighbours."""
    s = (2 ** bits) - 1
    k = np.arange(-2, s + 2, dtype=np.float64)
    mids = (2 * (k + 0.5) / s - 1).astype(np.float32)
    return np.concatenate([mids, np.nextafter(mids, np.float32(np.inf)), np.nextafter(mids, np.float32(-np.inf)),
                           np.array([-1.5, -1.0, 1.0, 1.5, 0.0, -0.0], np.float32)])


def gen_quantizers(ref_full, ref_gumbel):
    g = torch.Generator().manual_seed(1234)
    out = {}
    for bits in (4, 8, 10):
        rnd = (torch.rand(2, 16, 512, generator=g) * 2.4 - 1.2).float()
        adv = torch.from_numpy(adversarial_uniform(bits))
        pad = (-adv.numel()) % 512
        adv = torch.cat([adv, torch.zeros(pad)]).reshape(1, -1, 512)
        for tag, w in (("rand", rnd), ("adv", adv)):
            comp = ref_full.StyleGAN3Compressor(StubEncoder(w), StubGenerator())
            with quiet():
                q = comp.compress(torch.zeros(1), quantization_bits=bits, deterministic=True)
            out[f"uniform_b{bits}_{tag}_w"] = w.numpy()
            out[f"uniform_b{bits}_{tag}_q"] = q.numpy()
    # codebook argmin: random, exact midpoints, +-1 ulp, out of range
    disc = ref_gumbel.GumbelSoftmaxDiscretization(512, 256).eval()
    cb = disc.codebook.numpy()
    mids = ((cb[:-1].astype(np.float64) + cb[1:]) / 2).astype(np.float32)
    mids32 = ((cb[:-1] + cb[1:]) * np.float32(0.5)).astype(np.float32)
    specials = np.concatenate([mids, mids32, np.nextafter(mids, np.float32(np.inf)),
                               np.nextafter(mids, np.float32(-np.inf)), cb,
                               np.array([-1.5, 1.5, -1.0, 1.0, 0.0, 3.0, -3.0], np.float32)])
    rnd = (torch.rand(4, 16, 512, generator=g) * 2.2 - 1.1).numpy()
    z = np.concatenate([rnd.reshape(-1), specials])
    pad = (-z.size) % (16 * 512)
    z = np.concatenate([z, np.zeros(pad, np.float32)]).reshape(-1, 16, 512).astype(np.float32)
    with quiet(), torch.no_grad():
        _, _, idx = disc(torch.from_numpy(z), hard=True)
    out["codebook"] = cb
    out["codebook_z"] = z
    out["codebook_idx"] = idx.numpy().astype(np.int64)
    np.savez_compressed(os.path.join(OUT, "quantizers.npz"), **out)
    print("quantizers.npz", {k: v.shape for k, v in out.items()})


SMALL = dict(img_resolution=64, img_channels=3, w_dim=32, num_ws=16, block_split=(5, 12),
             channel_base=256, channel_max=32)


def gen_encoder_small(ref_full):
    torch.manual_seed(7)
    enc = ref_full.HVAE_VGG_Encoder(**SMALL)
    sd0 = {k: v.clone() for k, v in enc.state_dict().items()}
    x = (torch.rand(3, 3, 32, 32, generator=torch.Generator().manual_seed(8)) * 2 - 1)
    torch.manual_seed(9)
    with quiet(), torch.no_grad():
        w_plus, means, logvars = enc(x)
    sd1 = enc.state_dict()
    out = {"x": x.numpy(), "w_plus": w_plus.numpy(), "means": means.numpy(), "logvars": logvars.numpy(),
           "fine_fc1_weight": sd1["fine_projector.fc1.weight"].numpy(),
           "fine_fc1_bias": sd1["fine_projector.fc1.bias"].numpy()}
    out.update({"sd/" + k: v for k, v in sd_to_np(sd0).items()})
    # deterministic compress (uses means) at 8 bits through the reference compressor
    comp = ref_full.StyleGAN3Compressor(enc, StubGenerator())
    torch.manual_seed(9)
    with quiet(), torch.no_grad():
        q = comp.compress(x, quantization_bits=8, deterministic=True)
    out["compress_q8"] = q.numpy()
    np.savez_compressed(os.path.join(OUT, "encoder_small.npz"), **out)
    print("encoder_small.npz", len(out), "arrays")
    return enc


def gen_encoder_full(ref_full):
    """Full-size reference encoder: store seeds + hashes + latents, not the 150 MB of weights."""
    torch.manual_seed(0)
    enc = ref_full.HVAE_VGG_Encoder(img_resolution=1024)
    h = hashlib.sha256()
    for k, v in enc.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().numpy().tobytes())
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1
    torch.manual_seed(2)
    with quiet(), torch.no_grad():
        w_plus, means, logvars = enc(x)
    sd1 = enc.state_dict()
    out = {"state_sha256": np.frombuffer(h.digest(), np.uint8), "means": means.numpy(), "logvars": logvars.numpy(),
           "fine_fc1_weight": sd1["fine_projector.fc1.weight"].numpy(),
           "fine_fc1_bias": sd1["fine_projector.fc1.bias"].numpy(),
           "param_count": np.array(sum(p.numel() for p in enc.parameters()))}
    np.savez_compressed(os.path.join(OUT, "encoder_full.npz"), **out)
    print("encoder_full.npz sha", h.hexdigest()[:16], "params", int(out["param_count"]))


def gen_containers(ref_full, ref_gumbel, enc_small):
    """The reference's own .npz containers (save_compressed), kept byte-for-byte as fixtures."""
    x = torch.rand(1, 3, 32, 32, generator=torch.Generator().manual_seed(11)) * 2 - 1
    comp = ref_full.StyleGAN3Compressor(enc_small, StubGenerator())
    torch.manual_seed(12)
    with quiet():
        stats = comp.save_compressed(x, os.path.join(OUT, "ref_uniform_container.npz"), quantization_bits=8)
    gcomp = ref_gumbel.GumbelSoftmaxCompressor(enc_small, StubGenerator())
    torch.manual_seed(12)
    with quiet():
        gstats = gcomp.save_compressed(x, os.path.join(OUT, "ref_codebook_container.npz"))
    np.savez_compressed(os.path.join(OUT, "containers_input.npz"), x=x.numpy(),
                        uniform_stats=np.array(stats, np.float64), codebook_stats=np.array(gstats, np.float64))
    print("containers", stats, gstats)


GUMBEL_CASES = [  # (learnable_temp, temperature, hard, torch seed of the forward)
    (True, 1.0, False, 101),
    (True, 0.7, True, 101),
    (False, 0.7, False, 101),
    (False, 2.5, True, 101),
]


def gumbel_noise(seed, m, k):
    """The Gumbel noise F.gumbel_softmax draws inside GumbelSoftmaxDiscretization.forward
    (gumbel_softmax_compression.py:103-108) when the forward runs right after torch.manual_seed(seed):
    the forward consumes no other CPU RNG before it, and gumbel_softmax draws
    -empty_like(logits).exponential_().log() on the [m, k] logits."""
    torch.manual_seed(seed)
    return -torch.empty(m, k).exponential_().log()


def gen_gumbel(ref_gumbel):
    """Reference GumbelSoftmaxDiscretization.forward (soft / hard, learnable / fixed temperature, tau != 1):
    z, the outputs (disc, perplexity, indices), and the noise it drew.  Every case runs after the same seed,
    so one stored noise array serves all four (the CPU exponential_ stream is not bit-identical across
    host CPUs -- AVX2 vs AVX-512 -- so the GPU box cannot regenerate it; the sha256 lets a host check its
    own replay)."""
    g = torch.Generator().manual_seed(4321)
    z = (torch.rand(1, 8, 32, generator=g) * 2.4 - 1.2).float()
    m, k = z.numel(), 256
    out = {"z": z.numpy()}
    for ci, (learn, tau, hard, seed) in enumerate(GUMBEL_CASES):
        disc_mod = ref_gumbel.GumbelSoftmaxDiscretization(32, k, temperature=tau, learnable_temp=learn).eval()
        torch.manual_seed(seed)
        with quiet(), torch.no_grad():
            disc, perp, idx = disc_mod(z, hard=hard)
        noise = gumbel_noise(seed, m, k)
        # the replay reproduces the reference's output exactly (same op order as F.gumbel_softmax)
        logits = -torch.abs(z.reshape(-1, 1) - disc_mod.codebook.reshape(1, -1))
        y = ((logits + noise) / disc_mod.temperature).softmax(1)
        if hard:
            y = torch.zeros_like(logits).scatter_(1, y.max(1, keepdim=True)[1], 1.0) - y + y
        assert torch.equal(torch.matmul(y, disc_mod.codebook.reshape(-1, 1)).reshape(z.shape), disc), ci
        out[f"c{ci}_disc"] = disc.numpy()
        out[f"c{ci}_perplexity"] = perp.numpy()
        out[f"c{ci}_idx"] = idx.numpy().astype(np.int64)
        out["noise"] = noise.numpy()
        out[f"c{ci}_noise_sha256"] = np.frombuffer(hashlib.sha256(noise.numpy().tobytes()).digest(), np.uint8)
        out[f"c{ci}_meta"] = np.array([float(learn), tau, float(hard), float(seed)], np.float64)
    np.savez_compressed(os.path.join(OUT, "gumbel_forward.npz"), **out)
    print("gumbel_forward.npz", len(GUMBEL_CASES), "cases")


def main(only=None):
    ref_full, ref_gumbel = import_reference()
    if only == "gumbel":
        gen_gumbel(ref_gumbel)
        return
    gen_quantizers(ref_full, ref_gumbel)
    enc_small = gen_encoder_small(ref_full)
    gen_containers(ref_full, ref_gumbel, enc_small)
    gen_encoder_full(ref_full)
    gen_gumbel(ref_gumbel)


if __name__ == "__main__":
    with tempfile.TemporaryDirectory():
        main(sys.argv[1] if len(sys.argv) > 1 else None)
