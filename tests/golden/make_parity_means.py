"""Generates tests/golden/parity_means.npz: the fp32 oracle encoder's means on the benched workloads' inputs.

Runs in the build container (CPU only, seconds).  The fixture replaces running the CPU oracle encoder on the GPU box
in tests/test_gpu_c2_parity.py / test_gpu_c4_parity.py, and gives bench.py a committed parity reference for its own
input batch (bench.py 'parity' field).

Inputs (exactly what bench.py and the parity tests feed the encoder; seeded on the CPU generator):
  c2: x = torch.rand(32, 3, 256, 256, Generator().manual_seed(1000)) * 2 - 1   (bench --config c2/c2g, rank 0)
  c4: x = torch.rand(2, 3, 1024, 1024, Generator().manual_seed(1000)) * 2 - 1  (the first 2 images of the C4 batch)
Encoder: torch.manual_seed(0); HVAE_VGG_Encoder(img_resolution=1024) -- the product's seeded construction, which
reproduces the reference's state dict bit for bit (tests/test_host.py::test_encoder_init_matches_reference_full_sha).
Fine projector fc1: torch.manual_seed(5); nn.Linear(128, 256) -- the reference re-creates it from the CPU generator
on every call (stylegan3_hvae_full.py:225-230); bench.py and the tests seed that draw with 5.
Means: oracle/encoder.py encoder_forward (fp32; pinned to the reference's own encoder by tests/golden/encoder_full.npz).

    python tests/golden/make_parity_means.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "parity_means.npz")

INPUTS = {"c2": (32, 256), "c4": (2, 1024)}


def bench_input(n, res, seed=1000):
    """bench.py's per-rank input batch (rank r: seed 1000 + r)."""
    return torch.rand(n, 3, res, res, generator=torch.Generator().manual_seed(seed)) * 2 - 1


def fine_fc1():
    torch.manual_seed(5)
    lin = torch.nn.Linear(128, 256)
    return lin.weight.detach(), lin.bias.detach()


def main():
    import image_compression_2_amd as ic2
    from oracle import encoder as oe
    torch.set_num_threads(os.cpu_count() or 1)
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd = {k: v.detach() for k, v in enc.state_dict().items() if not k.startswith("fine_projector.fc1")}
    fc1 = fine_fc1()
    out = {}
    for key, (n, res) in INPUTS.items():
        x = bench_input(n, res)
        with torch.no_grad():
            _, m, _ = oe.encoder_forward(sd, x, fine_fc1=fc1)
        out[f"{key}_means"] = m.numpy().astype(np.float32)
        out[f"{key}_x_sha256"] = np.frombuffer(hashlib.sha256(x.numpy().tobytes()).digest(), dtype=np.uint8)
        print(f"[parity_means] {key}: {n} x {res}^2 -> means {tuple(m.shape)}, |m| max {m.abs().max().item():.3f}")
    np.savez_compressed(OUT, **out)
    print(f"[parity_means] wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
