"""Generates tests/golden/synthesis_ref.npz: the fp64 oracle synthesis (oracle/sg3.py) of the seeded SG3-T-256
generator for tests/test_gpu_path.py::test_synthesis_fp32_within_1e3_of_oracle, so the GPU box does not run the fp64
CPU synthesis (~30 s) inside the GPU suite.  CPU only, build container.

Inputs, exactly the test's: torch.manual_seed(1); Generator(img_resolution=256) (the gen256 fixture, default buffers);
ws = randn(2, 16, 512, Generator().manual_seed(3)) * 0.7.  Stored: the image as f32 (the bar is 1e-3 max-abs; f32
rounding of the fp64 values is ~1e-7), ws, and a sha256 of the generator's state dict, which
tests/test_oracle.py::test_synthesis_ref_fixture_inputs recomputes so a changed initialisation cannot go unnoticed.

    python tests/golden/make_synthesis_ref.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "synthesis_ref.npz")


def generator():
    import image_compression_2_amd as ic2
    torch.manual_seed(1)
    return ic2.Generator(img_resolution=256).eval()


def state_sha(G):
    h = hashlib.sha256()
    for k, v in sorted(G.state_dict().items()):
        h.update(k.encode())
        h.update(v.detach().float().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def inputs():
    return torch.randn(2, 16, 512, generator=torch.Generator().manual_seed(3)) * 0.7


def main():
    from oracle import sg3
    torch.set_num_threads(os.cpu_count() or 1)
    G = generator()
    sd = {k: v.detach().float().cpu() for k, v in G.state_dict().items()}
    ws = inputs()
    with torch.no_grad():
        img = sg3.synthesis_forward(sd, 256, ws, dtype=torch.float64)
    np.savez_compressed(OUT, img=img.float().numpy(), ws=ws.numpy(), state_sha256=np.frombuffer(
        bytes.fromhex(state_sha(G)), dtype=np.uint8))
    print(f"[synthesis_ref] wrote {OUT} ({os.path.getsize(OUT)} bytes), max|img| {img.abs().max().item():.4f}")


if __name__ == "__main__":
    main()
