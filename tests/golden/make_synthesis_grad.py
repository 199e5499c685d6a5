"""Generates tests/golden/synthesis_grad.npz: dL/dws through the fp64 oracle synthesis (oracle/sg3.py, autograd) for
tests/test_gpu_training.py::test_synthesis_network_gradient_wrt_ws, so the GPU box does not run the fp64 CPU
synthesis backward (~75 s) inside the GPU suite.  CPU only, build container.

Inputs, exactly the test's: torch.manual_seed(1); Generator(img_resolution=256) with magnitude_ema = 0.6 + 0.05 i per
layer (the gen256_frozen fixture); ws = randn(2, 16, 512, Generator().manual_seed(3)) * 0.7;
r = randn(2, 3, 256, 256, Generator().manual_seed(6)); L = sum(img * r).

    python tests/golden/make_synthesis_grad.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "synthesis_grad.npz")


def frozen_generator():
    import image_compression_2_amd as ic2
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256).eval().requires_grad_(False)
    with torch.no_grad():
        for i, L in enumerate(G.synthesis.layers()):
            L.magnitude_ema.fill_(0.6 + 0.05 * i)
    return G


def inputs():
    ws = torch.randn(2, 16, 512, generator=torch.Generator().manual_seed(3)) * 0.7
    r = torch.randn(2, 3, 256, 256, generator=torch.Generator().manual_seed(6))
    return ws, r


def main():
    from oracle import sg3
    torch.set_num_threads(os.cpu_count() or 1)
    G = frozen_generator()
    sd = {k: v.detach().double() for k, v in G.state_dict().items()}
    ws, r = inputs()
    wr = ws.double().requires_grad_(True)
    img = sg3.synthesis_forward(sd, 256, wr, dtype=torch.float64)
    (img * r.double()).sum().backward()
    np.savez_compressed(OUT, dws=wr.grad.numpy(), ws=ws.numpy())
    print(f"[synthesis_grad] wrote {OUT} ({os.path.getsize(OUT)} bytes), |dws| {wr.grad.norm().item():.4e}")


if __name__ == "__main__":
    main()
