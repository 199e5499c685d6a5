"""Eager vs graph-captured C5 training step (bench's C5 setup: f16 + loss scaler, B=16, 256^2) on one box:
ms/step of each over the same number of steps, and the losses of both runs (same initial weights; the noise
streams differ, so the losses agree to within the noise, not bit for bit).

    python tools/graph_c5_ab.py [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(graphed):
    import image_compression_2_amd as ic2
    from image_compression_2_amd import training as ict
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision="f16").to(dev)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256, precision="f16").to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G, training_resolution=256)
    x = (torch.rand(16, 3, 256, 256, generator=torch.Generator().manual_seed(1000)) * 2 - 1).to(dev)
    opt = ict.make_optimizer(enc, lr=1e-4, capturable=graphed)
    w_avg = G.mapping.w_avg.view(1, 1, -1)
    scaler = ict.make_f16(comp)
    kw = dict(rec_weight=1.0, perceptual_weight=0.0, kl_weight=0.01, scaler=scaler)
    if graphed:
        return ict.GraphedTrainStep(comp, x, opt, w_avg, warmup=3, **kw)
    return lambda: ict.train_step(comp, x, opt, w_avg, **kw)


def run(graphed, steps):
    t0 = time.time()
    step = build(graphed)
    print(f"{'graph' if graphed else 'eager'} setup {time.time() - t0:.1f} s", flush=True)
    losses = []
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
        losses.append(out["rec_loss"].clone())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    ls = [float(v) for v in losses]
    print(f"{'graph' if graphed else 'eager'}: {ms:.2f} ms/step  {16e3 / ms:.1f} img/s  rec_loss first/last "
          f"{ls[0]:.5f} / {ls[-1]:.5f}", flush=True)
    return ms, ls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    e = run(False, args.steps)
    g = run(True, args.steps)
    print(f"speedup {e[0] / g[0]:.3f}x")


if __name__ == "__main__":
    main()
