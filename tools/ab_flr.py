"""Per-layer timing of the fused filtered lrelu on the C2 shapes (SG3-T-256, batch 32, f16 NHWC16 in, bf16 out),
HIP events around 20 back-to-back calls per layer.  python tools/ab_flr.py [label]  (A/B: run once with
IC2_DEV=1 IC2_FLR_STRIP=0 for the round-2 tile kernel)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    res = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=res, precision="bf16").to(dev)
    total = 0.0
    for li, L in enumerate(G.synthesis.layers()):
        if L.is_torgb:
            continue
        conv = int(L.in_size[0]) + 2
        s_out = int(L.out_size[0])
        c_p = L.cout_p
        x = (torch.randn(n, c_p // 16, conv, conv, 16, device=dev) * 2).to(torch.float16)
        out = torch.empty(n, s_out, s_out, c_p, device=dev, dtype=torch.bfloat16)
        ps = torch.rand(n, c_p, device=dev) + 0.5

        def call():
            nv.call("ic2_flrelu_nhwc16", nv.ptr(x), nv.ptr(out), nv.F16, nv.BF16, n, c_p, conv, conv, s_out, s_out,
                    L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
                    L._fd.shape[0], None, L.up_factor, L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0,
                    nv.ptr(ps), nv.stream_of(x))
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        total += us
        byts = (conv * conv + s_out * s_out) * L.out_channels * 2 * n
        print(f"{label:10s} {G.synthesis.layer_names[li]:14s} up {L.up_factor} {us:8.1f} us  "
              f"{byts / us / 1e3:7.0f} GB/s (alg)", flush=True)
    print(f"{label:10s} total {total:8.1f} us")


if __name__ == "__main__":
    main()
