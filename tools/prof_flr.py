"""Run one synthesis-layer fused filtered-lrelu (SG3-T-256 layer shapes, batch 32, bf16 NHWC) a few
times: the target for rocprofv3 --pmc passes.   python tools/prof_flr.py [layer_index reps]"""
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
    li = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256, precision="bf16").to(dev)
    L = G.synthesis.layers()[li]
    n = 32
    conv = int(L.in_size[0]) + 2
    s_out = int(L.out_size[0])
    y = (torch.randn(n, conv, conv, L.cout_p, device=dev) * 2).to(torch.float16)
    out = torch.empty(n, s_out, s_out, L.cout_p, device=dev, dtype=torch.bfloat16)
    for _ in range(reps):
        nv.call("ic2_flrelu_nhwc", nv.ptr(y), nv.ptr(out), nv.F16, nv.BF16, n, L.cout_p, conv, conv, s_out, s_out,
                L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
                L._fd.shape[0], None, L.up_factor, L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0, None,
                nv.stream_of(y))
    torch.cuda.synchronize()
    print("ok", G.synthesis.layer_names[li], float(out.float().abs().mean()))


if __name__ == "__main__":
    main()
