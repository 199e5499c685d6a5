"""Runs one synthesis layer's fused filtered lrelu (C2 shape: SG3-T-256, batch 32, f16 NHWC16 in, bf16/f16 out)
`reps` times back to back -- a short target for rocprofv3 (kernel trace, PMC passes, PC sampling).
    python tools/flr_one.py [layer=8] [reps=20] [out=bf16|f16]"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    odt = torch.float16 if (len(sys.argv) > 3 and sys.argv[3] == "f16") else torch.bfloat16
    n = 32
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    L = ic2.Generator(img_resolution=256).synthesis.layers()[li]
    conv, s_out, c_p = int(L.in_size[0]) + 2, int(L.out_size[0]), L.cout_p
    x = (torch.randn(n, c_p // 16, conv, conv, 16, device=dev) * 2).to(torch.float16)
    out = torch.empty(n, s_out, s_out, c_p, device=dev, dtype=odt)
    ps = torch.rand(n, c_p, device=dev) + 0.5
    for _ in range(reps):
        nv.call("ic2_flrelu_nhwc16", nv.ptr(x), nv.ptr(out), nv.F16, nv.dtype_code(odt), n, c_p, conv, conv, s_out, s_out,
                L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
                L._fd.shape[0], None, L.up_factor, L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0,
                nv.ptr(ps), nv.stream_of(x))
    torch.cuda.synchronize()
    print(f"[flr_one] L{li} {conv}->{s_out} x {c_p} up {L.up_factor}: {reps} launches done")


if __name__ == "__main__":
    main()
