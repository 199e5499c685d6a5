"""Debug: the MFMA FLR backward vs the f32 kernel on one SG3-T-256 layer, error map by tile row / column.
    python tools/dbg_fbm.py layer [n c_p]"""
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
    li = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    cp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    clamp_heavy = len(sys.argv) > 4 and sys.argv[4] == "1"
    with_os = len(sys.argv) > 5 and sys.argv[5] == "1"
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256)
    L = G.synthesis.layers()[li]
    s = int(L.in_size[0]) + 2
    so = int(L.out_size[0])
    g = torch.Generator().manual_seed(5)
    y = torch.randn(n, s, s, cp, generator=g) * 3
    if clamp_heavy:
        y[..., : cp // 3] = y[..., : cp // 3] * 60 + 150
    y = y.half().to(dev)
    os_ = (torch.rand(n, cp, generator=g) + 0.5).to(dev) if with_os else None
    gout = torch.randn(n, so, so, cp, generator=g).bfloat16().to(dev)
    outs = {}
    for name, gdt in (("mfma", nv.BF16), ("f32", nv.F32)):
        gx = torch.zeros(n, s, s, cp, device=dev, dtype=torch.bfloat16 if gdt == nv.BF16 else torch.float32)
        rc = nv.load().ic2_flrelu_bwd_nhwc_ex(
            nv.ptr(y), nv.F16, nv.ptr(gout), nv.BF16, nv.ptr(gx), gdt, n, cp, s, s, so, so,
            L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
            L._fd.shape[0], L.up_factor, L.down_factor, *L.padding, float(L.act_gain), 0.2, 256.0, 0,
            None if os_ is None else nv.ptr(os_), None,
            None, 0, nv.stream_of(y))
        assert rc == 0, nv.load().ic2_last_error().decode()
        outs[name] = gx.float().cpu()
    torch.cuda.synchronize()
    a, b = outs["mfma"], outs["f32"]
    print("clamp_heavy", clamp_heavy, "oscale", with_os, "n", n, "c_p", cp)
    print("layer", li, "U", L.up_factor, "pad", L.padding, "s", s, "rel", float((a - b).norm() / b.norm()))
    e = (a - b).abs().sum(dim=(0, 3))  # [s, s]
    bn = b.abs().sum(dim=(0, 3))
    tjx = 16 if L.up_factor == 2 else 8
    print("rel error by row (gx row):", np.round((e.sum(1) / bn.sum(1)).numpy(), 3).tolist())
    print("rel error by col:", np.round((e.sum(0) / bn.sum(0)).numpy(), 3).tolist())
    print("rel error by channel:", np.round(((a - b).abs().sum(dim=(0, 1, 2)) / b.abs().sum(dim=(0, 1, 2))).numpy(), 3).tolist())
    print("ratio mfma/f32 (sum |.|):", float(a.abs().sum() / b.abs().sum()), "tjx", tjx)


if __name__ == "__main__":
    main()
