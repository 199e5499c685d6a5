"""Debug: test_flrelu_backward_mfma_kernel's construction, MFMA vs f32 kernel vs the fp64 oracle."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.nn.functional as F
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    from oracle import sg3
    li = int(sys.argv[1])
    cuda = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256)
    L = G.synthesis.layers()[li]
    c, cp = L.out_channels, L.cout_p
    n = 2
    s = int(L.in_size[0]) + L.conv_kernel - 1
    so = int(L.out_size[0])
    g = torch.Generator().manual_seed(100 + li)
    y = torch.randn(n, s, s, c, generator=g) * 3
    y[..., : c // 3] = y[..., : c // 3] * 60 + 150
    y = F.pad(y, (0, cp - c)).half()
    gout = F.pad(torch.randn(n, so, so, c, generator=g), (0, cp - c)).bfloat16()
    os_ = torch.rand(n, cp, generator=g) + 0.5
    bias = torch.randn(cp, generator=g)
    yd, gd_, osd, bd = y.to(cuda), gout.to(cuda), os_.to(cuda), bias.to(cuda)
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
    res = {}
    for name, dt, code in (("mfma", torch.bfloat16, nv.BF16), ("f32", torch.float32, nv.F32)):
        dc = (torch.empty if mode == "empty" else torch.zeros)(n, s, s, cp, device=cuda, dtype=dt)
        use_os = mode in ("os", "all")
        nyd = int(nv.query("ic2_flrelu_bwd_ydot_floats", n, cp, s, s, L.up_factor))
        ydot = torch.full([nyd], float("nan"), device=cuda)
        rc = nv.load().ic2_flrelu_bwd_nhwc_ex(
            nv.ptr(yd), nv.F16, nv.ptr(gd_), nv.BF16, nv.ptr(dc), code, n, cp, s, s, so, so,
            L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p), L._fd.shape[0],
            L.up_factor, L.down_factor, *L.padding, float(L.act_gain), 0.2, float(L.conv_clamp), 0,
            nv.ptr(osd) if use_os else None, nv.ptr(bd) if mode == "all" else None,
            nv.ptr(ydot) if mode == "all" else None, nyd if mode == "all" else 0, nv.stream_of(yd))
        assert rc == 0
        res[name] = (dc.float().cpu() / (os_[:, None, None, :] if use_os else 1.0))[..., :c]
    torch.cuda.synchronize()
    yr = y.double()[..., :c].permute(0, 3, 1, 2).requires_grad_(True)
    _, layers = sg3.layer_table(256)
    Lr = layers[li]
    print("mode", mode)
    print("layer", li, Lr["name"] if "name" in Lr else "", "up", Lr["up"], "pad", Lr["padding"], "L.padding", L.padding,
          "act_gain", L.act_gain, "clamp", L.conv_clamp)
    o = sg3.filtered_lrelu(yr, Lr["up_filter"].double(), Lr["down_filter"].double(), up=Lr["up"], down=Lr["down"],
                           padding=Lr["padding"], clamp=256)
    o.backward(gout.double()[..., :c].permute(0, 3, 1, 2))
    ref = yr.grad.permute(0, 2, 3, 1)
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())
    print("mfma vs oracle", rel(res["mfma"], ref), "f32 vs oracle", rel(res["f32"], ref), "mfma vs f32",
          rel(res["mfma"], res["f32"]))
    for nn in range(n):
        print(" sample", nn, "mfma", rel(res["mfma"][nn], ref[nn]), "f32", rel(res["f32"][nn], ref[nn]))
    cb = [rel(res["mfma"][..., k:k + 16], ref[..., k:k + 16]) for k in range(0, c, 16)]
    print(" per channel block mfma:", np.round(cb, 3).tolist())


if __name__ == "__main__":
    main()
