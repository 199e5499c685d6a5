"""Diagnostic: the MFMA FLR backward with its oscale row DMA'd into LDS (FBM_OS_DMA=2 build,
loaded under IC2_DEV=1 IC2_DEV_LIB=.../libic2ops_osdma.so) checks every item's LDS row against a plain load and
counts mismatches.  Runs the test geometries (up 4: L3, L5, L10; up 2: L2, L9).
    IC2_DEV=1 IC2_DEV_LIB=$PWD/image_compression_2_amd/libic2ops_osdma.so python tools/dbg_fbm_osdma.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lds_dw(up):
    """FbmGeom<U, TJX>::LDS_DW (the slot's dword index), restated from flrelu_bwd_mfma.hip (TJX 16 / 8 at up 2 / 4)."""
    tjx = 16 if up == 2 else 8
    s, ngx, nbx = 16 // up, up + 1, (up * (tjx - 1) + 6 * up + 15) // 16
    ninx, nox = (16 * (nbx - 1) // up + 6 + 15 // up) | 1, (8 * (nbx - 1) + 14) | 1
    xgi, ggi = (s * ninx * 2 + 63) // 64, (8 * nox * 2 + 63) // 64
    return ngx * xgi * 256 + 3 * ggi * 256 + 16 * (ninx * 8 + 2) + 16 * (nox * 8 + 2)


def main():
    import numpy as np
    import torch
    import torch.nn.functional as F
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    lib = nv.load()
    lib.ic2_fbm_debug_fetch.argtypes = [ctypes.c_void_p]
    cuda = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256).to(cuda).eval().requires_grad_(False)
    lib.ic2_fbm_debug_reset.argtypes = [ctypes.c_uint]
    for mode, li in [(0, li) for li in (3, 5, 10, 2, 9)] + [(1, 3), (1, 2)]:
        L = G.synthesis.layers()[li]
        c, cp, n = L.out_channels, L.cout_p, 2
        s = int(L.in_size[0]) + L.conv_kernel - 1
        so = int(L.out_size[0])
        g = torch.Generator().manual_seed(100 + li)
        y = F.pad(torch.randn(n, s, s, c, generator=g) * 3, (0, cp - c)).half().to(cuda)
        gout = F.pad(torch.randn(n, so, so, c, generator=g), (0, cp - c)).bfloat16().to(cuda)
        os_ = (torch.rand(n, cp, generator=g) + 0.5).to(cuda)
        bias = torch.randn(cp, generator=g).to(cuda)
        dc = torch.empty(n, s, s, cp, device=cuda, dtype=torch.bfloat16)
        nyd = int(nv.query("ic2_flrelu_bwd_ydot_floats", n, cp, s, s, L.up_factor))
        ydot = torch.empty([nyd], device=cuda)
        lib.ic2_fbm_debug_reset(mode)
        rc = lib.ic2_flrelu_bwd_nhwc_ex(
            nv.ptr(y), nv.F16, nv.ptr(gout), nv.BF16, nv.ptr(dc), nv.BF16, n, cp, s, s, so, so,
            L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
            L._fd.shape[0], L.up_factor, L.down_factor, *L.padding, float(L.act_gain), 0.2, float(L.conv_clamp), 0,
            nv.ptr(os_), nv.ptr(bias), nv.ptr(ydot), nyd, nv.stream_of(y))
        torch.cuda.synchronize()
        buf = (ctypes.c_uint * 64)()
        lib.ic2_fbm_debug_fetch(ctypes.cast(buf, ctypes.c_void_p))
        d = list(buf)
        f = lambda u: float(np.array([u], dtype=np.uint32).view(np.float32)[0])  # noqa: E731
        print(f"[fbm-osdma] mode {mode} L{li} up {L.up_factor} rc {rc}: at issue good {d[5]} bad {d[6]}; rows read {d[4]}, mismatches {d[0]} (first item {d[1]}, "
              f"later {d[2]}, = previous item's row {d[3]}); per wave {d[8:16]}; per lane group {d[16:20]}", flush=True)
        if d[32]:
            print(f"    first: item {d[33]} wave {d[34]} lane {d[35]} got {f(d[36]):.6f} want {f(d[37]):.6f} prev item "
                  f"{d[38] if d[38] != 0xffffffff else -1} block {d[39]} nitems {d[40]} grid {d[41]}", flush=True)
            print(f"    slot {[round(f(u), 4) for u in d[42:58]]}; slot's last DMA for item {d[62]}; expected value at LDS "
                  f"dwords {d[58:62]} (slot at {lds_dw(L.up_factor)})", flush=True)


if __name__ == "__main__":
    main()
