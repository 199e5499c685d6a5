"""Diagnostic (debug build with -DIC2_FM_DEBUG): compare workgroup 0's LDS images of the MFMA
filtered-lrelu with a numpy restatement of the same stages."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import image_compression_2_amd as ic2  # noqa: E402
from image_compression_2_amd import _native as nv  # noqa: E402

torch.manual_seed(1)
L = ic2.Generator(img_resolution=256).synthesis.layers()[int(sys.argv[1]) if len(sys.argv) > 1 else 0]
cuda = torch.device("cuda", 0)
n, c_p = 1, 16
conv = int(L.in_size[0]) + 2
s_out = int(L.out_size[0])
g = torch.Generator().manual_seed(20)
x = (torch.randn(n, conv, conv, c_p, generator=g) * 2).to(torch.bfloat16)
xd = x.to(cuda)
out = torch.zeros(n, s_out, s_out, c_p, device=cuda, dtype=torch.bfloat16)
nv.call("ic2_flrelu_nhwc", nv.ptr(xd), nv.ptr(out), nv.BF16, nv.BF16, n, c_p, conv, conv, s_out, s_out,
        L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
        L._fd.shape[0], None, L.up_factor, L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0,
        None, nv.stream_of(xd))
torch.cuda.synchronize()
lib = nv.load()
dumps = []
for w in range(3):
    buf = np.zeros(8192, dtype=np.uint32)
    assert lib.ic2_fm_debug_fetch(buf.ctypes.data_as(ctypes.c_void_p), w) == 0
    dumps.append(buf)


def bf_pairs(words):  # uint32 words -> float pairs (low half first)
    lo = (words.astype(np.uint32) << 16).view(np.float32)
    hi = (words.astype(np.uint32) & 0xffff0000).view(np.float32)
    return np.stack([lo, hi], -1).reshape(*words.shape[:-1], -1)


U = L.up_factor
TU = 6 * U
px0 = L.padding[0]
DELTA = ((px0 % U) + U) % U
RA = 42
NIN = (RA + TU - 2) // U + 1
xin = x.float().numpy()[0]
sy0 = (0 - L.padding[2] + DELTA) // U
sx0 = (0 - px0 + DELTA) // U
img = np.zeros((NIN, NIN, 16))
for jy in range(NIN):
    for xx in range(NIN):
        iy, ix = sy0 + jy, sx0 + xx
        if 0 <= iy < conv and 0 <= ix < conv:
            img[jy, xx] = xin[iy, ix]
got_in = bf_pairs(dumps[0][: NIN * NIN * 8].reshape(NIN, NIN, 8))
print("input image max|diff|:", np.abs(got_in - img).max())
gu = np.zeros(24)
gu[:TU] = L._fu[::-1] * U


def win(i):
    j = 0 if i < DELTA else (i - DELTA + U - 1) // U
    return min(j, NIN - 16)


G0 = np.zeros((16, 16))
for li in range(16):
    for k in range(16):
        tap = U * (win(0) + k) + DELTA - li
        if 0 <= tap < TU:
            G0[li, k] = gu[tap]
V = np.einsum("yk,kxc->yxc", G0, img[win(0):win(0) + 16])
vp = NIN * 8 + 2
got_v = bf_pairs(dumps[1][: 16 * vp].reshape(16, vp)[:, : NIN * 8].reshape(16, NIN, 8))
dv = np.abs(got_v - V)
print("V image max|diff|:", dv.max(), " by channel:", np.round(dv.max(axis=(0, 1)), 3).tolist())
print("  V[0,0,:4] got", got_v[0, 0, :4], "want", V[0, 0, :4])
print("  by ky:", np.round(dv.max(axis=(1, 2)), 3).tolist())

# ---- D image of block 0 from the device V image (isolates the horizontal stage)
gd = L._fd[::-1].astype(np.float64)
gdg = gd * np.sqrt(2)
lim = 256 / np.sqrt(2)
Gt = []
for t in range(3):
    M = np.zeros((16, 16))
    for li in range(16):
        for k in range(16):
            tap = U * (win(16 * t) + k) + DELTA - (16 * t + li)
            if 0 <= tap < TU:
                M[li, k] = gu[tap]
    Gt.append(M)
GdH = np.zeros((48, 16))
for kx in range(48):
    for ox in range(16):
        if 0 <= kx - 2 * ox < 12:
            GdH[kx, ox] = gdg[kx - 2 * ox]
Dref = np.zeros((16, 16, 16))
for kyl in range(16):
    us = []
    for t in range(3):
        u = Gt[t] @ got_v[kyl, win(16 * t):win(16 * t) + 16, :]
        us.append(np.clip(np.maximum(u, 0.2 * u), -lim, lim))
    Dref[kyl] = GdH.T @ np.concatenate(us, 0)
got_d = bf_pairs(dumps[2][: 16 * 168].reshape(16, 168)[:, :160].reshape(16, 16, 10)[:, :, :8])
dd = np.abs(got_d - Dref)
print("D image max|diff|:", dd.max(), " by channel:", np.round(dd.max(axis=(0, 1)), 3).tolist())
print("  by ox:", np.round(dd.max(axis=(0, 2)), 3).tolist())
print("  D[3,3,:4] got", got_d[3, 3, :4], "want", Dref[3, 3, :4])
