"""Diagnostic (not a test): where does the bf16 NHWC filtered-lrelu differ from the fp64 reference?"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import image_compression_2_amd as ic2  # noqa: E402
from image_compression_2_amd import _native as nv  # noqa: E402
from oracle import sg3  # noqa: E402

torch.manual_seed(1)
layers = ic2.Generator(img_resolution=256).synthesis.layers()
cuda = torch.device("cuda", 0)
for li in [int(v) for v in sys.argv[1:]] or [0]:
    L = layers[li]
    n, c_p = 1, 32
    conv = int(L.in_size[0]) + 2
    s_out = int(L.out_size[0])
    g = torch.Generator().manual_seed(20)
    x = (torch.randn(n, c_p, conv, conv, generator=g) * 2).to(torch.bfloat16).float()
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda, torch.bfloat16)
    out = torch.zeros(n, s_out, s_out, c_p, device=cuda, dtype=torch.bfloat16)
    nv.call("ic2_flrelu_nhwc", nv.ptr(xd), nv.ptr(out), nv.BF16, nv.BF16, n, c_p, conv, conv, s_out, s_out,
            L._fu.ctypes.data_as(ctypes.c_void_p), L._fu.shape[0], L._fd.ctypes.data_as(ctypes.c_void_p),
            L._fd.shape[0], None, L.up_factor, L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0,
            None, nv.stream_of(xd))
    torch.cuda.synchronize()
    r = sg3.filtered_lrelu(x.double(), torch.from_numpy(L._fu).double(), torch.from_numpy(L._fd).double(), None,
                           up=L.up_factor, down=L.down_factor, padding=L.padding, gain=np.sqrt(2), slope=0.2,
                           clamp=256.0).permute(0, 2, 3, 1).numpy()[0]
    y = out.float().cpu().numpy()[0]
    err = np.abs(y - r)
    bad = err > 0.05 * (1 + np.abs(r))
    print(f"layer {li}: max err {err.max():.3g}, ref max {np.abs(r).max():.3g}, out max {np.abs(y).max():.3g}, "
          f"bad frac {bad.mean():.3f}")
    print(" bad by channel:", np.round(bad.mean(axis=(0, 1)), 2).tolist())
    print(" bad by oy%16:", np.round(np.array([bad[o::16].mean() for o in range(16)]), 2).tolist())
    print(" bad by ox%16:", np.round(np.array([bad[:, o::16].mean() for o in range(16)]), 2).tolist())
    print(" sample y / r at (5,5,0..3):", y[5, 5, :4], r[5, 5, :4])
    print(" ratio y/r median:", np.median(y[np.abs(r) > 0.5] / r[np.abs(r) > 0.5]))
