"""CPU precision gate for a Winograd F(2x2, 3x3) synthesis conv: the SG3-T-256 synthesis in
fp64, except that every modulated 3x3 conv runs as a mode would compute it on the GPU, with f16 storage of the
conv output and of the next layer's scaled input (the f16 synthesis path's storage points).  Reports per mode the
whole-synthesis SNR against the fp64 oracle and the uint8 PSNR change at the bench's two operating points.

    python tools/wino_emu.py [n_images] [mode ...]
    modes: fp64 | direct (f16 operands, f32 accumulation: today's kernel) | wino (V and U computed in f32, rounded
           to f16) | wino_h (V by two rounded f16 add passes, as packed f16 VALU would) | wino_nohalf (U = G g G^T
           with G's 1/2 folded into A^T: integer-coefficient G, the 1/4 applied in the output transform)
"""
import math
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, "/root/repo")
from oracle import sg3  # noqa: E402

torch.set_num_threads(8)
BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def h16(t):
    return t.to(torch.float16).to(torch.float64)


def wino_conv(x, w, pad, mode):
    """x [N,C,H,W] (f16 values in f64), w [O,C,3,3] (f64): correlation with zero padding `pad`, F(2x2,3x3)."""
    n, c, h, wd = x.shape
    ho, wo = h + 2 * pad - 2, wd + 2 * pad - 2
    ty, tx = (ho + 1) // 2, (wo + 1) // 2
    xp = F.pad(x, (pad, 2 * tx + 2 - wd - pad, pad, 2 * ty + 2 - h - pad))
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)                       # [N,C,ty,tx,4,4]
    if mode == "wino_h":
        v = h16(torch.einsum("ij,nctxjk->nctxik", BT, d))          # column pass, rounded
        v = h16(torch.einsum("nctxik,lk->nctxil", v, BT))          # row pass, rounded
    else:
        v = h16(torch.einsum("ij,nctxjk,lk->nctxil", BT, d, BT))
    if mode == "wino_nohalf":
        g2 = G * 2
        u = h16(torch.einsum("ij,ocjk,lk->ocil", g2, w, g2))      # 4x the usual U, rounded
    else:
        u = h16(torch.einsum("ij,ocjk,lk->ocil", G, w, G))
    m = torch.einsum("ocij,nctxij->notxij", u, v)                 # f32-accumulated on the GPU; fp64 here
    y = torch.einsum("ai,notxij,bj->notxab", AT, m, AT)           # [N,O,ty,tx,2,2]
    if mode == "wino_nohalf":
        y = y * 0.25
    y = y.permute(0, 1, 2, 4, 3, 5).reshape(n, -1, 2 * ty, 2 * tx)
    return y[:, :, :ho, :wo]


def layer(sd, L, x, w, mode):
    p = f"synthesis.{L['name']}."
    styles = sg3.fully_connected(w, sd[p + "affine.weight"].double(), sd[p + "affine.bias"].double())
    wt = sd[p + "weight"].double()
    ig = float(sd[p + "magnitude_ema"].double().rsqrt())
    if L["is_torgb"] or mode == "fp64":
        y = sg3.modulated_conv2d(x, wt, styles if not L["is_torgb"] else styles / math.sqrt(L["in_channels"]),
                                 demodulate=not L["is_torgb"], padding=L["conv_kernel"] - 1, input_gain=ig)
        if mode != "fp64":
            y = h16(y)
    else:
        wn = wt * wt.square().mean([1, 2, 3], keepdim=True).rsqrt()
        s = styles * styles.square().mean().rsqrt()
        dco = ((wn.square().sum([2, 3]).unsqueeze(0) * s.square().unsqueeze(1)).sum(2) + 1e-8).rsqrt()  # [N,O]
        xs = h16(x * s[:, :, None, None])                       # the producer stores x * xscale in f16
        if mode == "direct":
            acc = F.conv2d(xs, h16(wn), padding=2)
        else:
            acc = wino_conv(xs, wn, 2, mode)
        y = h16(acc * (dco * ig)[:, :, None, None])            # conv epilogue: oscale, f16 store
    fu, fd = sd.get(p + "up_filter"), sd.get(p + "down_filter")
    return sg3.filtered_lrelu(y, fu=None if fu is None else fu.double(), fd=None if fd is None else fd.double(),
                              b=sd[p + "bias"].double(), up=L["up"], down=L["down"], padding=L["padding"],
                              gain=1 if L["is_torgb"] else math.sqrt(2), slope=1 if L["is_torgb"] else 0.2,
                              clamp=256)


def synth(sd, ws, mode):
    inp, layers = sg3.layer_table(256)
    wsu = ws.double().unbind(1)
    x = sg3.synthesis_input(sd, inp, wsu[0], torch.float64)
    for L, w in zip(layers, wsu[1:]):
        x = layer(sd, L, x, w, mode)
    return x * 0.25


def psnr_u8(img, target):
    a = ((img.clamp(-1, 1) + 1) * 127.5).round()
    b = ((target.clamp(-1, 1) + 1) * 127.5).round()
    mse = (a - b).square().mean()
    return 10 * math.log10(255 ** 2 / max(mse.item(), 1e-12))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    modes = sys.argv[2:] or ["direct", "wino", "wino_h"]
    sd = sg3.init_params(256, seed=1)
    ws = torch.rand(n, 16, 512, generator=torch.Generator().manual_seed(2)) * 2 - 1
    t0 = time.time()
    ref = synth(sd, ws, "fp64")
    print(f"fp64 reference {time.time() - t0:.1f}s", flush=True)
    gen = torch.Generator().manual_seed(3)
    targets = {sig: (ref + torch.randn(ref.shape, generator=gen, dtype=torch.float64) * sig) for sig in (0.039, 0.01)}
    for mode in modes:
        t0 = time.time()
        img = synth(sd, ws, mode)
        err = img - ref
        snr = 10 * math.log10(ref.square().mean().item() / max(err.square().mean().item(), 1e-300))
        dps = {f"dpsnr_sigma{sig}": round(psnr_u8(img, t) - psnr_u8(ref, t), 5) for sig, t in targets.items()}
        print(f"{mode:12s} SNR {snr:.2f} dB  max|err| {err.abs().max().item():.3e}  {dps}  ({time.time() - t0:.1f}s)",
              flush=True)


if __name__ == "__main__":
    main()
