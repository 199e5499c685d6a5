"""Per-section cycle split of ic2_conv_wino from the IC2_WX_STAMP diagnostic build (tools/build_abl.sh winostamp 1):
    IC2_DEV=1 IC2_DEV_LIB=$PWD/image_compression_2_amd/libic2ops_wxstamp1.so python tools/wino_stamps.py [cin cout size]
Prints, per wave half, the mean cycles per K-step of: R reads + V, R DMA issue, vmcnt wait, barrier after R, M issue,
barrier after M."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from image_compression_2_amd import _native as nv
    cin, cout, s = [int(v) for v in (sys.argv[1:] + ["512", "512", "148"][len(sys.argv) - 1:])]
    dev = torch.device("cuda", 0)
    n, pad = 32, 2
    ho = s + 2
    x = torch.randn(n, s, s, cin, device=dev).to(torch.float16)
    w = torch.randn(cout, cin, 3, 3, device=dev)
    u = torch.empty(cout, 3, 4, cin, device=dev, dtype=torch.float16)
    st = nv.stream_of(x)
    nv.call("ic2_pack_weight_wino", nv.ptr(w), cout, cin, cout, cin, 1, 1.0, nv.ptr(u), nv.F16, st)
    y = torch.empty(n, ho, ho, cout, device=dev, dtype=torch.float16)
    buf = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    nv.call("ic2_conv_wino_stamps", nv.ptr(buf), buf.numel())
    for _ in range(3):
        nv.call("ic2_conv_wino", nv.ptr(x), nv.ptr(u), nv.ptr(y), nv.F16, nv.F16, n, s, s, cin, cout, cout, pad, ho, ho,
                None, None, 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, st)
    torch.cuda.synchronize()
    name = nv.wino_plan(n, s, s, cin, cout, pad)
    t = buf.view(torch.int64).cpu()
    nz = int((t.view(-1, 8, 8)[:, 0, 6] > 0).sum())
    rec = t.view(-1, 8, 8)[:nz].double()
    steps = 3 * cin // 32
    labels = ["R reads+V", "R DMA issue", "vmcnt wait", "barrier after R", "M issue", "barrier after M", "loop total"]
    print(f"{name}: {nz} workgroups, {steps} K-steps; cycles per K-step (s_memtime), mean over workgroups")
    for h in range(2):
        r = rec[:, 4 * h:4 * h + 4, :].reshape(-1, 8).mean(0) / steps
        print(f"  waves {4 * h}-{4 * h + 3}: " + ", ".join(f"{labels[k]} {r[k]:.0f}" for k in range(7)))


if __name__ == "__main__":
    main()
