"""Winograd F(2,3)-along-x conv (ic2_conv_wino) against the direct implicit GEMM (ic2_conv_igemm_ws) on the
SG3-T-256 synthesis conv shapes at batch 32, f16 operands, NHWC16 f16 output (what the synthesis path runs):
time, algorithmic TF/s and the error of each against an fp32 torch conv of the same f16 operands.

    python tools/bench_wino.py [shape ...]     (IC2_DEV=1 knobs IC2_WINO_TWP / IC2_WINO_TH force a tile)
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, cin, cout, size_in): SG3-T-256 modulated convs (pad 2) and the hg4 layers
SHAPES = [("s36", 512, 512, 36), ("s52", 512, 512, 52), ("s84", 512, 512, 84), ("s148", 512, 512, 148),
          ("s148b", 512, 362, 148), ("s148c", 362, 256, 148), ("s276a", 256, 181, 276), ("s276b", 181, 128, 276),
          ("s276c", 128, 128, 276)]


def main():
    from image_compression_2_amd import _native as nv
    dev = torch.device("cuda", 0)
    only = set(sys.argv[1:])
    n, pad = int(os.environ.get("BW_N", 32)), 2
    res = {}
    for name, ci, co, s in SHAPES:
        if only and name not in only:
            continue
        cip, cop = nv.pad_synth(ci), nv.pad_synth(co)
        ho = s + 2
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.zeros(n, s, s, cip, device=dev, dtype=torch.float16)
        x[..., :ci] = torch.randn(n, s, s, ci, device=dev, generator=g).to(torch.float16)
        w = torch.randn(co, ci, 3, 3, device=dev, generator=g)
        wp = torch.empty(cop, 3, 3, cip, device=dev, dtype=torch.float16)
        u = torch.empty(cop, 3, 4, cip, device=dev, dtype=torch.float16)
        st = nv.stream_of(x)
        nv.call("ic2_pack_weight", nv.ptr(w), co, ci, 3, 3, cop, cip, 1, 1.0, nv.ptr(wp), nv.F16, None, st)
        nv.call("ic2_pack_weight_wino", nv.ptr(w), co, ci, cop, cip, 1, 1.0, nv.ptr(u), nv.F16, st)
        osc = (torch.rand(n, cop, device=dev, generator=g) + 0.5) / (9 * ci) ** 0.5
        bias = torch.zeros(cop, device=dev)
        yd = torch.empty(n, cop // 16, ho, ho, 16, device=dev, dtype=torch.float16)
        yw = torch.empty_like(yd)

        def direct():
            nv.conv_igemm(nv.ptr(x), nv.ptr(wp), nv.ptr(yd), nv.F16, nv.F16, n, s, s, cip, cop, co, 3, 3, pad, ho, ho,
                          nv.ptr(osc), nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC16, st, dev)

        def wino():
            nv.conv_wino(nv.ptr(x), nv.ptr(u), nv.ptr(yw), nv.F16, nv.F16, n, s, s, cip, cop, co, pad, ho, ho,
                         nv.ptr(osc), nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC16, st)

        row = {"plan_direct": nv.conv_plan(nv.F16, nv.F16, nv.NHWC16, n, s, s, cip, cop, co, 3, 3, pad),
               "plan_wino": nv.wino_plan(n, s, s, cip, cop, pad)}
        flops = 2.0 * n * ho * ho * co * ci * 9
        for tag, fn in (("direct", direct), ("wino", wino)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            row[tag] = [round(us, 1), round(flops / us / 1e6, 1)]
        # fp32 reference on the same f16 operands (first 2 images)
        wn = w * w.square().mean([1, 2, 3], keepdim=True).rsqrt()
        xr = x[:2, :, :, :ci].float().permute(0, 3, 1, 2)
        ref = F.conv2d(xr, wn.to(torch.float16).float(), padding=pad) * osc[:2, :co, None, None]
        scale = ref.abs().max().item()

        def err(y):
            yy = y[:2].permute(0, 1, 4, 2, 3).reshape(2, cop, ho, ho)[:, :co].float()
            return (yy - ref).abs().max().item() / scale
        row["max_err_rel_direct"] = float("%.3e" % err(yd))
        row["max_err_rel_wino"] = float("%.3e" % err(yw))
        row["speedup"] = round(row["direct"][0] / row["wino"][0], 3)
        res[name] = row
        print(name, json.dumps(row), flush=True)
        del x, w, wp, u, yd, yw
    return res


if __name__ == "__main__":
    main()
