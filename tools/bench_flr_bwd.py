"""Per-layer timing of the fused filtered-lrelu backward (ic2_flrelu_bwd_nhwc) on the SG3-T-256 layers at the
C5 batch, bf16 mode (f16 input, bf16 output gradient).  IC2_FLRB_VARIANT selects the tile variant (read once
per process).  Prints one JSON line: per-layer ms and a checksum of the gradients."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import image_compression_2_amd as ic2  # noqa: E402
from image_compression_2_amd import _native as nv  # noqa: E402


def main():
    batch = int(os.environ.get("B", "16"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256).to(dev)
    res, total, csum = {}, 0.0, 0.0
    lib = nv.load()
    for L in G.synthesis.layers():
        if L.is_torgb:
            continue
        s = int(L.in_size[0]) + L.conv_kernel - 1
        so = int(L.out_size[0])
        g = torch.Generator(device=dev).manual_seed(3)
        y = (torch.randn(batch, s, s, L.cout_p, generator=g, device=dev) * 3).half()
        dout = torch.randn(batch, so, so, L.cout_p, generator=g, device=dev).bfloat16()
        dy = torch.empty(batch, s, s, L.cout_p, dtype=torch.float32, device=dev)
        px0, px1, py0, py1 = L.padding

        def run():
            rc = lib.ic2_flrelu_bwd_nhwc(nv.ptr(y), nv.F16, nv.ptr(dout), nv.BF16, nv.ptr(dy), batch, L.cout_p, s, s, so,
                                         so, L._fu.ctypes.data_as(nv.ctypes.c_void_p), L._fu.shape[0],
                                         L._fd.ctypes.data_as(nv.ctypes.c_void_p), L._fd.shape[0], L.up_factor,
                                         L.down_factor, px0, px1, py0, py1, float(L.act_gain), 0.2, 256.0, 0,
                                         nv.stream_of(y))
            assert rc == 0, lib.ic2_last_error()
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        name = f"L{L.up_factor}x_{s}_{L.cout_p}"
        res[name] = round(ms, 3)
        total += ms
        csum += float(dy.double().abs().sum())
    print(json.dumps({"variant": os.environ.get("IC2_FLRB_VARIANT", "default"), "batch": batch,
                      "total_ms": round(total, 3), "layers_ms": res, "checksum": csum}))


if __name__ == "__main__":
    main()
