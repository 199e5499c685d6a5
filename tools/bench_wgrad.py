"""Per-layer timing of the encoder weight gradient (ic2_conv_wgrad) on the C5 shapes: HVAE_VGG_Encoder
(img_resolution=1024) on 256^2 images, batch 16, f16 operands -- HIP events around `reps` back-to-back calls.
    python tools/bench_wgrad.py [label] [batch=16] [dtype=f16|bf16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dt = torch.bfloat16 if (len(sys.argv) > 3 and sys.argv[3] == "bf16") else torch.float16
    dev = torch.device("cuda", 0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    p32 = lambda c: (int(c) + 31) // 32 * 32  # noqa: E731
    shapes, h = [], 256
    for blk in enc.blocks:
        if h <= 1:
            break
        for conv in (blk.conv1, blk.conv2):
            shapes.append((p32(conv.in_channels), p32(conv.out_channels), h, conv.kernel_size[0], conv.padding[0]))
        h //= 2
    total_ms, total_gf = 0.0, 0.0
    for i, (cin, cout, h, k, pad) in enumerate(shapes):
        x = (torch.randn(n, h, h, cin, device=dev)).to(dt)
        ho = h + 2 * pad - k + 1
        dy = (torch.randn(n, ho, ho, cout, device=dev)).to(dt)
        dw = torch.empty(cout, k, k, cin, device=dev)
        nfl = int(nv.query("ic2_conv_wgrad_ws_floats", n, h, h, cin, cout, k, k, pad))
        ws = torch.empty(max(nfl, 1), device=dev)

        def call():
            nv.call("ic2_conv_wgrad", nv.ptr(x), nv.ptr(dy), nv.ptr(dw), nv.dtype_code(dt), n, h, h, cin, cout, k, k,
                    pad, nv.ptr(ws), nfl, nv.stream_of(x))
        for _ in range(3):
            call()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gf = 2.0 * n * ho * ho * cout * cin * k * k / 1e9
        total_ms += ms
        total_gf += gf
        print(f"{label:10s} conv{i:2d} {cin:4d}->{cout:4d} {h:4d}^2  {ms * 1e3:8.1f} us  {gf / ms:7.1f} TF/s "
              f"(ws {nfl * 4 / 2 ** 20:.0f} MiB)", flush=True)
    print(f"{label:10s} total {total_ms * 1e3:8.1f} us  {total_gf / total_ms:7.1f} TF/s (x2 per C5 step: two encoder passes)")


if __name__ == "__main__":
    main()
