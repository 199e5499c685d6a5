"""Probe: how much of the C2 step can two concurrent half-batch pipelines recover?

    python tools/overlap_probe.py [--precision f16|bf16] [--steps 20] [--warmup 5]

Modes (each: K steps of compress -> decompress -> uint8 SSE over a batch of 32 256^2 images, wall time between
synchronizes; the per-step fine-projector fc1 draw is seeded as in bench.py):
  one      the bench step (one stream, batch 32)
  two      two streams, batch 16 each, started together
  offset   two streams, batch 16 each; stream 2 starts its half when stream 1's half has finished its encoder
  synth2   encoder on one stream (batch 32), then the two synthesis halves on two streams, stream 2 one layer behind
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="f16")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--modes", default="one,synth2,one")
    args = ap.parse_args()
    import bench
    import image_compression_2_amd as ic2
    from image_compression_2_amd import metrics as icm
    enc_prec, syn_prec = bench.PRECISIONS[args.precision]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=enc_prec).to(dev).eval().requires_grad_(False)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256, precision=syn_prec).to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G)
    x = torch.rand(32, 3, 256, 256, generator=torch.Generator(device=dev).manual_seed(1000), device=dev) * 2 - 1
    xa, xb = x[:16].contiguous(), x[16:].contiguous()
    main_s = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def half(xh):
        q = comp.compress(xh, 8, True)
        img = comp.decompress(q)
        return icm.uint8_sse(img, xh)

    def step_one():
        torch.manual_seed(5)
        with torch.no_grad():
            return half(x)

    def step_two(offset):
        torch.manual_seed(5)
        ev0 = torch.cuda.Event()
        ev0.record(main_s)
        with torch.no_grad():
            with torch.cuda.stream(s1):
                s1.wait_event(ev0)
                q = comp.compress(xa, 8, True)
                e_enc = torch.cuda.Event()
                e_enc.record(s1)
                ra = icm.uint8_sse(comp.decompress(q), xa)
            with torch.cuda.stream(s2):
                s2.wait_event(e_enc if offset else ev0)
                rb = half(xb)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)
        return ra, rb

    S = G.synthesis
    layers = S.layers()
    sdt = torch.float16 if syn_prec == "f16" else torch.bfloat16
    ldx = S.num_ws * S.w_dim

    def step_synth2():
        """encoder + quantizer on the main stream (batch 32); the synthesis as two batch-16 chains on two streams,
        the conv launches alternating A, B, A, B (B's conv of layer L after A's, A's conv of L+1 after B's of L), so
        each half's filtered lrelu runs beside the other half's conv"""
        torch.manual_seed(5)
        with torch.no_grad():
            q = comp.compress(x, 8, True)
            ev0 = torch.cuda.Event()
            ev0.record(main_s)
            halves = [q[:16].contiguous(), q[16:].contiguous()]
            st = [s1, s2]
            xs, scs = [None, None], [None, None]
            for h in range(2):
                with torch.cuda.stream(st[h]):
                    st[h].wait_event(ev0)
                    ws = halves[h]
                    scs[h] = S.scales_batched(ws, ldx, 16, sdt)
                    xs[h] = S.input.run_nhwc(ws, ldx, 16, sdt, scs[h][0][0])
            prev_b = None
            for i, L in enumerate(layers):
                post = [scs[h][i + 1][0] if i + 1 < len(layers) else None for h in range(2)]
                if L.is_torgb:
                    for h in range(2):
                        with torch.cuda.stream(st[h]):
                            xs[h] = L.run_nhwc(xs[h], 16, sdt, scs[h][i][1], None, final_scale=S.output_scale)
                    continue
                ys = [None, None]
                for h in range(2):
                    with torch.cuda.stream(st[h]):
                        if h == 0 and prev_b is not None:
                            st[0].wait_event(prev_b)
                        if h == 1:
                            st[1].wait_event(ea)
                        ys[h] = L.conv_nhwc(xs[h], 16, sdt, scs[h][i][1])
                        e = torch.cuda.Event()
                        e.record(st[h])
                        if h == 0:
                            ea = e
                        else:
                            prev_b = e
                        xs[h] = L.flrelu_nhwc(ys[h][0], sdt, post[h], blocked=ys[h][1])
            r = [None, None]
            for h in range(2):
                with torch.cuda.stream(st[h]):
                    r[h] = icm.uint8_sse(xs[h], x[16 * h:16 * h + 16])
            main_s.wait_stream(s1)
            main_s.wait_stream(s2)
            return r

    steps = {"one": step_one, "two": lambda: step_two(False), "offset": lambda: step_two(True), "synth2": step_synth2}
    for mode in args.modes.split(","):
        f = steps[mode]
        for _ in range(args.warmup):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        print(f"[overlap] {args.precision} {mode:7s} {dt * 1e3:8.3f} ms/step  {32 / dt:8.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
