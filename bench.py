"""Benchmark of the encode -> 8-bit quantize -> synthesize path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4] [--batch B] [--precision bf16|fp32]

A step = one pass of the hot path over one synthetic batch already resident in HBM:
HVAE_VGG_Encoder(img_resolution=1024) on 256^2 images -> 8-bit uniform quantizer (deterministic, means)
-> StyleGAN3-T synthesis -> uint8 PSNR sums vs the input -> all_reduce(SUM) of the fp64 metric record.
Random-init weights of the named architectures (no checkpoints offline), seeded synthetic inputs.
For N > 1 (torchrun, one process per GPU, RCCL) every rank runs its own batch: weak scaling.
Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (input res, generator res, per-GPU batch, description)
    "c2": (256, 256, 32, "batch=32 256x256 encode+8bit quantize+decode, SG3-T-256 generator"),
    "c4": (1024, 1024, 8, "batch=8 1024x1024 encode+8bit quantize+decode, SG3-T-1024 generator"),
}
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA, MI355X_MICROARCH.md
F32_PEAK_TFLOPS = 157.3     # f32 MFMA / VALU
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline-images", type=int, default=3, help="0 disables the CPU baseline leg")
    ap.add_argument("--no-roofline", action="store_true")
    return ap.parse_args()


class IgemmTimer:
    """Wraps every ic2_conv_igemm[_ws] call (the dominant kernel, plus its split-K combine where the launch
    plan splits K: all encoder convs, the synthesis input 1x1 and every modulated conv) with HIP events on
    the launching stream -- torch's current stream, which is the stream every libic2ops kernel is enqueued on."""

    def __init__(self, nv):
        self.nv = nv
        self.orig = nv.call
        self.events = []
        self.enabled = False

    def install(self):
        timer = self

        def call(name, *args):
            if not timer.enabled or name not in ("ic2_conv_igemm", "ic2_conv_igemm_ws"):
                return timer.orig(name, *args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rc = timer.orig(name, *args)
            e.record()
            timer.events.append((s, e))
            return rc

        self.nv.call = call

    def result(self):
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in self.events), len(self.events)


def algorithmic_flops_per_image(enc, G, res):
    """MFMA-eligible FLOPs per image (unpadded): encoder convs + synthesis input 1x1 + modconvs."""
    total = 0.0
    h = res
    total += 2 * h * h * enc.from_rgb.out_channels * 9 * enc.from_rgb.in_channels
    for blk in enc.blocks:
        if h <= 1:
            break
        ci, co = blk.conv1.in_channels, blk.conv1.out_channels
        total += 2 * h * h * co * 9 * ci + 2 * h * h * co * 9 * co
        h = h // 2 if h > 1 else h
    S = int(G.synthesis.input.size[0])
    C = G.synthesis.input.channels
    total += 2 * S * S * C * C
    for L in G.synthesis.layers():
        s = int(L.in_size[0]) + L.conv_kernel - 1
        total += 2 * s * s * L.out_channels * L.conv_kernel ** 2 * L.in_channels
    return total


def algorithmic_bytes_per_image(enc, G, res, esz):
    """Compulsory HBM bytes of the igemm launches per image: each conv reads its input activation and
    writes its output once (padded channel strides, esz bytes each; ToRGB writes 3 f32 channels).
    Weights are per launch, not per image, and are added by the caller."""
    p32 = lambda c: (int(c) + 31) // 32 * 32
    total, h = 0.0, res
    total += h * h * (p32(enc.from_rgb.in_channels) + p32(enc.from_rgb.out_channels)) * esz
    for blk in enc.blocks:
        if h <= 1:
            break
        ci, co = p32(blk.conv1.in_channels), p32(blk.conv1.out_channels)
        total += h * h * (ci + co) * esz + h * h * (co + co) * esz
        h = h // 2
    S, C = int(G.synthesis.input.size[0]), p32(G.synthesis.input.channels)
    total += 2 * S * S * C * esz
    for L in G.synthesis.layers():
        s_in = int(L.in_size[0])
        s = s_in + L.conv_kernel - 1
        out = s * s * 3 * 4 if L.is_torgb else s * s * p32(L.out_channels) * esz
        total += s_in * s_in * p32(L.in_channels) * esz + out
    return total


def weight_bytes(enc, G, res, esz):
    """Packed weight bytes of the convs one step runs, and their count (= igemm calls per step)."""
    p32 = lambda c: (int(c) + 31) // 32 * 32
    convs, h = [enc.from_rgb], res
    for blk in enc.blocks:
        if h <= 1:
            break
        convs += [blk.conv1, blk.conv2]
        h = h // 2
    tot = sum(p32(c.out_channels) * p32(c.in_channels) * c.kernel_size[0] * c.kernel_size[1] * esz for c in convs)
    C = p32(G.synthesis.input.channels)
    tot += C * C * esz
    tot += sum(p32(L.out_channels) * p32(L.in_channels) * L.conv_kernel ** 2 * esz for L in G.synthesis.layers())
    return tot, len(convs) + 1 + len(list(G.synthesis.layers()))


def pmc_traffic(config, precision, batch):
    """roofline.traffic: HBM bytes per igemm launch from the committed PMC run for this exact workload
    (tools/pmc_traffic.sh; FETCH_SIZE x2 + WRITE_SIZE, KiB -> bytes), or None when there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_traffic_{config}_{precision}_b{batch}.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    return rec["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def cpu_baseline(res, gen_res, n_images):
    """The oracle (pure-PyTorch fp32 CPU restatement) timed on the host cores: encode + quantize + decode."""
    from oracle import encoder as oe
    from oracle import sg3
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd_e = {k: v.detach() for k, v in enc.state_dict().items()}
    sd_g = sg3.init_params(gen_res, seed=1)
    x = torch.rand(n_images, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    fc1 = (torch.randn(256, 128) * 0.05, torch.zeros(256))
    t0 = time.perf_counter()
    with torch.no_grad():
        _, m, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
        q = oe.quantize_uniform(m, 8)
        sg3.synthesis_forward(sd_g, gen_res, q)
    dt = time.perf_counter() - t0
    return dict(value=round(n_images / dt, 4), unit="images/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{n_images} image(s) {res}x{res}, encoder(1024-config) + 8-bit quantize + SG3-T-{gen_res} "
                       f"synthesis, fp32, oracle/ restatement, {dt:.1f} s")


def main():
    args = parse()
    from image_compression_2_amd import distributed as icd
    rank, world, local = icd.init()
    assert world == args.gpus or (world == 1 and args.gpus == 1), \
        f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torchrun)"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    from image_compression_2_amd import metrics as icm

    res, gen_res, batch, desc = CONFIGS[args.config]
    batch = args.batch or batch
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=args.precision).to(dev).eval()
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=gen_res, precision=args.precision).to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.rand(batch, 3, res, res, generator=g, device=dev) * 2 - 1

    timer = IgemmTimer(nv)
    timer.install()

    def step():
        with torch.no_grad():
            q = comp.compress(x, quantization_bits=8, deterministic=True)
            img = comp.decompress(q)
            sse = icm.uint8_sse(img, x)
        vec = torch.stack([sse.sum(), torch.tensor(float(img.numel()), device=dev, dtype=torch.float64),
                           torch.tensor(float(batch), device=dev, dtype=torch.float64)])
        return icd.allreduce_sum(vec, device=dev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    icd.barrier(dev)
    torch.cuda.synchronize()
    timer.enabled = not args.no_roofline
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vec = step()
    torch.cuda.synchronize()
    icd.barrier(dev)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    elapsed = icd.allreduce_max(elapsed, device=dev)
    igemm_ms, n_launch = timer.result()

    total_images = batch * args.steps * world
    value = total_images / elapsed
    vec = vec.cpu()
    psnr = icm.psnr_from_sums(vec[0].item(), vec[1].item())
    flops_img = algorithmic_flops_per_image(enc, G, res)
    peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
    out = {
        "metric": "images/sec encode+decode 256px" if args.config == "c2" else "images/sec encode+decode 1024px",
        "value": round(value, 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded uniform [-1,1] images resident in HBM; random-init encoder + SG3-T weights)",
        "config": {"workload": desc, "global_batch": batch * world, "per_gpu_batch": batch, "resolution": res,
                   "generator": f"stylegan3-t-{gen_res} (random init)", "encoder": "HVAE_VGG_Encoder(img_resolution=1024)",
                   "quantization_bits": 8, "parallelism": f"dp{world} (batch-sharded, RCCL metric all_reduce)"},
        "psnr_db_vs_input": round(psnr, 4),
    }
    if not args.no_roofline and igemm_ms > 0:
        per_launch_ms = igemm_ms / n_launch
        traffic, traffic_src = pmc_traffic(args.config, args.precision, batch)
        esz = 2 if args.precision == "bf16" else 4
        wb, n_conv = weight_bytes(enc, G, res, esz)
        alg_bytes = (algorithmic_bytes_per_image(enc, G, res, esz) * batch + wb) / n_conv
        achieved = flops_img * batch * args.steps / (igemm_ms * 1e-3) / 1e12
        out["roofline"] = {"bound": "mfma", "kernel": "ic2 igemm_kernel (all conv/modconv launches)",
                           "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                           "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                           "traffic_src": traffic_src, "algorithmic_bytes_per_launch": round(alg_bytes),
                           "launches": n_launch, "avg_launch_ms": round(per_launch_ms, 4),
                           "path_frac": round(value / world * flops_img / (peak * 1e12), 4),
                           "algorithmic_gflop_per_image": round(flops_img / 1e9, 2)}
    if rank == 0 and world == 1 and args.cpu_baseline_images > 0:
        out["cpu_baseline"] = cpu_baseline(res if args.config == "c2" else 256, gen_res if args.config == "c2" else 256,
                                           args.cpu_baseline_images)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
