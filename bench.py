"""Benchmark of the encode -> 8-bit quantize -> synthesize path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5] [--batch B] [--precision bf16|fp32]
                    [--no-roofline] [--cpu-baseline-images M] [--dry-run]

A step = one pass of the hot path over one synthetic batch already resident in HBM:
HVAE_VGG_Encoder(img_resolution=1024) on 256^2 images -> 8-bit uniform quantizer (deterministic, means)
-> StyleGAN3-T synthesis -> uint8 PSNR sums vs the input -> all_reduce(SUM) of the fp64 metric record.
Random-init weights of the named architectures (no checkpoints offline), seeded synthetic inputs
(seed 1000 + rank).

--config c5 (BASELINE config 5, the reference's train_hvae_encoder step, stylegan3_hvae_full.py:655-707): a step
is one optimisation step of the encoder through the frozen synthesis network (forward, the reference's second
encoder pass for the KL term, backward, data-parallel gradient all_reduce over RCCL, Adam); LPIPS excluded
(its pretrained VGG weights are not available offline).

Multi-GPU: one process per GPU, batch-sharded, weak scaling (every rank runs its own batch).  Under torchrun
the ranks come from the env; `python bench.py --gpus N` without torchrun spawns the N ranks itself
(distributed.launch: the parent never touches the GPU).  `--dry-run` runs the same launcher, rank seeding,
barrier / max-over-ranks timing and reductions on the CPU over gloo with a stand-in step (tests).

Timing protocol: W untimed warm-up steps, then EXACTLY K steps bracketed by a barrier +
synchronize on both sides; value = images of all ranks / the max over ranks of that wall time.  Each timed
step is also bracketed by HIP events on the launching stream (torch's current stream, which every libic2ops
kernel is enqueued on): ms_per_step_median.  The per-kernel roofline timers run in a SEPARATE instrumented
pass after the headline loop, so the headline number carries no instrumentation.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from image_compression_2_amd import distributed as icd  # noqa: E402  (no GPU access at import)

CONFIGS = {
    # name: (input res, generator res, per-GPU batch, description)
    "c2": (256, 256, 32, "batch=32 256x256 encode+8bit quantize+decode, SG3-T-256 generator"),
    "c4": (1024, 1024, 8, "batch=8 1024x1024 encode+8bit quantize+decode, SG3-T-1024 generator"),
    # reading (ii) of the 256^2 configs: the reference's default 1024 generator, its output bilinearly
    # decimated to the 256^2 input (StyleGAN3Compressor.forward, stylegan3_hvae_full.py:277-279)
    "c2r": (256, 1024, 32, "batch=32 256x256 encode+8bit quantize+decode on SG3-T-1024, bilinear decimation to 256"),
    "c5": (256, 256, 16, "HVAE encoder training step (rec MSE + 0.01 KL, Adam 1e-4) through frozen SG3-T-256, "
                         "256x256, per-GPU batch 16, grad all_reduce"),
}
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA, MI355X_MICROARCH.md
F32_PEAK_TFLOPS = 157.3     # f32 MFMA / VALU
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline-images", type=int, default=3, help="0 disables the CPU baseline leg")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU / gloo rehearsal of launcher + timing + reductions")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file (rank 0)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------
# instrumentation (separate pass)
class CallTimer:
    """Brackets every libic2ops call whose name is in `names` with HIP events on the launching stream
    (torch's current stream: every libic2ops kernel is enqueued there)."""

    def __init__(self, nv, names):
        self.nv = nv
        self.names = set(names)
        self.events = {n: [] for n in names}
        self.enabled = False
        self._orig = None

    def install(self):
        timer, orig = self, self.nv.call
        self._orig = orig

        def call(name, *args):
            if not timer.enabled or name not in timer.names:
                return orig(name, *args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rc = orig(name, *args)
            e.record()
            timer.events[name].append((s, e))
            return rc

        self.nv.call = call

    def uninstall(self):
        if self._orig is not None:
            self.nv.call = self._orig

    def total(self, names):
        torch.cuda.synchronize()
        ev = [p for n in names for p in self.events[n]]
        return sum(s.elapsed_time(e) for s, e in ev), len(ev)


def algorithmic_flops_per_image(enc, G, res, split=False):
    """MFMA-eligible FLOPs per image (unpadded): encoder convs + synthesis input 1x1 + modconvs
    (split=True -> (encoder, synthesis))."""
    total = 0.0
    h = res
    total += 2 * h * h * enc.from_rgb.out_channels * 9 * enc.from_rgb.in_channels
    for blk in enc.blocks:
        if h <= 1:
            break
        ci, co = blk.conv1.in_channels, blk.conv1.out_channels
        total += 2 * h * h * co * 9 * ci + 2 * h * h * co * 9 * co
        h = h // 2 if h > 1 else h
    enc_total = total
    S = int(G.synthesis.input.size[0])
    C = G.synthesis.input.channels
    total += 2 * S * S * C * C
    for L in G.synthesis.layers():
        s = int(L.in_size[0]) + L.conv_kernel - 1
        total += 2 * s * s * L.out_channels * L.conv_kernel ** 2 * L.in_channels
    return (enc_total, total - enc_total) if split else total


def training_flops_per_image(enc, G, res):
    """Conv FLOPs of one c5 step per image: encoder forward twice (the reference's second pass for the KL
    term), its dgrad (all but from_rgb, whose input needs no gradient) and wgrad; synthesis 1x1 input mix in
    torch, its modulated convs forward + dgrad."""
    e, s = algorithmic_flops_per_image(enc, G, res, split=True)
    rgb = 2 * res * res * enc.from_rgb.out_channels * 9 * enc.from_rgb.in_channels
    S, C = int(G.synthesis.input.size[0]), G.synthesis.input.channels
    s_mod = s - 2 * S * S * C * C
    return 2 * e + (e - rgb) + e + 2 * s_mod


def algorithmic_bytes_per_image(enc, G, res, esz):
    """Compulsory HBM bytes of the conv launches per image: each conv reads its input activation and writes
    its output once (padded channel strides, esz bytes each; ToRGB writes 3 f32 channels).  Weights are per
    launch, not per image, and are added by the caller."""
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
    """Packed weight bytes of the convs one step runs, and their count (= conv calls per step)."""
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


def flr_work_per_image(G):
    """Filtered-lrelu algorithmic work per image: polyphase separable FIR FLOPs
    (vertical up: U1 x S_conv outputs x taps_u/up, horizontal up: U1 x U1 x taps_u/up, horizontal down:
    U1 x S_out x taps_d, vertical down: S_out^2 x taps_d; 2 FLOP per tap) x channels, and the fused kernel's
    compulsory bytes (conv output in, 2 B, + layer output, 2 B, unpadded channels).  -> (flops, bytes, bound_s)
    with bound_s = sum over layers of max(FIR / 157.3 TF, bytes / 8 TB/s)."""
    flops = byts = bound = 0.0
    for L in G.synthesis.layers():
        if L.is_torgb:
            continue
        c = L.out_channels
        s_conv = int(L.in_size[0]) + L.conv_kernel - 1
        s_out = int(L.out_size[0])
        up, tu, td = L.up_factor, L.up_taps, L.down_taps
        u1 = (s_out - 1) * L.down_factor + td  # lrelu-grid side that feeds the outputs
        f = 2 * c * (u1 * s_conv * tu / up + u1 * u1 * tu / up + u1 * s_out * td + s_out * s_out * td)
        b = c * (s_conv * s_conv + s_out * s_out) * 2
        flops += f
        byts += b
        bound += max(f / (F32_PEAK_TFLOPS * 1e12), b / (HBM_PEAK_GBS * 1e9))
    return flops, byts, bound


def pmc_traffic(config, precision, batch):
    """roofline.traffic: HBM bytes per conv launch from the newest committed PMC run for this exact workload
    (tools/pmc_traffic.sh; FETCH_SIZE x2 + WRITE_SIZE, KiB -> bytes), or None when there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_traffic_{config}_{precision}_b{batch}.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    return rec["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(res, gen_res, n_images):
    """The oracle (pure-PyTorch fp32 CPU restatement) timed on the host cores: encode + quantize + decode of
    n_images, the fine fc1 drawn exactly as the reference re-creates it (nn.Linear(128, 256) default init,
    stylegan3_hvae_full.py:225-230)."""
    from oracle import encoder as oe
    from oracle import sg3
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd_e = {k: v.detach() for k, v in enc.state_dict().items()}
    sd_g = sg3.init_params(gen_res, seed=1)
    x = torch.rand(n_images, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    torch.manual_seed(5)
    lin = torch.nn.Linear(128, 256)
    fc1 = (lin.weight.detach(), lin.bias.detach())
    t0 = time.perf_counter()
    with torch.no_grad():
        _, m, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
        q = oe.quantize_uniform(m, 8)
        img = sg3.synthesis_forward(sd_g, gen_res, q)
        if img.shape[2] != res:
            torch.nn.functional.interpolate(img, size=(res, res), mode="bilinear", align_corners=False)
    dt = time.perf_counter() - t0
    return dict(value=round(n_images / dt, 4), unit="images/s", cores=torch.get_num_threads(), kind="port",
                cpu_model=cpu_model(),
                sample=f"{n_images} image(s) {res}x{res}, encoder(1024-config) + 8-bit quantize + SG3-T-{gen_res} "
                       f"{'(+ bilinear decimation) ' if gen_res != res else ''}"
                       f"synthesis, fp32, oracle/ restatement on {torch.get_num_threads()} threads, {dt:.1f} s; "
                       f"B=1 / B=32 / 1024^2 rows: profiles/r2_cpu_baseline.json")


def cpu_baseline_train(res, gen_res, n_images):
    """The oracle's fp32 CPU restatement of one c5 training step on n_images: encoder forward (x2, as the
    reference), synthesis forward, rec MSE + 0.01 KL, backward into the encoder's parameters."""
    from oracle import encoder as oe
    from oracle import sg3
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd_e = {k: v.detach().clone().requires_grad_(True) for k, v in enc.state_dict().items()}
    sd_g = sg3.init_params(gen_res, seed=1)
    x = torch.rand(n_images, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    torch.manual_seed(5)
    lin = torch.nn.Linear(128, 256)
    fc1 = (lin.weight.detach(), lin.bias.detach())
    w_avg = torch.zeros(1, 1, 512)
    t0 = time.perf_counter()
    w, _, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
    img = sg3.synthesis_forward(sd_g, gen_res, w)
    _, m, lv = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
    kl = 0.5 * torch.mean(torch.sum((m - w_avg) ** 2 + lv.exp() - lv - 1, dim=[1, 2]))
    loss = torch.nn.functional.mse_loss(x, img) + 0.01 * kl
    loss.backward()
    dt = time.perf_counter() - t0
    return dict(value=round(n_images / dt, 4), unit="images/s", cores=torch.get_num_threads(), kind="port",
                cpu_model=cpu_model(),
                sample=f"{n_images} image(s) {res}x{res}: encoder(1024-config) fwd x2 + SG3-T-{gen_res} synthesis fwd "
                       f"+ MSE/KL + backward, fp32 autograd over the oracle/ restatement on {torch.get_num_threads()} "
                       f"threads, {dt:.1f} s")


# ------------------------------------------------------------------------------------------------
def timed_loop(step, steps, sync, barrier, use_events):
    """Barrier + sync, EXACTLY `steps` steps, sync + barrier + sync.  -> (last output, wall s, per-step ms)."""
    sync()
    barrier()
    sync()
    marks = []
    out = None
    t0 = time.perf_counter()
    for _ in range(steps):
        if use_events:
            s = torch.cuda.Event(enable_timing=True)
            s.record()
            out = step()
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append((s, e))
        else:
            ts = time.perf_counter()
            out = step()
            marks.append(time.perf_counter() - ts)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    per = [s.elapsed_time(e) for s, e in marks] if use_events else [m * 1e3 for m in marks]
    return out, elapsed, per


def run(args):
    dry = args.dry_run
    rank, world, local = icd.init("gloo" if dry else None)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    res, gen_res, batch, desc = CONFIGS[args.config]
    batch = args.batch or batch
    if dry:
        dev = torch.device("cpu")
        sync = lambda: None
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    barrier = lambda: icd.barrier(dev)

    if dry:
        # stand-in step: the same seeded per-rank batch, a metric record and its all_reduce
        g = torch.Generator().manual_seed(1000 + rank)
        x = torch.rand(batch, 3, 16, 16, generator=g) * 2 - 1
        from oracle import metrics as om

        def step():
            sse = float(om.sse_uint8(x, x.flip(0)).sum())
            vec = torch.tensor([sse, float(x.numel()), float(batch)], dtype=torch.float64)
            return icd.allreduce_sum(vec)
        enc = G = comp = nv = None
    else:
        import image_compression_2_amd as ic2
        from image_compression_2_amd import _native as nv
        from image_compression_2_amd import metrics as icm
        train = args.config == "c5"
        torch.manual_seed(0)
        enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=args.precision).to(dev)
        if not train:
            enc.eval().requires_grad_(False)
        torch.manual_seed(1)
        G = ic2.Generator(img_resolution=gen_res, precision=args.precision).to(dev).eval()
        comp = ic2.StyleGAN3Compressor(enc, G, training_resolution=res if train else None)
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        x = torch.rand(batch, 3, res, res, generator=g, device=dev) * 2 - 1
        # (pixel count, image count) of the metric record: device constants made once, so the step has no
        # host->device copy (a pageable one stalls the host until the stream drains)
        counts = torch.tensor([float(x.numel()), float(batch)], dtype=torch.float64, device=dev)

        if train:
            from image_compression_2_amd import training as ict
            opt = ict.make_optimizer(enc, lr=1e-4)
            w_avg = G.mapping.w_avg.view(1, 1, -1)

            def train_step():
                losses = ict.train_step(comp, x, opt, w_avg, rec_weight=1.0, perceptual_weight=0.0, kl_weight=0.01)
                vec = torch.cat([(losses["rec_loss"].double() * batch).view(1),
                                 (losses["kl_loss"].double() * batch).view(1), counts[1:]])
                return icd.allreduce_sum(vec, device=dev)

        def step():
            with torch.no_grad():
                q = comp.compress(x, quantization_bits=8, deterministic=True)
                img = comp.decompress(q)
                if img.shape[2] != res:
                    img = ic2.resize_bilinear(img, (res, res))
                sse = icm.uint8_sse(img, x)
            vec = torch.cat([sse.sum().view(1), counts])
            return icd.allreduce_sum(vec, device=dev)

    if not dry and args.config == "c5":
        step = train_step
    for _ in range(args.warmup):
        step()
    vec, elapsed, per_step = timed_loop(step, args.steps, sync, barrier, use_events=not dry)
    elapsed_max = icd.allreduce_max(elapsed, device=dev)
    per_rank_ms = [round(t / args.steps * 1e3, 3) for t in icd.allgather_floats(elapsed, device=dev)]
    median_ms = statistics.median(per_step)
    median_max = icd.allreduce_max(median_ms, device=dev)
    checksum = icd.allgather_floats(float(x.double().sum()), device=dev)

    total_images = batch * args.steps * world
    value = total_images / elapsed_max
    vec = vec.cpu()
    metric = {"c2": "images/sec encode+decode 256px", "c4": "images/sec encode+decode 1024px",
              "c2r": "images/sec encode+decode 256px (1024 generator, decimated)",
              "c5": "images/sec encoder training step 256px"}[args.config]
    out = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded uniform [-1,1] images resident in HBM, seed 1000+rank; random-init encoder + "
                "SG3-T weights)",
        "config": {"workload": desc, "global_batch": batch * world, "per_gpu_batch": batch, "resolution": res,
                   "generator": f"stylegan3-t-{gen_res} (random init)", "encoder": "HVAE_VGG_Encoder(img_resolution=1024)",
                   "quantization_bits": 8, "parallelism": f"dp{world} (batch-sharded, RCCL metric all_reduce)"},
        "world_size": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
        "ms_per_step_median": round(median_max, 3),
        "per_rank_ms_per_step": per_rank_ms,
        "rank_input_checksums": [round(c, 6) for c in checksum],
    }
    if dry:
        out["dry_run"] = True
        out["psnr_db_record"] = float(10 * torch.log10(255.0 ** 2 / (vec[0] / vec[1])))
    elif args.config == "c5":
        out["config"].update(quantization_bits=None, loss="rec MSE + 0.01 KL(w_avg); LPIPS excluded (no weights "
                             "offline)", optimizer="Adam(1e-4, (0.9, 0.999))",
                             parallelism=f"dp{world} (batch-sharded, RCCL gradient all_reduce)")
        out["last_step_losses"] = {"rec_loss": round(vec[0].item() / vec[2].item(), 6),
                                   "kl_loss": round(vec[1].item() / vec[2].item(), 4)}
    else:
        from image_compression_2_amd import metrics as icm
        out["psnr_db_vs_input"] = round(icm.psnr_from_sums(vec[0].item(), vec[1].item()), 4)

    if not dry and not args.no_roofline and args.config == "c5":
        names = ("ic2_conv_igemm", "ic2_conv_igemm_ws", "ic2_conv_wgrad")
        timer = CallTimer(nv, names)
        timer.install()
        timer.enabled = True
        n_inst = min(args.steps, 5)
        timed_loop(step, n_inst, sync, barrier, use_events=True)
        timer.enabled = False
        timer.uninstall()
        conv_ms, n_launch = timer.total(names)
        flops_img = training_flops_per_image(enc, G, res)
        peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
        achieved = flops_img * batch * n_inst / (conv_ms * 1e-3) / 1e12
        out["roofline"] = {"bound": "mfma", "kernel": "ic2 conv family forward + dgrad (implicit GEMM) + wgrad",
                           "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                           "frac": round(achieved / peak, 4), "traffic": None, "launches": n_launch,
                           "avg_launch_ms": round(conv_ms / max(n_launch, 1), 4),
                           "conv_ms_per_step": round(conv_ms / n_inst, 3),
                           "path_frac": round(value / world * flops_img / (peak * 1e12), 4),
                           "algorithmic_gflop_per_image": round(flops_img / 1e9, 2)}
    elif not dry and not args.no_roofline:
        conv_names = ("ic2_conv_igemm", "ic2_conv_igemm_ws")
        timer = CallTimer(nv, conv_names + ("ic2_flrelu_nhwc", "ic2_flrelu_nhwc16"))
        timer.install()
        timer.enabled = True
        n_inst = min(args.steps, 10)
        timed_loop(step, n_inst, sync, barrier, use_events=True)
        timer.enabled = False
        timer.uninstall()
        conv_ms, n_launch = timer.total(conv_names)
        flr_ms, n_flr = timer.total(("ic2_flrelu_nhwc", "ic2_flrelu_nhwc16"))
        flops_img = algorithmic_flops_per_image(enc, G, res)
        peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
        traffic, traffic_src = pmc_traffic(args.config, args.precision, batch)
        esz = 2 if args.precision == "bf16" else 4
        wb, n_conv = weight_bytes(enc, G, res, esz)
        alg_bytes = (algorithmic_bytes_per_image(enc, G, res, esz) * batch + wb) / n_conv
        achieved = flops_img * batch * n_inst / (conv_ms * 1e-3) / 1e12
        out["roofline"] = {"bound": "mfma", "kernel": "ic2 conv family (igemm / halo conv / ToRGB, every "
                                                      "encoder conv, synthesis input 1x1 and modulated conv)",
                           "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                           "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                           "traffic_src": traffic_src, "algorithmic_bytes_per_launch": round(alg_bytes),
                           "launches": n_launch, "avg_launch_ms": round(conv_ms / max(n_launch, 1), 4),
                           "conv_ms_per_step": round(conv_ms / n_inst, 3),
                           "path_frac": round(value / world * flops_img / (peak * 1e12), 4),
                           "algorithmic_gflop_per_image": round(flops_img / 1e9, 2)}
        if args.precision == "bf16" and n_flr:
            f_img, b_img, bound_img = flr_work_per_image(G)
            flr_step = flr_ms / n_inst
            bound_step = bound_img * batch * 1e3
            out["roofline"]["flr"] = {
                "kernel": "ic2 flrelu_mfma (fused filtered lrelu, every synthesis layer but ToRGB)",
                "bound": "valu (FIR on f32 VALU, SURVEY.md 8(d)); the kernel itself runs the FIR on f16 MFMA",
                "fir_gflop_per_image": round(f_img / 1e9, 3), "bytes_per_image": round(b_img),
                "ms_per_step": round(flr_step, 3), "bound_ms_per_step": round(bound_step, 3),
                "frac_of_bound": round(bound_step / flr_step, 4),
                "achieved_tflops": round(f_img * batch / (flr_step * 1e-3) / 1e12, 2),
                "achieved_gbs": round(b_img * batch / (flr_step * 1e-3) / 1e9, 1), "launches": n_flr}

    if rank == 0 and world == 1 and args.cpu_baseline_images > 0 and not dry and args.config == "c5":
        out["cpu_baseline"] = cpu_baseline_train(res, gen_res, 1)
    elif rank == 0 and world == 1 and args.cpu_baseline_images > 0 and not dry:
        if args.config == "c2r":
            out["cpu_baseline"] = cpu_baseline(res, gen_res, 1)
        else:
            out["cpu_baseline"] = cpu_baseline(res if args.config == "c2" else 256,
                                               gen_res if args.config == "c2" else 256, args.cpu_baseline_images)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        torch.distributed.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        icd.launch(args.gpus, run, args)   # self-launch: one spawned process per GPU
        return
    run(args)


if __name__ == "__main__":
    main()
