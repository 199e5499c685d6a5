"""Benchmark of the encode -> 8-bit quantize -> synthesize path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2g|c2r|c4|c5] [--batch B]
                    [--precision f16|bf16|bf16-all|fp32] [--no-roofline] [--no-parity] [--cpu-baseline-images M]
                    [--dry-run]

A step = one pass of the hot path over one synthetic batch already resident in HBM:
HVAE_VGG_Encoder(img_resolution=1024) on 256^2 images -> 8-bit uniform quantizer (deterministic, means)
-> StyleGAN3-T synthesis -> uint8 PSNR sums vs the input + the code record (8-bit code histogram, index
mismatches against the first step's codes) -> all_reduce(SUM) of the fp64 metric record.
Random-init weights of the named architectures (no checkpoints offline), seeded synthetic inputs (seed 1000 + rank,
drawn on the host generator and copied to HBM once before the timed region).

--precision (encoder, synthesis): f16 (default, round 4) = split-bf16 encoder ('bf16x3': three bf16 MFMA terms per
product, f32 between layers -- the 8-bit indices of the fp32 reference) + f16 synthesis (bf16's MFMA rate, 11-bit
significands: the north-star PSNR bar met at the 34 dB and the 46 dB operating points, pixels within ~1e-3 of fp32,
tests/test_gpu_c2_parity.py); bf16 = split-bf16 encoder + bf16 synthesis (meets the PSNR bar at 34 dB, not at 46 dB);
bf16-all = bf16 encoder + bf16 synthesis (round 2's mode: 4.6 % of the 8-bit indices differ from the reference's);
fp32 = the exact-fp32 parity mode.

Parity in the line (rank 0, outside the timed region; --no-parity skips it): 'parity' holds the benched encoder's
8-bit indices against the committed fp32 oracle means of the same input images (tests/golden/parity_means.npz,
made by tests/golden/make_parity_means.py) and the north-star PSNR deltas of the benched images at the 34 dB and
46 dB operating points, against the fp32 HIP path on the same latents and against the reconstruction of the
oracle's codes (hvae_training.py:368-395 PSNR, README.md:381 operating point).

--config c2g: the codebook path, GumbelSoftmaxCompressor.compress -> decompress (gumbel_softmax_compression.py:
213-264) with the codes kept on the device (the reference's API moves them to the host; that PCIe round trip is
not in the timed value).  --config c5 (BASELINE config 5, the reference's train_hvae_encoder step,
stylegan3_hvae_full.py:655-707): one optimisation step of the encoder through the frozen synthesis network
(forward, the reference's second encoder pass for the KL term, backward, data-parallel gradient all_reduce over
RCCL, Adam); LPIPS excluded (its pretrained VGG weights are not available offline).  The two encoder calls on the
batch share one trunk and run the projector heads twice (training.train_step shared_trunk: the reference's values
and RNG draws, one trunk backward for both heads' gradients).

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
import collections
import json
import math
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
    "c2g": (256, 256, 32, "batch=32 256x256 encode+8bit codebook quantize (GumbelSoftmaxCompressor.compress -> "
                          "decompress, 256-entry codebook)+decode, SG3-T-256 generator"),
    "c4": (1024, 1024, 8, "batch=8 1024x1024 encode+8bit quantize+decode, SG3-T-1024 generator"),
    # reading (ii) of the 256^2 configs: the reference's default 1024 generator, its output bilinearly
    # decimated to the 256^2 input (StyleGAN3Compressor.forward, stylegan3_hvae_full.py:277-279)
    "c2r": (256, 1024, 32, "batch=32 256x256 encode+8bit quantize+decode on SG3-T-1024, bilinear decimation to 256"),
    "c5": (256, 256, 16, "HVAE encoder training step (rec MSE + 0.01 KL, Adam 1e-4) through frozen SG3-T-256, "
                         "256x256, per-GPU batch 16, grad all_reduce"),
}
# --precision -> (encoder precision, synthesis precision)
DEFAULT_PRECISION = "f16"
PRECISIONS = {
    "bf16": ("bf16x3", "bf16"),
    "bf16-all": ("bf16", "bf16"),
    "f16": ("bf16x3", "f16"),
    "fp32": ("fp32", "fp32"),
}
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA, MI355X_MICROARCH.md
F32_PEAK_TFLOPS = 157.3     # f32 MFMA / VALU
HBM_PEAK_GBS = 8000.0
N_CODES = 256               # 8-bit codes: the record's histogram width

CONV_ENTRIES = ("ic2_conv_igemm_ws", "ic2_conv3x3_gn_fwd", "ic2_conv3x3_gn_fwd_scaled", "ic2_conv3x3_gnin_gn_fwd",
                "ic2_from_rgb_conv", "ic2_from_rgb_conv_x3", "ic2_from_rgb_conv_f16", "ic2_conv_wino")
TRAIN_CONV_ENTRIES = CONV_ENTRIES + ("ic2_conv_wgrad", "ic2_conv_wgrad_oihw")
FLR_ENTRIES = ("ic2_flrelu_nhwc", "ic2_flrelu_nhwc16")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--precision", default=DEFAULT_PRECISION, choices=sorted(PRECISIONS))
    ap.add_argument("--cpu-baseline-images", type=int, default=3, help="0 disables the CPU baseline leg")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the parity record (rank 0, untimed)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the untimed secondary C4 entry of the default c2 line (rank 0, N=1)")
    ap.add_argument("--dry-run", action="store_true", help="CPU / gloo rehearsal of launcher + timing + reductions")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file (rank 0)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------
# instrumentation (separate pass)
class CallTimer:
    """Brackets every libic2ops call whose name is in `names` with HIP events on the launching stream (torch's
    current stream: every libic2ops kernel is enqueued there).  Conv calls also carry the algorithmic FLOPs the
    product code announced for them (_native.note_flops) and their arguments (-> the kernel the launch plan ran)."""

    def __init__(self, nv, names):
        self.nv = nv
        self.names = set(names)
        self.records = []      # (name, args, algorithmic flops | None, start event, end event)
        self.enabled = False
        self.pending = None
        self._orig = None

    def install(self):
        timer, orig = self, self.nv.call
        self._orig = orig

        def call(name, *args):
            f = None
            if name in CONV_ENTRIES or name in ("ic2_conv_wgrad", "ic2_conv_wgrad_oihw"):
                f, timer.pending = timer.pending, None
            if not timer.enabled or name not in timer.names:
                return orig(name, *args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rc = orig(name, *args)
            e.record()
            timer.records.append((name, args, f, s, e))
            return rc

        def hook(f):
            timer.pending = f

        self.nv.call = call
        self.nv._flops_hook = hook

    def uninstall(self):
        if self._orig is not None:
            self.nv.call = self._orig
        self.nv._flops_hook = None

    def calls(self, names):
        """[(name, args, alg_flops, ms)] of the recorded calls named in `names`."""
        torch.cuda.synchronize()
        return [(n, a, f, s.elapsed_time(e)) for (n, a, f, s, e) in self.records if n in names]


def conv_call_plan(nv, name, args):
    """(kernel instance(s) the launch plan ran, MFMA FLOPs it executed incl. channel padding) of one conv call."""
    if name in ("ic2_from_rgb_conv", "ic2_from_rgb_conv_x3", "ic2_from_rgb_conv_f16"):
        cin, (n, h, w, cout_p) = args[1], args[6:10]
        return name[4:], 2 * n * h * w * cout_p * 9 * cin
    if name == "ic2_conv_igemm_ws":
        dt, odt, n, h, w, cin_p, cout_p, cv, kh, kw, pad = args[3:14]
        layout = args[23]
    elif name in ("ic2_conv3x3_gn_fwd", "ic2_conv3x3_gn_fwd_scaled"):
        dt, (n, h, w, cin_p, cout_p, cv, kh, kw, pad) = args[3], args[4:13]
        odt, layout = dt, nv.NHWC
        if dt == nv.BF16X3:  # split-bf16 encoder: bf16 GEMM over the tripled K, f32 out
            dt, odt = nv.BF16, nv.F32
        elif dt == nv.F16X2:  # its first blocks: f16 GEMM over the doubled K, f16 out
            odt = nv.F16
    elif name == "ic2_conv3x3_gnin_gn_fwd":
        dt, (n, h, w, cin_p, cout_p, cv, kh, kw, pad) = args[5], args[6:15]
        odt, layout = dt, nv.NHWC
    elif name == "ic2_conv_wgrad":
        dt, (n, h, w, cin_p, cout_p, kh, kw, pad) = args[3], args[4:12]
        return "conv_wgrad", 2 * n * h * w * cout_p * kh * kw * cin_p
    elif name == "ic2_conv_wgrad_oihw":   # the same GEMM, written in the parameter's layout
        dt, (n, h, w, cin_p, cout_p) = args[3], args[4:9]
        kh, kw, pad = args[11:14]
        return "conv_wgrad", 2 * n * h * w * cout_p * kh * kw * cin_p
    elif name == "ic2_conv_wino":
        # Winograd F(2,3) along x: 4 positions x 3 kernel rows = 12 MFMA products per output pair (the direct conv's
        # 18); executed = those products over the padded channels and every output pair
        n, h, w, cin_p, cout_p, cv, pad, ho, wo = args[5:14]
        return nv.wino_plan(n, h, w, cin_p, cout_p, pad), 2 * n * ho * ((wo + 1) // 2) * cout_p * 12 * cin_p
    else:
        raise KeyError(name)
    ho, wo = h + 2 * pad - kh + 1, w + 2 * pad - kw + 1
    plan = nv.conv_plan(dt, odt, layout, n, h, w, cin_p, cout_p, cv, kh, kw, pad)
    if (name in ("ic2_conv3x3_gn_fwd", "ic2_conv3x3_gn_fwd_scaled") and (odt == nv.F32 or dt == nv.F16X2)
            and plan.startswith("hg4_o")):
        # the split conv with the GroupNorm statistics in its epilogue (igemm.hip x3_gn_hg4: 12-row tiles for 64-wide)
        f16 = plan.endswith("_f16")
        base = plan[:-4] if f16 else plan
        plan = ("hg4_o64_w32_t12_gn" if base.startswith("hg4_o64") else base + "_gn") + ("_f16" if f16 else "")
    return plan, 2 * n * ho * wo * cout_p * kh * kw * cin_p


def algorithmic_flops_per_image(enc, G, res, split=False):
    """MFMA-eligible FLOPs per image (unpadded; the reference's convs): encoder convs + synthesis input 1x1 +
    modconvs (split=True -> (encoder, synthesis))."""
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


def _h2_blocks(enc_split):
    """Encoder blocks whose convs run split-weight f16 in the split mode (stylegan3_hvae_full._SPLIT_F16_BLOCKS)."""
    from image_compression_2_amd import stylegan3_hvae_full as shf
    return shf._SPLIT_F16_BLOCKS if enc_split else 0


def algorithmic_bytes_per_image(enc, G, res, esz, enc_split=False):
    """Compulsory HBM bytes of the conv launches per image: each conv reads its input activation and writes
    its output once (padded channel strides, esz bytes each; ToRGB writes 3 f32 channels).  enc_split: the
    split-bf16 encoder ('bf16x3') reads its conv operands as [hi | lo] bf16 (4 B per channel; the GEMM reads the hi
    block twice, the second time from cache) and writes f32 (4 B); its first blocks in split-weight f16 read and write
    f16 (2 B), and from_rgb writes f16 when block 0 is one of them, else the split form.  Weights are per launch, not
    per image, and are added by the caller."""
    p32 = lambda c: (int(c) + 31) // 32 * 32
    nh2 = _h2_blocks(enc_split)
    total, h = 0.0, res
    total += h * h * (enc.from_rgb.in_channels * 4 +
                      p32(enc.from_rgb.out_channels) * ((2 if nh2 > 0 else 4) if enc_split else esz))
    for i, blk in enumerate(enc.blocks):
        if h <= 1:
            break
        e_in, e_out = ((2, 2) if i < nh2 else (4, 4)) if enc_split else (esz, esz)
        ci, co = p32(blk.conv1.in_channels), p32(blk.conv1.out_channels)
        total += h * h * (ci * e_in + co * e_out) + h * h * (co * e_in + co * e_out)
        h = h // 2
    S, C = int(G.synthesis.input.size[0]), p32(G.synthesis.input.channels)
    total += 2 * S * S * C * esz
    for L in G.synthesis.layers():
        s_in = int(L.in_size[0])
        s = s_in + L.conv_kernel - 1
        out = s * s * 3 * 4 if L.is_torgb else s * s * p32(L.out_channels) * esz
        total += s_in * s_in * p32(L.in_channels) * esz + out
    return total


def weight_bytes(enc, G, res, esz, enc_split=False):
    """Packed weight bytes of the convs one step runs, and their count (= conv calls per step).  enc_split: the
    encoder's packed weights are [hi | lo | hi] (3 bf16 per value), [hi | lo] f16 (2 per value) in its split-weight
    f16 blocks."""
    p32 = lambda c: (int(c) + 31) // 32 * 32
    nh2 = _h2_blocks(enc_split)
    convs, h = [(enc.from_rgb, 6)], res
    for i, blk in enumerate(enc.blocks):
        if h <= 1:
            break
        ew = 4 if i < nh2 else 6
        convs += [(blk.conv1, ew), (blk.conv2, ew)]
        h = h // 2
    tot = sum(p32(c.out_channels) * p32(c.in_channels) * c.kernel_size[0] * c.kernel_size[1] * (ew if enc_split else esz)
              for c, ew in convs)
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


def plan_kernel_tags(plan):
    """Substrings of the kernel function names a launch-plan instance (ic2_conv_plan / ic2_conv_wino_plan names, as
    roofline.per_kernel lists them) dispatches -- to check a committed PMC record against the current plan."""
    p = plan[:-4] if plan.endswith("_f16") else plan
    if p.startswith("wino_fx"):
        return ["wino_fx"]
    if p.startswith("igemm8_og2+og1"):
        return ["igemm8_og2", "igemm8_og1"]
    if p.startswith("igemm8_"):
        return [p.replace("_splitk", "").replace("_tail", "")]
    if p.startswith("igemm_"):
        return ["igemm_kernel"]
    if p.startswith("hg4_"):
        return [p]
    if p.startswith("hconv"):
        return ["hconv_kernel"]
    if p == "torgb":
        return ["torgb_kernel"]
    if p.startswith("from_rgb"):
        return ["from_rgb_kernel"]
    return [p]


def pmc_traffic(config, precision, batch):
    """roofline.traffic: HBM bytes per conv launch from the newest committed PMC run for this exact workload
    (tools/pmc_traffic.sh; FETCH_SIZE x2 + WRITE_SIZE, KiB -> bytes), or None when there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_traffic_{config}_{precision}_b{batch}.json")))
    if not files:
        return None
    rec = json.load(open(files[-1]))
    rec["src"] = os.path.relpath(files[-1], ROOT)
    return rec


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on (the GPU box's CPU share), capped by
    OMP_NUM_THREADS when set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def _oracle_setup(res, gen_res, n_images):
    from oracle import sg3
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd_e = {k: v.detach() for k, v in enc.state_dict().items()}
    sd_g = sg3.init_params(gen_res, seed=1)
    x = torch.rand(n_images, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    torch.manual_seed(5)
    lin = torch.nn.Linear(128, 256)
    return sd_e, sd_g, x, (lin.weight.detach(), lin.bias.detach())


def cpu_baseline(res, gen_res, n_images, codebook=False):
    """The oracle (pure-PyTorch fp32 CPU restatement) timed on the host cores: encode + quantize + decode of
    n_images, the fine fc1 drawn exactly as the reference re-creates it (nn.Linear(128, 256) default init,
    stylegan3_hvae_full.py:225-230).  codebook: the reference's GumbelSoftmaxCompressor quantizer (its full
    discretization forward with Gumbel noise over [N*8192, 256], gumbel_softmax_compression.py:229) + lookup."""
    from oracle import encoder as oe
    from oracle import sg3
    nt = cpu_threads()
    torch.set_num_threads(nt)
    sd_e, sd_g, x, fc1 = _oracle_setup(res, gen_res, n_images)
    t0 = time.perf_counter()
    with torch.no_grad():
        _, m, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
        if codebook:
            noise = oe.gumbel_noise(7, m.numel())
            _, _, idx = oe.gumbel_forward(m, noise, 1.0, True)
            q = oe.codebook_lookup(idx.reshape(m.shape))
        else:
            q = oe.quantize_uniform(m, 8)
        img = sg3.synthesis_forward(sd_g, gen_res, q)
        if img.shape[2] != res:
            torch.nn.functional.interpolate(img, size=(res, res), mode="bilinear", align_corners=False)
    dt = time.perf_counter() - t0
    out = dict(value=round(n_images / dt, 4), unit="images/s", cores=nt, kind="port", cpu_model=cpu_model(),
               host_cpus=os.cpu_count(),
               sample=f"{n_images} image(s) {res}x{res}, encoder(1024-config) + 8-bit "
                      f"{'codebook (Gumbel forward + argmin + lookup)' if codebook else 'uniform'} quantize + "
                      f"SG3-T-{gen_res} {'(+ bilinear decimation) ' if gen_res != res else ''}synthesis, fp32, "
                      f"oracle/ restatement on {nt} threads, {dt:.1f} s")
    if codebook:
        # the quantizer alone at the reference's N=32 (2.19 s on 8 Xeon cores)
        z = torch.randn(32, 16, 512, generator=torch.Generator().manual_seed(3)) * 0.5
        t0 = time.perf_counter()
        oe.gumbel_forward(z, oe.gumbel_noise(8, z.numel()), 1.0, True)
        out["quantizer_only_n32_s"] = round(time.perf_counter() - t0, 3)
    return out


def cpu_baseline_train(res, gen_res, n_images):
    """The oracle's fp32 CPU restatement of one c5 training step on n_images: encoder forward (x2, as the
    reference), synthesis forward, rec MSE + 0.01 KL, backward into the encoder's parameters."""
    from oracle import encoder as oe
    from oracle import sg3
    nt = cpu_threads()
    torch.set_num_threads(nt)
    sd_e, sd_g, x, fc1 = _oracle_setup(res, gen_res, n_images)
    sd_e = {k: v.clone().requires_grad_(True) for k, v in sd_e.items()}
    w_avg = torch.zeros(1, 1, 512)
    t0 = time.perf_counter()
    w, _, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
    img = sg3.synthesis_forward(sd_g, gen_res, w)
    _, m, lv = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
    kl = 0.5 * torch.mean(torch.sum((m - w_avg) ** 2 + lv.exp() - lv - 1, dim=[1, 2]))
    loss = torch.nn.functional.mse_loss(x, img) + 0.01 * kl
    loss.backward()
    dt = time.perf_counter() - t0
    return dict(value=round(n_images / dt, 4), unit="images/s", cores=nt, kind="port", cpu_model=cpu_model(),
                host_cpus=os.cpu_count(),
                sample=f"{n_images} image(s) {res}x{res}: encoder(1024-config) fwd x2 + SG3-T-{gen_res} synthesis fwd "
                       f"+ MSE/KL + backward, fp32 autograd over the oracle/ restatement on {nt} threads, {dt:.1f} s")


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


def record_summary(vec, n_codes=N_CODES):
    """The all-reduced metric record [sse, pixels, images, index mismatches vs the first step, codes out of
    range, hist[n_codes]] -> reported fields (global over ranks)."""
    hist = vec[5:5 + n_codes].double()
    total = float(hist.sum()) + float(vec[4])
    p = hist / max(total, 1.0)
    perplexity = float(torch.exp(-torch.sum(p * torch.log(p + 1e-10))))
    return {"psnr_db_vs_input": None, "codes": int(round(total)), "index_mismatch_vs_first_step": int(vec[3]),
            "codes_out_of_range": int(vec[4]), "code_perplexity": round(perplexity, 3),
            "hist_nonzero_bins": int((hist > 0).sum())}


def run(args):
    dry = args.dry_run
    # rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, collectives over gloo (not a measurement)
    share = os.environ.get("IC2_BENCH_SHARE_GPU") == "1"
    rank, world, local = icd.init("gloo" if dry or share else None)
    if share:
        local = 0
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    res, gen_res, batch, desc = CONFIGS[args.config]
    batch = args.batch or batch
    enc_prec, syn_prec = PRECISIONS[args.precision]
    if dry:
        dev = torch.device("cpu")
        sync = lambda: None
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    barrier = lambda: icd.barrier(dev)

    if dry:
        # stand-in step: the same seeded per-rank batch, a metric record (SSE, counts, 8-bit code histogram of
        # the image itself) and its all_reduce
        g = torch.Generator().manual_seed(1000 + rank)
        x = torch.rand(batch, 3, 16, 16, generator=g) * 2 - 1
        from oracle import metrics as om
        from oracle import encoder as oe
        codes = oe.uniform_indices(x, 8).reshape(-1)

        def step():
            sse = float(om.sse_uint8(x, x.flip(0)).sum())
            hist = torch.bincount(codes.clamp(0, N_CODES - 1), minlength=N_CODES).double()
            vec = torch.cat([torch.tensor([sse, float(x.numel()), float(batch), 0.0, 0.0], dtype=torch.float64), hist])
            return icd.allreduce_sum(vec)
        enc = G = comp = nv = None
    else:
        import image_compression_2_amd as ic2
        from image_compression_2_amd import _native as nv
        from image_compression_2_amd import metrics as icm
        train = args.config == "c5"
        torch.manual_seed(0)
        enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=syn_prec if train else enc_prec).to(dev)
        if not train:
            enc.eval().requires_grad_(False)
        torch.manual_seed(1)
        G = ic2.Generator(img_resolution=gen_res, precision=syn_prec).to(dev).eval()
        if args.config == "c2g":
            comp = ic2.GumbelSoftmaxCompressor(enc, G).to(dev)
        else:
            comp = ic2.StyleGAN3Compressor(enc, G, training_resolution=res if train else None)
        # drawn on the host generator (the committed parity fixture and the CPU baseline use the same images) and
        # copied to HBM once, before anything is timed
        x_host = torch.rand(batch, 3, res, res, generator=torch.Generator().manual_seed(1000 + rank)) * 2 - 1
        x = x_host.to(dev)
        # (pixel count, image count) of the metric record: device constants made once, so the step has no
        # host->device copy (a pageable one stalls the host until the stream drains)
        counts = torch.tensor([float(x.numel()), float(batch)], dtype=torch.float64, device=dev)
        stream = nv.stream_of(x)
        golden = {}

        if train:
            from image_compression_2_amd import training as ict
            opt = ict.make_optimizer(enc, lr=1e-4)
            w_avg = G.mapping.w_avg.view(1, 1, -1)
            # BASELINE config 5 is fp16: the reference's autocast + GradScaler (stylegan3_hvae_full.py:487,669,693-696)
            # as f16 encoder / synthesis with a dynamic loss scaler
            scaler = ict.make_f16(comp) if syn_prec == "f16" else None

            def train_step():
                losses = ict.train_step(comp, x, opt, w_avg, rec_weight=1.0, perceptual_weight=0.0, kl_weight=0.01,
                                        scaler=scaler)
                vec = torch.cat([(losses["rec_loss"].double() * batch).view(1),
                                 (losses["kl_loss"].double() * batch).view(1), counts[1:]])
                return icd.allreduce_sum(vec, device=dev)

        def code_record(codes, kind):
            """[index mismatches vs the first step's codes, out-of-range codes, hist[256]] (ic2_code_record)."""
            rec = torch.zeros(N_CODES + 2, dtype=torch.int32, device=dev)
            if "codes" not in golden:
                golden["codes"] = codes.clone()
            gold = golden["codes"]
            nv.call("ic2_code_record", nv.ptr(codes), kind, N_CODES, 8 if kind == 0 else 0, nv.ptr(gold),
                    codes.numel(), nv.ptr(rec), stream)
            return torch.cat([rec[N_CODES + 1:], rec[N_CODES:N_CODES + 1], rec[:N_CODES]]).double()

        def step():
            # the fine projector re-draws its fc1 from the CPU generator on every call (reference quirk,
            # stylegan3_hvae_full.py:225-230): a fixed seed per step makes that draw -- and so every code -- the same
            # on every step and every rank (the record's index-mismatch count is then a determinism check)
            torch.manual_seed(5)
            with torch.no_grad():
                if args.config == "c2g":
                    codes = comp.compress_codes(x, discrete_bits=8)
                    img = comp.decompress(codes)
                    rec = code_record(codes, 1)
                else:
                    q = comp.compress(x, quantization_bits=8, deterministic=True)
                    img = comp.decompress(q)
                    rec = code_record(q, 0)
                if img.shape[2] != res:
                    img = ic2.resize_bilinear(img, (res, res))
                sse = icm.uint8_sse(img, x)
            vec = torch.cat([sse.sum().view(1), counts, rec])
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
              "c2g": "images/sec encode+codebook quantize+decode 256px",
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
        "dtype": {"bf16": "bf16", "bf16-all": "bf16", "f16": "f16 (synthesis) / split-bf16 (encoder)",
                  "fp32": "fp32"}[args.precision],
        "data": "synthetic (seeded uniform [-1,1] images resident in HBM, seed 1000+rank; random-init encoder + "
                "SG3-T weights)",
        "config": {"workload": desc, "global_batch": batch * world, "per_gpu_batch": batch, "resolution": res,
                   "generator": f"stylegan3-t-{gen_res} (random init)", "encoder": "HVAE_VGG_Encoder(img_resolution=1024)",
                   "quantization_bits": 8, "parallelism": f"dp{world} (batch-sharded, RCCL metric all_reduce)",
                   "precision": {"encoder": enc_prec if args.config != "c5" else syn_prec, "synthesis": syn_prec}},
        "world_size": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
        "ms_per_step_median": round(median_max, 3),
        "per_rank_ms_per_step": per_rank_ms,
        "rank_input_checksums": [round(c, 6) for c in checksum],
    }
    if dry:
        out["dry_run"] = True
        out["psnr_db_record"] = float(10 * torch.log10(255.0 ** 2 / (vec[0] / vec[1])))
        out["metric_record"] = record_summary(vec)
        out["metric_record"]["hist_sum"] = int(vec[5:].sum())
    elif args.config == "c5":
        out["config"].update(quantization_bits=None, loss="rec MSE + 0.01 KL(w_avg); LPIPS excluded (no weights "
                             "offline)", optimizer="Adam(1e-4, (0.9, 0.999))",
                             encoder_calls="2 per step as the reference (:669, :678), sharing one trunk "
                                           "(from_rgb + blocks + GAP) with the projector heads run twice",
                             parallelism=f"dp{world} (batch-sharded, RCCL gradient all_reduce)")
        out["last_step_losses"] = {"rec_loss": round(vec[0].item() / vec[2].item(), 6),
                                   "kl_loss": round(vec[1].item() / vec[2].item(), 4)}
        if syn_prec == "f16":
            out["config"]["loss_scaler"] = "torch.amp.GradScaler (dynamic, init 2^16; the reference's fp16 branch)"
            out["dtype"] = "f16 (encoder + synthesis, f32 accumulate and master weights)"
    else:
        from image_compression_2_amd import metrics as icm
        out["psnr_db_vs_input"] = round(icm.psnr_from_sums(vec[0].item(), vec[1].item()), 4)
        rs = record_summary(vec)
        rs.pop("psnr_db_vs_input")
        out["metric_record"] = rs
        if args.config == "c2g":
            out["config"]["quantizer"] = "GumbelSoftmaxCompressor (linspace(-1,1,256) codebook, exact argmin)"

    if not dry and not args.no_roofline:
        out["roofline"] = roofline(args, nv, step, sync, barrier, enc, G, res, batch, value / world, enc_prec,
                                   syn_prec)
    if not dry and rank == 0 and not args.no_parity and args.config in ("c2", "c2g", "c4"):
        out["parity"] = parity_record(args, comp, enc, G, x, x_host, res, syn_prec)

    if not dry and rank == 0 and world == 1 and args.config == "c2" and not args.no_secondary:
        # the headline models are done: free them before the C4 models are built, and never let the secondary
        # measurement (an OOM, a parity assertion) cost the headline line
        import gc
        comp = enc = G = step = None
        gc.collect()
        torch.cuda.empty_cache()
        try:
            out["secondary"] = {"c4": secondary_c4(args, dev, sync)}
        except Exception as e:  # noqa: BLE001 -- recorded in the line instead
            out["secondary"] = {"c4": {"error": f"{type(e).__name__}: {e}"[:500]}}
            torch.cuda.empty_cache()

    if rank == 0 and world == 1 and args.cpu_baseline_images > 0 and not dry:
        if args.config == "c5":
            out["cpu_baseline"] = cpu_baseline_train(res, gen_res, 1)
        elif args.config in ("c2r", "c4"):
            out["cpu_baseline"] = cpu_baseline(res, gen_res, 1)
        else:
            out["cpu_baseline"] = cpu_baseline(res, gen_res, args.cpu_baseline_images, codebook=args.config == "c2g")
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        torch.distributed.destroy_process_group()


def secondary_c4(args, dev, sync, steps=10, warmup=3):
    """BASELINE config 4 (batch 8, 1024^2, SG3-T-1024) measured after the headline run, on rank 0 at N=1, so the
    driver's default line carries it: the same step as `--config c4` (encode -> 8-bit quantize -> synthesis -> uint8
    SSE; the code record and metric all_reduce, a few microseconds, left out), HIP events around each of `steps`
    steps after `warmup`, and its parity record.  Not part of `value`."""
    import image_compression_2_amd as ic2
    from image_compression_2_amd import metrics as icm
    res, gen_res, batch, desc = CONFIGS["c4"]
    enc_prec, syn_prec = PRECISIONS[args.precision]
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=enc_prec).to(dev).eval().requires_grad_(False)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=gen_res, precision=syn_prec).to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G)
    x_host = torch.rand(batch, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    x = x_host.to(dev)

    def step():
        torch.manual_seed(5)
        with torch.no_grad():
            q = comp.compress(x, quantization_bits=8, deterministic=True)
            img = comp.decompress(q)
            return icm.uint8_sse(img, x)
    for _ in range(warmup):
        step()
    _, elapsed, per = timed_loop(step, steps, sync, lambda: None, use_events=True)
    rec = {"workload": desc, "value": round(batch * steps / elapsed, 3), "unit": "images/s",
           "ms_per_step": round(elapsed / steps * 1e3, 3), "ms_per_step_median": round(statistics.median(per), 3),
           "steps": steps, "warmup": warmup,
           "note": "untimed w.r.t. the headline value: measured after it, same protocol on one GPU"}
    if not args.no_parity:
        ns = argparse.Namespace(**vars(args))
        ns.config = "c4"
        rec["parity"] = parity_record(ns, comp, enc, G, x, x_host, res, syn_prec)
    return rec


PARITY_FIXTURE = os.path.join(ROOT, "tests", "golden", "parity_means.npz")
PARITY_SIGMAS = {"34dB": 0.039, "46dB": 0.01}   # target = reference + N(0, sigma^2): README.md:381's ~34 dB, and 46 dB
PARITY_BARS = {"index_mismatch_frac": 1e-3, "psnr_delta_db": 0.01}   # north star: bit-exact indices, 0.01 dB


def parity_record(args, comp, enc, G, x, x_host, res, syn_prec):
    """Parity of the benched mode on the benched input (rank 0, untimed).
      indices: the benched encoder's 8-bit indices vs the fp32 oracle's, from the committed oracle means of the same
               images (tests/golden/parity_means.npz; input checked by its sha256), both through the product's
               bit-exact quantizer kernel;
      psnr:    north-star PSNR deltas (uint8 PSNR, hvae_training.py:368-395) at targets = reference + N(0, sigma^2):
               'same_latents' = the benched synthesis vs the fp32 HIP path on the benched codes (all images);
               'end_to_end' = the benched encode + quantize + synthesis vs the fp32 reconstruction of the oracle's codes
               (the fixture's images).  The fp32 path is pinned to the CPU synthesis restatement within 1e-3
               (tests/test_gpu_path.py)."""
    import hashlib
    import numpy as np
    import image_compression_2_amd as ic2
    from image_compression_2_amd import metrics as icm
    key = "c4" if args.config == "c4" else "c2"
    fx = np.load(PARITY_FIXTURE)
    m_or = torch.from_numpy(fx[f"{key}_means"]).to(x.device)
    k = min(m_or.shape[0], x.shape[0])
    sha = hashlib.sha256(x_host[:m_or.shape[0]].numpy().tobytes()).digest()
    rec = {"reference": f"fp32 oracle means of the first {k} benched images ({os.path.relpath(PARITY_FIXTURE, ROOT)})",
           "input_sha256_matches_fixture": bool(sha == bytes(fx[f"{key}_x_sha256"]))}
    if not rec["input_sha256_matches_fixture"] or x.shape[2] != res:
        rec["error"] = "benched input differs from the fixture's"
        return rec
    with torch.no_grad():
        torch.manual_seed(5)   # the benched step's fc1 draw
        _, m, _ = enc(x)
        q_b, i_b = ic2.quantize_uniform(m, 8, return_indices=True)
        q_or, i_or = ic2.quantize_uniform(m_or, 8, return_indices=True)
        d = (i_b[:k] - i_or[:k]).abs()
        mism = int((d > 0).sum())
        rec["indices"] = {"bits": 8, "latents": int(d.numel()), "mismatches": mism,
                          "mismatch_frac": mism / d.numel(), "max_abs_index_diff": int(d.max()),
                          "max_abs_mean_diff": float((m[:k] - m_or[:k]).abs().max()),
                          "bar": PARITY_BARS["index_mismatch_frac"]}
        if args.config == "c2g":
            rec["indices"]["note"] = ("uniform 8-bit indices of the benched encoder's means; the codebook argmin over "
                                      "linspace(-1, 1, 256) is the same grid")
        img_b = G.synthesis(q_b)
        img_or_b = G.synthesis(q_or[:k])
        prec = G.precision
        try:
            G.set_precision("fp32")
            ref_same = G.synthesis(q_b)
            ref_or = G.synthesis(q_or[:k])
        finally:
            G.set_precision(prec)
        if img_b.shape[2] != res:
            img_b, img_or_b, ref_same, ref_or = (ic2.resize_bilinear(t, (res, res))
                                                 for t in (img_b, img_or_b, ref_same, ref_or))
        psnr = {}
        for name, sigma in PARITY_SIGMAS.items():
            cases = {"same_latents": (img_b, ref_same), "end_to_end": (img_b[:k], ref_or),
                     "synthesis_only": (img_or_b, ref_or)}
            row = {"sigma": sigma}
            for case, (a, ref) in cases.items():
                g = torch.Generator().manual_seed(77)
                target = ref + (sigma * torch.randn(ref.shape, generator=g)).to(ref.device)
                p_ref = icm.psnr(ref, target)
                row[case] = {"psnr_ref_db": round(p_ref, 4), "delta_db": round(icm.psnr(a, target) - p_ref, 5)}
            psnr[name] = row
        rec["psnr"] = psnr
        rec["max_abs_pixel_diff_same_latents"] = float((img_b - ref_same).abs().max())
    deltas = [abs(v["delta_db"]) for row in rec["psnr"].values() for c, v in row.items() if c != "sigma"]
    rec["synthesis_precision"] = syn_prec
    rec["bar_psnr_delta_db"] = PARITY_BARS["psnr_delta_db"]
    rec["meets_bars"] = bool(rec["indices"]["mismatch_frac"] <= PARITY_BARS["index_mismatch_frac"]
                             and rec["indices"]["max_abs_index_diff"] <= 1 and max(deltas) < PARITY_BARS["psnr_delta_db"])
    return rec


def practical_peak(rl, size=8192, reps=10):
    """The dense 16-bit MFMA rate this box delivers, measured beside the kernels: torch.matmul (hipBLASLt) on bf16
    size^3 operands, HIP events over `reps` calls after 3 warmups.  Under a sustained MFMA load the chip runs below the
    clock the 2.5 PF spec assumes (profiles/r2_gemm_calibration.json: ~1.4 PF), so this is the ceiling
    a conv kernel can practically reach; `peak` / `frac` stay on the spec figure."""
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(size, size, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(size, size, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(3):
        c = a @ b
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    tf = 2.0 * size ** 3 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    del a, b, c
    out = {"kernel": f"torch.matmul bf16 {size}^3 (hipBLASLt), same process", "achieved_tflops": round(tf, 1),
           "spec_frac": round(tf / BF16_PEAK_TFLOPS, 4), "conv_family_frac": round(rl["achieved"] / tf, 4)}
    dm = rl.get("dominant", {})
    if dm.get("achieved") is not None:
        out["dominant_frac"] = round(dm["achieved"] / tf, 4)
    if dm.get("achieved_algorithmic") is not None:
        out["dominant_frac_algorithmic"] = round(dm["achieved_algorithmic"] / tf, 4)
    return out


def roofline(args, nv, step, sync, barrier, enc, G, res, batch, img_s_per_gpu, enc_prec, syn_prec):
    """The instrumented pass: every conv entry point (and every filtered lrelu) bracketed by HIP events.
      conv family: algorithmic FLOPs announced by the product per launch (the reference's conv FLOPs) / the summed
                   time of every conv launch -> achieved, frac of the dense bf16 peak;
      dominant:    the kernel instance with the largest share of that time (launch plan, ic2_conv_plan): its
                   launches' algorithmic and executed (padded-channel) MFMA FLOPs / their time;
      flr:         the fused filtered lrelu against its FIR-on-VALU bound and its HBM floor."""
    train = args.config == "c5"
    conv_names = TRAIN_CONV_ENTRIES if train else CONV_ENTRIES
    timer = CallTimer(nv, conv_names + FLR_ENTRIES)
    timer.install()
    timer.enabled = True
    n_inst = min(args.steps, 5 if train else 10)
    try:
        timed_loop(step, n_inst, sync, barrier, use_events=True)
    finally:
        timer.enabled = False
        timer.uninstall()
    conv_calls = timer.calls(conv_names)
    conv_ms = sum(c[3] for c in conv_calls)
    peak = BF16_PEAK_TFLOPS if args.precision != "fp32" else F32_PEAK_TFLOPS
    per = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # plan -> calls, ms, alg flops, executed flops
    for name, a, f, ms in conv_calls:
        plan, exe = conv_call_plan(nv, name, a)
        r = per[plan]
        r[0] += 1
        r[1] += ms
        r[2] += f or 0.0
        r[3] += exe
    if train:
        alg = training_flops_per_image(enc, G, res) * batch * n_inst
        kernel = "ic2 conv family forward + dgrad (implicit GEMM) + wgrad"
    else:
        alg = sum(f for _, _, f, _ in conv_calls if f)
        missing = [n for n, _, f, _ in conv_calls if f is None]
        assert not missing, f"conv calls without announced FLOPs: {set(missing)}"
        kernel = ("ic2 conv family: every conv entry point of the step (from_rgb, encoder convs, synthesis input 1x1, "
                  "modulated convs, ToRGB)")
    achieved = alg / (conv_ms * 1e-3) / 1e12
    dom_plan, d = max(per.items(), key=lambda kv: kv[1][1])
    rl = {"bound": "mfma", "kernel": kernel, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
          "frac": round(achieved / peak, 4), "traffic": None, "launches": len(conv_calls),
          "avg_launch_ms": round(conv_ms / max(len(conv_calls), 1), 4), "conv_ms_per_step": round(conv_ms / n_inst, 3),
          "algorithmic_gflop_per_image": round(alg / (batch * n_inst) / 1e9, 2),
          "executed_gflop_per_image": round(sum(r[3] for r in per.values()) / (batch * n_inst) / 1e9, 2),
          "path_frac": round(img_s_per_gpu * alg / (batch * n_inst) / (peak * 1e12), 4),
          "precision": {"encoder": enc_prec, "synthesis": syn_prec}}
    rl["dominant"] = {"kernel": dom_plan, "launches_per_step": round(d[0] / n_inst, 2),
                      "ms_per_step": round(d[1] / n_inst, 3), "avg_launch_ms": round(d[1] / d[0], 4),
                      "algorithmic_gflop_per_launch": round(d[2] / d[0] / 1e9, 3) if d[2] else None,
                      "achieved": round(d[2] / (d[1] * 1e-3) / 1e12, 2) if d[2] else None,
                      "executed_achieved": round(d[3] / (d[1] * 1e-3) / 1e12, 2),
                      "frac": round(d[2] / (d[1] * 1e-3) / 1e12 / peak, 4) if d[2] else None,
                      "executed_frac": round(d[3] / (d[1] * 1e-3) / 1e12 / peak, 4)}
    if dom_plan.startswith("wino"):
        # a Winograd instance issues 2/3 of the direct conv's MFMA FLOPs: its roofline fraction is the executed
        # (MFMA-issued) one, <= 1; the algorithmic (direct-conv FLOPs) figure stays beside it
        dm = rl["dominant"]
        dm["frac_algorithmic"], dm["frac"] = dm["frac"], dm["executed_frac"]
        dm["achieved_algorithmic"], dm["achieved"] = dm["achieved"], dm["executed_achieved"]
    rl["per_kernel"] = {k: {"launches_per_step": round(v[0] / n_inst, 2), "ms_per_step": round(v[1] / n_inst, 3),
                            "alg_tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[2] else None,
                            "executed_tflops": round(v[3] / (v[1] * 1e-3) / 1e12, 1)}
                        for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}
    if not train:
        esz = 2 if args.precision != "fp32" else 4
        split = enc_prec == "bf16x3"
        wb, n_conv = weight_bytes(enc, G, res, esz, enc_split=split)
        rl["algorithmic_bytes_per_launch"] = round(
            (algorithmic_bytes_per_image(enc, G, res, esz, enc_split=split) * batch + wb) / n_conv)
        pm = pmc_traffic(args.config, args.precision, batch)
        if pm is not None:
            # the committed PMC run describes the code it ran: its dispatch names must cover every kernel instance
            # the current launch plan runs, else the figure is from an earlier build and is reported as stale
            names = list(pm.get("dispatches", {}))
            missing = sorted({t for plan in per for t in plan_kernel_tags(plan) if not any(t in d for d in names)})
            rl["traffic_src"] = pm["src"]
            rl["traffic_unit"] = "bytes/launch"
            if missing:
                rl["traffic_stale"] = {"pmc_bytes_per_launch": pm["hbm_bytes_per_launch"],
                                       "kernels_not_in_pmc_run": missing}
            else:
                rl["traffic"] = pm["hbm_bytes_per_launch"]
    if args.precision != "fp32":
        rl["practical_peak"] = practical_peak(rl)
    flr_calls = timer.calls(FLR_ENTRIES)
    if syn_prec in ("bf16", "f16") and flr_calls and not train:
        flr_ms = sum(c[3] for c in flr_calls)
        f_img, b_img, bound_img = flr_work_per_image(G)
        flr_step = flr_ms / n_inst
        hbm_floor = b_img * batch / (HBM_PEAK_GBS * 1e9) * 1e3
        rl["flr"] = {
            "kernel": "ic2 flrelu_mfma (fused filtered lrelu, every synthesis layer but ToRGB)",
            "bound": "hbm (the kernel runs its FIRs on f16 MFMA, so its floor is the compulsory bytes at 8 TB/s); "
                     "bound_ms_per_step = SURVEY 8(d)'s FIR-on-f32-VALU bound, for comparison",
            "fir_gflop_per_image": round(f_img / 1e9, 3), "bytes_per_image": round(b_img),
            "ms_per_step": round(flr_step, 3), "hbm_floor_ms_per_step": round(hbm_floor, 3),
            "frac_of_hbm_floor": round(hbm_floor / flr_step, 4),
            "achieved_gbs": round(b_img * batch / (flr_step * 1e-3) / 1e9, 1),
            "bound_ms_per_step": round(bound_img * batch * 1e3, 3),
            "frac_of_bound": round(bound_img * batch * 1e3 / flr_step, 4),
            "achieved_tflops": round(f_img * batch / (flr_step * 1e-3) / 1e12, 2), "launches": len(flr_calls)}
    return rl


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        icd.launch(args.gpus, run, args)   # self-launch: one spawned process per GPU
        return
    run(args)


if __name__ == "__main__":
    main()
