"""Parity of the BENCHED mode: the exact C2 workload (BASELINE.json configs[1]) -- batch 32, 256^2,
HVAE_VGG_Encoder(img_resolution=1024) -> 8-bit uniform quantizer -> SG3-T-256 synthesis, in bench.py's precisions
(encoder split-bf16 'bf16x3'; synthesis f16 = the default since round 4, and bf16) -- against the oracle.

Reference path: stylegan3_hvae_full.py:295-329 (compress -> decompress), metric hvae_training.py:368-395.
The fp32 oracle means of this exact input (bench.py's rank-0 batch) are the committed fixture
tests/golden/parity_means.npz (tests/golden/make_parity_means.py: oracle/encoder.py, pinned to the reference's own
encoder by tests/golden/encoder_full.npz; the fixture itself is re-derived on 2 images by
tests/test_oracle.py::test_parity_means_fixture); the reference reconstruction is the fp32 path on the oracle's
quantized latents (pinned to the CPU synthesis restatement at 1e-3 by test_gpu_path.py, re-checked here on 1 image).

What is asserted (thresholds are module constants, measured values are printed and recorded in DESIGN.md (c)):
  (a) quantized indices (north star: bit-exact): the benched encoder's means within ENC_TOL of the oracle's;
      at most IDX_FRAC of the 8-bit indices differ, each by one and only where the oracle latent lies within
      HALF_STEP of a rounding boundary (the fp32 oracle's own reduction-order noise is ~1e-6 there);
  (b) reconstruction: signal-to-error of the bf16 image against the reference reconstruction, synthesis only
      (same latents) and end to end (benched latents), above SNR_FLOOR_SYN / SNR_FLOOR_E2E;
  (c) the north-star PSNR bar: |PSNR(bench, target) - PSNR(reference, target)| below PSNR_TOL at a target
      where PSNR is sensitive (reference reconstruction + Gaussian noise at the README's 34 dB operating
      point), and at 46 dB.
The all-bf16 encoder (bench --precision bf16-all) is measured alongside and reported, not asserted.  The f16
synthesis (bench --precision f16: 11-bit significands at the bf16 MFMA rate) is asserted against its own, tighter
floor and against the PSNR bar at both operating points, 46 dB included.
The perturbation test shows (b) can fail: one bf16-ulp (2^-8) error in every layer's filtered-lrelu gain
or up-filter taps drops the SNR below the floor.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

import image_compression_2_amd as ic2
from image_compression_2_amd import metrics as icm
from oracle import encoder as oe
from oracle import sg3

pytestmark = pytest.mark.gpu
GOLDEN_MEANS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "parity_means.npz")

B = 32
# thresholds.  Round 2 (all-bf16 encoder) measured max|dm| 2.4e-3 and 4.6 % of the indices off by one; the split-bf16
# encoder is emulated on the CPU at max|dm| 3.5e-6, 1 flip in 32768 at 1.4e-6 from a half-step
ENC_TOL = 5e-5          # max |means_bench - means_oracle| (latent units; the 8-bit step is 2/255 = 0.0078)
IDX_FRAC = 1e-3         # fraction of the 8-bit indices that may differ (by one) from the oracle's
HALF_STEP = 1e-4        # a differing index's oracle latent lies within this of a rounding boundary
SNR_FLOOR_SYN = 38.0    # dB, bf16 synthesis vs the fp32 reference on identical latents
SNR_FLOOR_E2E = 38.0    # dB, benched encode + quantize + synthesis vs the reference reconstruction
PSNR_TOL = 0.005        # dB at the 34 dB operating point, end to end (north star: 0.01)
PSNR_TOL_46 = 0.01      # dB at 46 dB
IDX_COUNT_BENCH = 69    # index mismatches of the benched mode at round 5 (BENCH_r05 parity): a ceiling, not a target
IDX_COUNT_FP32 = 4      # the fp32 parity mode: measured 2 on this batch (round 6)
SNR_FLOOR_F16 = 52.0    # dB, the f16 synthesis (bench --precision f16) vs the fp32 reference (CPU emulation: 60.5)


def _snr_db(a, ref):
    a, ref = a.double().cpu(), ref.double().cpu()
    return 10 * np.log10((ref ** 2).sum().item() / max(((a - ref) ** 2).sum().item(), 1e-300))


@pytest.fixture(scope="module")
def c2(cuda):
    import bench
    from conftest import golden_script
    pm = golden_script("make_parity_means")
    bench_input, fine_fc1 = pm.bench_input, pm.fine_fc1
    enc_prec, syn_prec = bench.PRECISIONS[bench.DEFAULT_PRECISION]   # the bench's default mode is the one tested here
    assert (enc_prec, syn_prec) == ("bf16x3", "f16")
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=enc_prec).to(cuda).eval().requires_grad_(False)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256).to(cuda).eval().requires_grad_(False)
    x = bench_input(B, 256)
    fx = np.load(GOLDEN_MEANS)
    assert bytes(fx["c2_x_sha256"]) == hashlib.sha256(x.numpy().tobytes()).digest()
    with torch.no_grad():
        torch.manual_seed(5)  # the fine projector re-draws fc1 from the CPU RNG (ref :225-230)
        _, m16, _ = enc(x.to(cuda))
        w1, b1 = fine_fc1()   # the draw the fixture's oracle means were computed with
        assert torch.equal(enc.fine_projector.fc1.weight.detach().cpu(), w1)
        assert torch.equal(enc.fine_projector.fc1.bias.detach().cpu(), b1)
        enc.set_precision("bf16")
        torch.manual_seed(5)
        _, m_allbf16, _ = enc(x.to(cuda))
        enc.set_precision("fp32")
        torch.manual_seed(5)
        _, m_fp32, _ = enc(x.to(cuda))
        enc.set_precision(enc_prec)
        m_or = torch.from_numpy(fx["c2_means"])
        q16, i16 = ic2.quantize_uniform(m16, 8, return_indices=True)
        q_or = oe.quantize_uniform(m_or, 8)
        G.set_precision("fp32")
        ref = G.synthesis(q_or.to(cuda))
        G.set_precision("bf16")
        img_e2e = G.synthesis(q16)
        img_syn = G.synthesis(q_or.to(cuda))
        G.set_precision("f16")
        img_e2e_f16 = G.synthesis(q16)
        img_syn_f16 = G.synthesis(q_or.to(cuda))
        G.set_precision("fp32")
    return dict(enc=enc, G=G, x=x, m16=m16.cpu(), m_or=m_or, i16=i16.cpu().long(), q_or=q_or, ref=ref,
                img_e2e=img_e2e, img_syn=img_syn, m_allbf16=m_allbf16.cpu(), img_e2e_f16=img_e2e_f16,
                img_syn_f16=img_syn_f16, m_fp32=m_fp32.cpu())


def test_c2_reference_reconstruction_is_the_oracle(c2):
    """The fp32 reference reconstruction equals the CPU synthesis restatement (1 of the 32 images)."""
    sd = {k: v.detach().float().cpu() for k, v in c2["G"].state_dict().items()}
    r = sg3.synthesis_forward(sd, 256, c2["q_or"][:1], dtype=torch.float32)
    err = (c2["ref"][:1].cpu() - r).abs().max().item()
    print(f"[c2] fp32 path vs CPU oracle (1 image): max|err| = {err:.2e}")
    assert err < 1e-3


def _index_stats(m, m_or):
    err = (m - m_or).abs()
    i_or = oe.uniform_indices(m_or, 8)
    d = oe.uniform_indices(m, 8) - i_or
    mism = d != 0
    # distance of each mismatched oracle latent to the nearest rounding boundary of the 8-bit grid
    u = (m_or.double() + 1) * 0.5 * 255
    dist = ((u - u.floor() - 0.5).abs() * 2 / 255)[mism]
    return err, d, mism, dist


def test_c2_bench_indices_vs_oracle(c2):
    m16, m_or = c2["m16"], c2["m_or"]
    err, d, mism, dist = _index_stats(m16, m_or)
    assert torch.equal(oe.uniform_indices(m16, 8), c2["i16"])   # the kernel's indices = the closed form
    frac = mism.float().mean().item()
    print(f"[c2] encoder (bench mode) vs oracle: max|dm| = {err.max().item():.3e}, mean|dm| = {err.mean().item():.3e}, "
          f"index mismatches {int(mism.sum())}/{mism.numel()} = {frac:.2e}, max |didx| = {int(d.abs().max())}, "
          f"max half-step distance of a mismatch = {dist.max().item() if dist.numel() else 0.0:.3e}")
    e2, d2, mism2, dist2 = _index_stats(c2["m_allbf16"], m_or)
    print(f"[c2] all-bf16 encoder (reported): max|dm| = {e2.max().item():.3e}, index mismatches "
          f"{int(mism2.sum())}/{mism2.numel()} = {mism2.float().mean().item():.2e}")
    assert err.max().item() < ENC_TOL
    assert d.abs().max().item() <= 1
    assert frac <= IDX_FRAC
    assert int(mism.sum()) <= IDX_COUNT_BENCH
    assert (dist <= HALF_STEP).all()


def test_c2_fp32_mode_indices_vs_oracle(c2):
    """The fp32 parity mode (exact-f32 MFMA encoder) on the C2 batch: a count bar of its own, tighter than the benched
    mode's, every flip by one and at a half-step."""
    err, d, mism, dist = _index_stats(c2["m_fp32"], c2["m_or"])
    print(f"[c2] encoder (fp32 mode) vs oracle: max|dm| = {err.max().item():.3e}, index mismatches "
          f"{int(mism.sum())}/{mism.numel()}, max half-step distance of a mismatch = "
          f"{dist.max().item() if dist.numel() else 0.0:.3e}")
    assert err.max().item() < ENC_TOL
    assert d.abs().max().item() <= 1
    assert int(mism.sum()) <= IDX_COUNT_FP32
    assert (dist <= HALF_STEP).all()


def test_c2_bf16_reconstruction_snr(c2):
    syn = _snr_db(c2["img_syn"], c2["ref"])
    e2e = _snr_db(c2["img_e2e"], c2["ref"])
    p_syn = icm.psnr(c2["img_syn"], c2["ref"])
    p_e2e = icm.psnr(c2["img_e2e"], c2["ref"])
    print(f"[c2] bf16 synthesis-only SNR {syn:.2f} dB (uint8 PSNR {p_syn:.2f}); end-to-end SNR {e2e:.2f} dB "
          f"(uint8 PSNR {p_e2e:.2f})")
    assert syn > SNR_FLOOR_SYN
    assert e2e > SNR_FLOOR_E2E


@pytest.mark.parametrize("sigma,tol", [(0.039, PSNR_TOL), (0.01, None)])
def test_c2_bf16_psnr_bar(c2, sigma, tol):
    """North star: PSNR within 0.01 dB of the reference's.  Target = reference reconstruction + N(0, sigma^2):
    sigma 0.039 puts the reference at ~34 dB (README.md:381's operating point), 0.01 at ~46 dB."""
    g = torch.Generator().manual_seed(77)
    ref = c2["ref"].cpu()
    target = (ref + sigma * torch.randn(ref.shape, generator=g)).to(c2["ref"].device)
    p_ref = icm.psnr(c2["ref"], target)
    out = {}
    for key in ("img_syn", "img_e2e"):
        out[key] = icm.psnr(c2[key], target) - p_ref
    print(f"[c2] sigma={sigma}: PSNR(reference) = {p_ref:.3f} dB; bf16 delta synthesis-only {out['img_syn']:+.4f} dB, "
          f"end-to-end {out['img_e2e']:+.4f} dB")
    if tol is not None:
        assert abs(out["img_syn"]) < tol
        assert abs(out["img_e2e"]) < tol


@pytest.mark.parametrize("what", ["gain", "taps"])
def test_c2_snr_floor_detects_one_ulp_per_layer(c2, what):
    """The floor is not vacuous: a 2^-8 (one bf16 ulp) error in every layer's filtered-lrelu gain, or in the
    largest up-filter tap of every layer, pushes the synthesis-only SNR below SNR_FLOOR_SYN."""
    G = c2["G"]
    layers = [L for L in G.synthesis.layers() if not L.is_torgb]
    saved = [(L.act_gain, L._fu) for L in layers]
    try:
        for L in layers:
            if what == "gain":
                L.act_gain = L.act_gain * (1 + 2 ** -8)
            else:
                fu = L._fu.copy()
                k = int(np.argmax(np.abs(fu)))
                fu[k] = fu[k] * (1 + 2 ** -8)
                L._fu = fu
        G.set_precision("bf16")
        with torch.no_grad():
            img = G.synthesis(c2["q_or"].to(c2["ref"].device))
    finally:
        G.set_precision("fp32")
        for L, (g_, fu) in zip(layers, saved):
            L.act_gain, L._fu = g_, fu
    snr = _snr_db(img, c2["ref"])
    print(f"[c2] perturbed ({what}, 2^-8 per layer): synthesis SNR {snr:.2f} dB")
    assert snr < SNR_FLOOR_SYN


def test_c2_f16_reconstruction_snr(c2):
    syn = _snr_db(c2["img_syn_f16"], c2["ref"])
    e2e = _snr_db(c2["img_e2e_f16"], c2["ref"])
    d = (c2["img_syn_f16"] - c2["ref"]).abs()
    print(f"[c2] f16 synthesis-only SNR {syn:.2f} dB; end-to-end SNR {e2e:.2f} dB; synthesis-only pixel error "
          f"max {d.max().item():.2e} mean {d.mean().item():.2e} (image range [-1, 1]); fraction of pixels within "
          f"1e-3: {(d <= 1e-3).float().mean().item():.4f}")
    assert syn > SNR_FLOOR_F16
    assert e2e > SNR_FLOOR_F16 - 6.0  # the split-bf16 encoder's 20 / 262144 boundary flips cost some


@pytest.mark.parametrize("sigma,tol", [(0.039, PSNR_TOL), (0.01, PSNR_TOL_46)])
def test_c2_f16_psnr_bar(c2, sigma, tol):
    """The PSNR bar in the f16 synthesis mode, asserted at 34 dB and 46 dB (the bf16 mode meets it at 34 dB)."""
    g = torch.Generator().manual_seed(77)
    ref = c2["ref"].cpu()
    target = (ref + sigma * torch.randn(ref.shape, generator=g)).to(c2["ref"].device)
    p_ref = icm.psnr(c2["ref"], target)
    d_syn = icm.psnr(c2["img_syn_f16"], target) - p_ref
    d_e2e = icm.psnr(c2["img_e2e_f16"], target) - p_ref
    print(f"[c2] sigma={sigma}: PSNR(reference) = {p_ref:.3f} dB; f16 delta synthesis-only {d_syn:+.4f} dB, "
          f"end-to-end {d_e2e:+.4f} dB")
    assert abs(d_syn) < tol
    assert abs(d_e2e) < tol


def test_c2_f16_floor_detects_one_ulp_per_layer(c2):
    """The f16 floor is not vacuous: a 2^-11 (one f16 ulp) error in every layer's filtered-lrelu gain pushes the f16
    synthesis SNR below SNR_FLOOR_F16."""
    G = c2["G"]
    layers = [L for L in G.synthesis.layers() if not L.is_torgb]
    saved = [L.act_gain for L in layers]
    try:
        for L in layers:
            L.act_gain = L.act_gain * (1 + 2 ** -11)
        G.set_precision("f16")
        with torch.no_grad():
            img = G.synthesis(c2["q_or"].to(c2["ref"].device))
    finally:
        G.set_precision("fp32")
        for L, g_ in zip(layers, saved):
            L.act_gain = g_
    snr = _snr_db(img, c2["ref"])
    print(f"[c2] perturbed (gain, 2^-11 per layer): f16 synthesis SNR {snr:.2f} dB")
    assert snr < SNR_FLOOR_F16
