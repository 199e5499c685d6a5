"""CPU: the C-ABI library, the host-side mirror of the reference interface, and the no-fallback rule."""
import hashlib
import os
import re

import numpy as np
import pytest
import torch

import image_compression_2_amd as ic2
from image_compression_2_amd import _native as nv
from image_compression_2_amd import distributed as icd
from oracle import sg3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ C ABI
def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "ic2ops.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ic2_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = nv.load()
    declared = _declared_symbols()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(nv.exported_symbols()), "ctypes signature table out of sync with ic2ops.h"
    assert lib.ic2_abi_version() == 1


def test_integration_index_lists_every_entry_point():
    """INTEGRATION.md's entry-point index names every function the header declares (`x`(`_floats`) names both)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    doc = re.sub(r"`(ic2_\w+)`\(`(_\w+)`\)", lambda m: f"`{m.group(1)}` `{m.group(1)}{m.group(2)}`", doc)
    listed = set(re.findall(r"`(ic2_[a-z0-9_]+)`", doc))
    assert [s for s in _declared_symbols() if s not in listed] == []


def test_argument_errors_are_reported_without_a_gpu():
    """Validation happens before any launch: a bad call returns IC2_E_INVALID with a message."""
    lib = nv.load()
    rc = lib.ic2_quantize_uniform(None, 16, 99, None, None, None)
    assert rc == 1
    assert b"bits" in lib.ic2_last_error()
    rc = lib.ic2_conv_igemm(None, None, None, 0, 0, 1, 8, 8, 32, 32, 32, 3, 3, 1, 8, 8, None, None, 0, 0.0, 1.0, -1.0,
                            1.0, 0, None)
    assert rc == 1


def test_round2_entry_points_validate_before_launch():
    """The batched modulation prep, the direct from_rgb, the GroupNorm affine table and the GroupNorm-input conv
    reject bad arguments (IC2_E_INVALID / IC2_E_UNSUPPORTED + message) before any HIP call."""
    import ctypes
    import numpy as np
    lib = nv.load()
    rec = np.zeros([21, 16], dtype=np.int64)
    # 21 layers > 20
    assert lib.ic2_modconv_prep_batched(ctypes.c_void_p(16), 512 * 16, 2, 512, 21, rec.ctypes.data_as(ctypes.c_void_p),
                                        None) == 1
    assert b"nl=21" in lib.ic2_last_error()
    # a record with null pointers
    assert lib.ic2_modconv_prep_batched(ctypes.c_void_p(16), 512 * 16, 2, 512, 1, rec.ctypes.data_as(ctypes.c_void_p),
                                        None) == 1
    assert b"layer record 0" in lib.ic2_last_error()
    # rows longer than the LDS-staged small GEMM holds
    rec[0, :6] = 16
    rec[0, 6:12] = [512, 600, 640, 64, 64, 1]
    assert lib.ic2_modconv_prep_batched(ctypes.c_void_p(16), 512 * 16, 2, 512, 1, rec.ctypes.data_as(ctypes.c_void_p),
                                        None) == 1
    assert b"longer than 512" in lib.ic2_last_error()
    # from_rgb: 5 input channels / a 96-wide output
    f = ctypes.c_void_p(16)
    assert nv.query("ic2_from_rgb_conv", f, 5, f, 32, f, f, 1, 8, 8, 32, None) == 1
    assert b"cin" in lib.ic2_last_error()
    assert nv.query("ic2_from_rgb_conv", f, 3, f, 32, f, f, 1, 8, 8, 96, None) == 1
    # GroupNorm affine table: channels not divisible by the groups
    assert nv.query("ic2_gn_affine_table", f, f, f, 2, 30, 32, 32, f, None) == 1
    # GroupNorm-input conv: only where the 64-channel halo conv runs the shape
    assert nv.query("ic2_conv3x3_gnin_supported", 1, 8, 256, 256, 64, 64, 3, 3, 1) == 1
    assert nv.query("ic2_conv3x3_gnin_supported", 1, 8, 256, 256, 32, 64, 3, 3, 1) == 0
    assert nv.query("ic2_conv3x3_gnin_supported", 0, 8, 256, 256, 64, 64, 3, 3, 1) == 0
    assert nv.query("ic2_conv3x3_gnin_gn_fwd", f, None, 0.2, f, f, 1, 8, 256, 256, 64, 64, 64, 3, 3, 1, f, 32,
                    1e-5, f, 1 << 20, None, 0, -1, None) == 1


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
@pytest.mark.parametrize("os_dma", [0, 1])
def test_lds_dma_wait_states(os_dma):
    """Every asm LDS-DMA of the strip kernels (fm_dma16) has the wait states the hardware needs in front of it: 5 after
    a VALU write of a descriptor SGPR, 1 after the SALU write of M0 (round-3 oscale-row failures: a spilled descriptor
    restored by v_readlane one instruction before the DMA).  Audited on the gfx950 assembly by tools/audit_lds_dma.py,
    for the production build and the backward's oscale-row DMA (FBM_OS_DMA)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "audit_lds_dma.py"), f"-DFBM_OS_DMA={os_dma}"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 short of wait states" in r.stdout


def test_conv_gn_rejects_f16_operands():
    """the fused conv + GroupNorm statistics path is bf16 halo-conv code.  f16 operands are
    refused at the entry point (never reach the bf16 MFMA) and the fusion query never reports f16 as fusable."""
    import ctypes
    lib = nv.load()
    f = ctypes.c_void_p(16)
    for fuse in (-1, 0, 1):
        # 64 -> 64 channels at 256^2: the halo conv's shape, fused on request in bf16
        assert nv.query("ic2_conv3x3_gn_fuses", nv.F16, 8, 256, 256, 64, 64, 64, 3, 3, 1, 32, fuse) == 0
        assert nv.query("ic2_conv3x3_gn_fwd", f, f, f, nv.F16, 8, 256, 256, 64, 64, 64, 3, 3, 1, f, 32, 1e-5, f,
                        1 << 24, None, 0, fuse, None) == 1
        assert b"dtype" in lib.ic2_last_error()
        assert nv.query("ic2_conv3x3_gnin_gn_fwd", f, f, 0.2, f, f, nv.F16, 8, 256, 256, 64, 64, 64, 3, 3, 1, f, 32,
                        1e-5, f, 1 << 24, None, 0, fuse, None) == 1
    assert nv.query("ic2_conv3x3_gn_fuses", nv.BF16, 8, 256, 256, 64, 64, 64, 3, 3, 1, 32, 1) == 1


def test_product_path_refuses_cpu_tensors():
    with pytest.raises(RuntimeError, match="ROCm"):
        ic2.quantize_uniform(torch.zeros(4, 16, 512))
    enc = ic2.HVAE_VGG_Encoder(img_resolution=64, channel_base=256, channel_max=32, w_dim=32)
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm"):
        enc(torch.zeros(1, 3, 32, 32))


def test_grad_mode_forwards_reach_the_device_and_refuse_backward():
    """Inference keeps working in grad mode: no forward refuses up front any more -- each one reaches the
    device check (CPU tensors: no fallback) -- and a HIP forward without a backward returns outputs whose
    .backward() raises AutogradUnsupported (nv.refuse_backward) instead of silently training nothing."""
    enc = ic2.HVAE_VGG_Encoder(img_resolution=64, channel_base=256, channel_max=32, w_dim=32)
    with pytest.raises(RuntimeError, match="ROCm"):
        enc(torch.zeros(1, 3, 32, 32))   # the encoder trains through its HIP autograd path (autograd_ops)
    with pytest.raises(RuntimeError, match="ROCm"):
        enc.blocks[0](torch.zeros(1, 32, 8, 8))
    G = ic2.Generator(img_resolution=256)
    ws = torch.zeros(1, 16, 512)
    for w in (ws, ws.clone().requires_grad_(True)):
        with pytest.raises(RuntimeError, match="ROCm"):
            G.synthesis(w)               # unfrozen G: the inference path (its output refuses backward)
    G.requires_grad_(False)
    with pytest.raises(RuntimeError, match="ROCm"):
        G.synthesis(ws.clone().requires_grad_(True))   # frozen G, grads into W+: the HIP autograd path
    disc = ic2.GumbelSoftmaxDiscretization(32, 256)   # learnable temperature
    with pytest.raises(RuntimeError, match="ROCm"):
        disc(torch.zeros(1, 16, 32))
    # the refusal node itself: pass-through in the forward (same storage), raise on backward, no-op without grad
    p = torch.nn.Linear(2, 2)
    out = torch.randn(4)
    y, idx = nv.refuse_backward("t", (out, torch.arange(3)), (), (p,))
    assert y.requires_grad and y.data_ptr() == out.data_ptr() and idx.dtype == torch.int64
    with pytest.raises(nv.AutogradUnsupported):
        y.sum().backward()
    with torch.no_grad():
        assert nv.refuse_backward("t", out, (), (p,)) is out
    p.requires_grad_(False)
    assert nv.refuse_backward("t", out, (torch.zeros(2),), (p,)) is out


# ------------------------------------------------------------------ seeded construction = reference
def test_encoder_init_matches_reference_small(golden_dir):
    d = np.load(os.path.join(golden_dir, "encoder_small.npz"))
    torch.manual_seed(7)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=64, img_channels=3, w_dim=32, num_ws=16, block_split=(5, 12),
                               channel_base=256, channel_max=32)
    sd = enc.state_dict()
    ref_keys = sorted(k[3:] for k in d.files if k.startswith("sd/"))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:
        assert np.array_equal(sd[k].numpy(), d["sd/" + k]), k


def test_encoder_init_matches_reference_full_sha(golden_dir):
    d = np.load(os.path.join(golden_dir, "encoder_full.npz"))
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    h = hashlib.sha256()
    for k, v in enc.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().numpy().tobytes())
    assert np.frombuffer(h.digest(), np.uint8).tolist() == d["state_sha256"].tolist()


@pytest.mark.parametrize("res", [256, 1024])
def test_generator_matches_oracle_construction(res):
    torch.manual_seed(5)
    G = ic2.Generator(z_dim=512, w_dim=512, img_resolution=res, img_channels=3)
    sd = G.state_dict()
    ref = sg3.init_params(res, seed=5)
    for k, v in ref.items():
        assert k in sd, k
        assert torch.equal(sd[k].float(), v.float()), k
    assert G.num_ws == 16 and G.synthesis.num_ws == 16
    _, layers = sg3.layer_table(res)
    assert G.synthesis.layer_names == [L["name"] for L in layers]
    for L, name in zip(layers, G.synthesis.layer_names):
        mine = getattr(G.synthesis, name)
        assert mine.padding == L["padding"] and mine.up_factor == L["up"] and mine.down_factor == L["down"]


def test_generator_duck_type():
    G = ic2.Generator(img_resolution=256)
    assert (G.z_dim, G.w_dim, G.num_ws, G.img_resolution, G.img_channels) == (512, 512, 16, 256, 3)
    assert G.mapping.w_avg.shape == (512,)
    assert sum(p.numel() for p in G.synthesis.parameters()) > 20_000_000


def test_compressor_freezes_generator():
    G = ic2.Generator(img_resolution=256)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=64, channel_base=256, channel_max=32, w_dim=512)
    ic2.StyleGAN3Compressor(enc, G, training_resolution=256)
    assert not any(p.requires_grad for p in G.parameters())
    gc = ic2.GumbelSoftmaxCompressor(enc, G)
    assert torch.equal(gc.discretization.codebook, torch.linspace(-1, 1, 256))
    assert gc.discretization.log_temperature.requires_grad


# ------------------------------------------------------------------ host-side sharding
@pytest.mark.parametrize("n,world", [(256, 8), (32, 1), (10, 4), (3, 4), (0, 2)])
def test_shard_partition(n, world):
    spans = [icd.shard(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, _) in zip(spans, spans[1:]):
        assert b == c and b >= a
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


# ------------------------------------------------------------------ launch plan (host-only query) + knob gating
def test_conv_launch_plan_names():
    """ic2_conv_plan is the dispatcher's own plan function (no GPU needed): the SG3-T-256 / encoder shapes of the
    C2 workload land on the instances DESIGN.md lists."""
    plan = lambda *a: nv.conv_plan(*a)
    B = 32
    # SG3-T-256 L8 (512 -> 512 at 148^2, f16 NHWC16 out): the 8-phase 256 x 256 kernel
    assert plan(nv.BF16, nv.F16, nv.NHWC16, B, 148, 148, 512, 512, 512, 3, 3, 2) == "igemm8_og2"
    # L9 (512 -> 362, cout_p 384): 256-wide + 128 x 512 launches
    assert plan(nv.BF16, nv.F16, nv.NHWC16, B, 148, 148, 512, 384, 362, 3, 3, 2) == "igemm8_og2+og1"
    # L11 (256 -> 181 at 276^2, cout_p 192): the 4-wave halo GEMM, two 96-wide o-tiles on 8 x 32-pixel tiles
    assert plan(nv.BF16, nv.F16, nv.NHWC16, B, 276, 276, 256, 192, 181, 3, 3, 2) == "hg4_o96_w32_p2"
    # a 192-wide output that pads less on 16-wide pixel tiles keeps the 192-wide 16-wide-tile instance
    assert plan(nv.BF16, nv.F16, nv.NHWC16, B, 47, 47, 256, 192, 192, 3, 3, 1) == "hg4_o192_w16_s4"
    # ToRGB: the VALU 1x1 kernel
    assert plan(nv.BF16, nv.F32, nv.NCHW, B, 256, 256, 128, 32, 3, 1, 1, 0) == "torgb"
    # encoder block 0 conv2 in bf16 (64 -> 64 at 256^2): the halo direct conv; split-bf16 (192 tripled channels): hg4
    assert plan(nv.BF16, nv.BF16, nv.NHWC, B, 256, 256, 64, 64, 64, 3, 3, 1) == "hconv_64_64"
    assert plan(nv.BF16, nv.F32, nv.NHWC, B, 256, 256, 192, 64, 64, 3, 3, 1).startswith("hg4_o64")
    # L0-L2 (512 -> 512, 36^2 pad 2 at batch 32: 362 tiles = 1.41 rounds): whole rounds at full K + the tail split
    # over K (f32 partials in a caller-owned workspace of 2 x M x cout_p floats); L3 (52^2: 730 tiles) is not split
    assert plan(nv.F16, nv.F16, nv.NHWC16, B, 36, 36, 512, 512, 512, 3, 3, 2) == "igemm8_og2_tail_f16"
    assert nv.query("ic2_conv_igemm_ws_bytes", nv.F16, B, 36, 36, 512, 512, 3, 3, 2) == 2 * B * 38 * 38 * 512 * 4
    assert plan(nv.F16, nv.F16, nv.NHWC16, B, 52, 52, 512, 512, 512, 3, 3, 2) == "igemm8_og2_f16"
    # small late encoder blocks: split-K implicit GEMM; fp32 mode: the exact-f32 tile
    assert plan(nv.BF16, nv.F32, nv.NHWC, B, 4, 4, 1536, 512, 512, 3, 3, 1).endswith("_splitk")
    assert plan(nv.F32, nv.F32, nv.NHWC, 2, 16, 16, 64, 64, 64, 3, 3, 1).startswith("igemm_f32")


def test_knobs_are_ignored_without_dev_mode():
    """The development knobs (forced instances / A/B switches) change the launch plan only under IC2_DEV=1."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from image_compression_2_amd import _native as nv; "
            "print(nv.conv_plan(nv.BF16, nv.F16, nv.NHWC16, 32, 148, 148, 512, 512, 512, 3, 3, 2), "
            "nv.query('ic2_dev_mode'))" % ROOT)
    outs = {}
    for dev in ("0", "1"):
        env = dict(os.environ, IC2_IGEMM_TILE="4", IC2_DEV=dev)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs[dev] = r.stdout.split()
    assert outs["0"] == ["igemm8_og2", "0"]
    assert outs["1"] == ["igemm_128x128", "1"]
