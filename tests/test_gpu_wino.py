"""ic2_conv_wino (fused Winograd F(2,3) along x, f16 MFMA) against an fp64 conv of the same operands, next to the
direct f16 implicit GEMM on the same inputs.  Reference: the grouped conv2d of modulated_conv2d [SG3-public] in
its activation-scaling form (stylegan3_hvae_full.py:274,329), i.e. ic2_conv_igemm's contract for 3x3."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from image_compression_2_amd import _native as nv

pytestmark = pytest.mark.gpu


def _run(cuda, n, ci, co, s, pad, layout, out_dt, act, seed=0, cin_p=None, cout_p=None):
    g = torch.Generator(device=cuda).manual_seed(seed)
    cip = cin_p or nv.pad32(ci)
    cop = cout_p or nv.pad32(co)
    ho = s + 2 * pad - 2
    x = torch.zeros(n, s, s, cip, device=cuda, dtype=torch.float16)
    x[..., :ci] = torch.randn(n, s, s, ci, device=cuda, generator=g).to(torch.float16)
    w = torch.randn(co, ci, 3, 3, device=cuda, generator=g)
    st = nv.stream_of(x)
    wp = torch.empty(cop, 3, 3, cip, device=cuda, dtype=torch.float16)
    u = torch.empty(cop, 3, 4, cip, device=cuda, dtype=torch.float16)
    nv.call("ic2_pack_weight", nv.ptr(w), co, ci, 3, 3, cop, cip, 1, 1.0, nv.ptr(wp), nv.F16, None, st)
    nv.call("ic2_pack_weight_wino", nv.ptr(w), co, ci, cop, cip, 1, 1.0, nv.ptr(u), nv.F16, st)
    osc = (torch.rand(n, cop, device=cuda, generator=g) + 0.5) / (9 * ci) ** 0.5
    bias = torch.randn(cop, device=cuda, generator=g) * 0.1
    slope, gain, clamp, mul = (0.2, 1.4142135, 2.5, 0.75) if act else (0.0, 1.0, -1.0, 1.0)
    if layout == nv.NCHW:
        shape = [n, co, ho, ho]
    elif layout == nv.NHWC16:
        shape = [n, cop // 16, ho, ho, 16]
    else:
        shape = [n, ho, ho, cop]
    yd = torch.full(shape, 7.0, device=cuda, dtype=out_dt)
    yw = torch.full(shape, 7.0, device=cuda, dtype=out_dt)
    odt = nv.dtype_code(out_dt)
    nv.conv_igemm(nv.ptr(x), nv.ptr(wp), nv.ptr(yd), nv.F16, odt, n, s, s, cip, cop, co, 3, 3, pad, ho, ho, nv.ptr(osc),
                  nv.ptr(bias), int(act), slope, gain, clamp, mul, layout, st, cuda)
    nv.conv_wino(nv.ptr(x), nv.ptr(u), nv.ptr(yw), nv.F16, odt, n, s, s, cip, cop, co, pad, ho, ho, nv.ptr(osc),
                 nv.ptr(bias), int(act), slope, gain, clamp, mul, layout, st)
    torch.cuda.synchronize()
    # fp64 reference: the f16 input, the f32 pre-normalised weights (each kernel rounds its own weights)
    wn = (w * w.square().mean([1, 2, 3], keepdim=True).rsqrt()).double()
    xr = x[..., :ci].double().permute(0, 3, 1, 2)
    ref = F.conv2d(xr, wn, padding=pad) * osc[:, :co, None, None].double() + bias[None, :co, None, None].double()
    if act:
        ref = (torch.where(ref < 0, ref * slope, ref) * gain).clamp(-clamp, clamp)
    ref = ref * mul

    def as_nchw(y):
        if layout == nv.NCHW:
            return y.double()
        if layout == nv.NHWC16:
            y = y.permute(0, 1, 4, 2, 3).reshape(n, cop, ho, ho)
        else:
            y = y.permute(0, 3, 1, 2)
        return y[:, :co].double()
    return as_nchw(yd), as_nchw(yw), ref, yw


CASES = [  # n, cin, cout, size, pad
    (2, 32, 32, 9, 2),        # tiny, odd output width (11)
    (2, 64, 96, 13, 1),       # pad 1, odd output, cout not a multiple of 128
    (3, 128, 160, 20, 2),     # two o-tiles, the second partial
    (1, 512, 512, 36, 2),     # SG3-T-256 L0 geometry
    (2, 96, 64, 33, 0),       # pad 0
    (2, 256, 384, 52, 2),     # three o-tiles
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_c%d_o%d_s%d_p%d" % c)
@pytest.mark.parametrize("layout,out_dt,act", [(nv.NHWC16, torch.float16, False), (nv.NHWC, torch.float16, True),
                                               (nv.NCHW, torch.float32, True), (nv.NHWC, torch.bfloat16, False)],
                         ids=["nhwc16_f16", "nhwc_f16_act", "nchw_f32_act", "nhwc_bf16"])
def test_conv_wino_matches_fp64(cuda, case, layout, out_dt, act):
    n, ci, co, s, pad = case
    with torch.no_grad():
        yd, yw, ref, _ = _run(cuda, n, ci, co, s, pad, layout, out_dt, act)
    yw, yd, ref = yw.cpu(), yd.cpu(), ref.cpu()
    scale = ref.abs().max().item()
    e_w = (yw - ref).abs().max().item() / scale
    e_d = (yd - ref).abs().max().item() / scale
    # f16 operands: the direct conv's error is the weight / output rounding (~2^-11); the Winograd adds the rounding
    # of U = G g and of V = B^T d (packed f16 adds) -- bounded at 4x the direct conv's, and absolutely
    assert e_w < 4e-3 and e_w <= 4 * e_d + 1e-4, (e_w, e_d)
    assert torch.isfinite(yw).all()


@pytest.mark.parametrize("layout", [nv.NHWC16, nv.NHWC], ids=["nhwc16", "nhwc"])
def test_conv_wino_leaves_padding_channels_and_bounds(cuda, layout):
    """Stores stay inside the tensor: the output is a view into a buffer with sentinel guard bands
    of GUARD elements before and after it; the kernel's input reads deliberately run past the halo lines
    (csrc/wino.hip:41,146), so its stores are checked here.  After the launch both guards are bit-unchanged, every
    valid channel was written (no 7.0 sentinel left), and the padded output channels 40..63 (zero U rows) hold
    0 * acc * oscale + bias = the f16-rounded bias."""
    n, ci, co, cop, s, pad = 2, 64, 40, 64, 17, 2
    ho = s + 2 * pad - 2
    GUARD = 8192
    g = torch.Generator(device=cuda).manual_seed(11)
    cip = nv.pad32(ci)
    x = torch.zeros(n, s, s, cip, device=cuda, dtype=torch.float16)
    x[..., :ci] = torch.randn(n, s, s, ci, device=cuda, generator=g).to(torch.float16)
    w = torch.randn(co, ci, 3, 3, device=cuda, generator=g)
    st = nv.stream_of(x)
    u = torch.empty(cop, 3, 4, cip, device=cuda, dtype=torch.float16)
    nv.call("ic2_pack_weight_wino", nv.ptr(w), co, ci, cop, cip, 1, 1.0, nv.ptr(u), nv.F16, st)
    osc = (torch.rand(n, cop, device=cuda, generator=g) + 0.5) / (9 * ci) ** 0.5
    bias = torch.randn(cop, device=cuda, generator=g) * 0.1
    shape = [n, cop // 16, ho, ho, 16] if layout == nv.NHWC16 else [n, ho, ho, cop]
    numel = n * ho * ho * cop
    base = torch.full([GUARD + numel + GUARD], -1234.5, device=cuda, dtype=torch.float16)
    base[GUARD:GUARD + numel] = 7.0
    y = base[GUARD:GUARD + numel].view(shape)
    assert y.data_ptr() % 16 == 0
    with torch.no_grad():
        nv.conv_wino(nv.ptr(x), nv.ptr(u), nv.ptr(y), nv.F16, nv.F16, n, s, s, cip, cop, co, pad, ho, ho, nv.ptr(osc),
                     nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, layout, st)
    torch.cuda.synchronize()
    b = base.cpu()
    assert (b[:GUARD] == -1234.5).all() and (b[GUARD + numel:] == -1234.5).all(), "store outside the output tensor"
    yc = y.cpu().float()
    yc = yc.permute(0, 1, 4, 2, 3).reshape(n, cop, ho, ho) if layout == nv.NHWC16 else yc.permute(0, 3, 1, 2)
    assert not (yc[:, :co] == 7.0).any(), "a valid output was not written"
    pad_ref = bias[co:].to(torch.float16).float().cpu()[None, :, None, None].expand(n, cop - co, ho, ho)
    assert torch.equal(yc[:, co:], pad_ref)


def test_conv_wino_plan_names_a_tile(cuda):
    for s in (36, 52, 84, 148, 276):
        name = nv.wino_plan(32, s, s, 512, 512, 2)
        assert name.startswith("wino_fx_o128_p") and name.endswith("_f16"), name


def test_wino_adjoint_dgrad_matches_fp64(cuda):
    """The training path's dgrad through the Winograd kernel: conv_nhwc on the adjoint weights (normalised W flipped
    in space, transposed in channels, packed by SynthesisLayer.packed_adjoint_wino) equals dL/da = conv_transpose2d
    of the gradient with W_norm (pad 2 forward -> valid adjoint), next to the direct implicit GEMM on the same pack."""
    from image_compression_2_amd import autograd_ops as ao
    from image_compression_2_amd.networks_stylegan3 import SynthesisLayer

    torch.manual_seed(0)
    L = SynthesisLayer(w_dim=512, is_torgb=False, is_critically_sampled=False, use_fp16=False, in_channels=250,
                       out_channels=320, in_size=50, out_size=50, in_sampling_rate=16, out_sampling_rate=16,
                       in_cutoff=8, out_cutoff=8, in_half_width=4, out_half_width=4).to(cuda)
    n, s_in = 2, 50
    conv = s_in + 2
    assert nv.wino_preferred(nv.F16, n, conv, conv, L.cout_p, L.cin_p, 3, 3, 0)
    g = torch.Generator(device=cuda).manual_seed(3)
    dc = torch.zeros(n, conv, conv, L.cout_p, device=cuda, dtype=torch.float16)
    dc[..., :L.out_channels] = torch.randn(n, conv, conv, L.out_channels, device=cuda, generator=g).to(torch.float16)
    with torch.no_grad():
        da_w = ao.conv_nhwc(dc, L.packed_adjoint(torch.float16), None, L.in_channels, 3, 0, wino=L.packed_adjoint_wino)
        da_d = ao.conv_nhwc(dc, L.packed_adjoint(torch.float16), None, L.in_channels, 3, 0)
    torch.cuda.synchronize()
    w = L.weight.detach().double()
    wn = w * w.square().mean([1, 2, 3], keepdim=True).rsqrt()
    ref = F.conv_transpose2d(dc[..., :L.out_channels].double().permute(0, 3, 1, 2), wn, padding=2)
    got_w = da_w[..., :L.in_channels].double().permute(0, 3, 1, 2)
    got_d = da_d[..., :L.in_channels].double().permute(0, 3, 1, 2)
    scale = ref.abs().max().item()
    e_w, e_d = (got_w - ref).abs().max().item() / scale, (got_d - ref).abs().max().item() / scale
    print(f"[adjoint wino] rel err wino {e_w:.2e}, direct {e_d:.2e}")
    assert e_w < 4e-3 and e_w <= 4 * e_d + 1e-4, (e_w, e_d)
    if L.cin_p > L.in_channels:  # padded input channels: zero adjoint rows
        assert da_w[..., L.in_channels:].abs().max().item() == 0.0


def _adjoint_layer(cuda):
    from image_compression_2_amd.networks_stylegan3 import SynthesisLayer
    torch.manual_seed(0)
    return SynthesisLayer(w_dim=512, is_torgb=False, is_critically_sampled=False, use_fp16=False, in_channels=250,
                          out_channels=320, in_size=50, out_size=50, in_sampling_rate=16, out_sampling_rate=16,
                          in_cutoff=8, out_cutoff=8, in_half_width=4, out_half_width=4).to(cuda)


def test_wino_dgrad_overflows_at_the_direct_gemms_scale(cuda):
    """V = B^T dc is formed with f16 adds, so opposite-sign dc values above 2^15 overflow inside the
    Winograd kernel where the direct implicit GEMM (f16 products, f32 sums) would not.  dL/da -- a sum over 9 * cout
    products, stored f16 IEEE -- overflows first: scaling a gradient by 2^k (the loss scaler's doublings), both dgrads
    turn non-finite at the same k, so the Winograd dgrad costs the GradScaler no headroom.  Up to that k they agree
    (the Winograd bound of test_wino_adjoint_dgrad_matches_fp64)."""
    from image_compression_2_amd import autograd_ops as ao
    L = _adjoint_layer(cuda)
    n, conv = 2, 52
    g = torch.Generator(device=cuda).manual_seed(5)
    dc0 = torch.zeros(n, conv, conv, L.cout_p, device=cuda)
    dc0[..., :L.out_channels] = torch.randn(n, conv, conv, L.out_channels, device=cuda, generator=g)
    first = {}
    for k in range(0, 15):
        dc = (dc0 * 2.0 ** k).to(torch.float16)
        assert torch.isfinite(dc).all()
        with torch.no_grad():
            dd = ao.conv_nhwc(dc, L.packed_adjoint(torch.float16), None, L.in_channels, 3, 0, grad=True)
            dw = ao.conv_nhwc(dc, L.packed_adjoint(torch.float16), None, L.in_channels, 3, 0, grad=True,
                              wino=L.packed_adjoint_wino)
        torch.cuda.synchronize()
        for tag, d in (("direct", dd), ("wino", dw)):
            if tag not in first and not torch.isfinite(d).all():
                first[tag] = k
        if "direct" not in first:
            ref = dd[..., :L.in_channels].double()
            err = (dw[..., :L.in_channels].double() - ref).abs().max().item() / ref.abs().max().item()
            assert err < 4e-3, (k, err)
        if len(first) == 2:
            break
    print(f"[wino dgrad] first non-finite scale 2^k: {first}")
    assert "direct" in first and first.get("wino") == first["direct"], first


def test_synth_layer_dgrad_overflow_reaches_the_scaler_as_inf(cuda):
    """The training path's layer backward (_synth_layer_grads: Winograd dgrad, f16 output converted IEEE) is linear in the upstream gradient up to the f16 limit of dL/da: scaled by 2^k so that max|dL/da| lies in
    [2^15, 2^16) it equals 2^k times the unscaled result (power-of-two scaling is exact away from f16 subnormals: rtol
    1e-3), and scaled 4x further it overflows to inf -- not to a saturated +-65504, which a GradScaler would take for a
    clean step (the gradient convs' IC2_F16_IEEE output; activations keep saturating)."""
    from image_compression_2_amd import autograd_ops as ao
    L = _adjoint_layer(cuda)
    n, conv, s_out = 2, 52, 50
    assert nv.wino_preferred(nv.F16, n, conv, conv, L.cout_p, L.cin_p, 3, 3, 0)
    g = torch.Generator(device=cuda).manual_seed(6)
    y = torch.zeros(n, conv, conv, L.cout_p, device=cuda, dtype=torch.float16)
    y[..., :L.out_channels] = (torch.randn(n, conv, conv, L.out_channels, device=cuda, generator=g) * 2).to(torch.float16)
    dout = torch.zeros(n, s_out, s_out, L.cout_p, device=cuda, dtype=torch.float16)
    dout[..., :L.out_channels] = (torch.randn(n, s_out, s_out, L.out_channels, device=cuda, generator=g) * 1e-3).to(
        torch.float16)
    os_ = (torch.rand(n, L.cout_p, device=cuda, generator=g) + 0.5).contiguous()

    def grads(k):
        with torch.no_grad():
            return ao._synth_layer_grads(L, torch.float16, os_, y, (dout.float() * 2.0 ** k).to(torch.float16))
    da1, dos1 = grads(0)
    torch.cuda.synchronize()
    m1 = da1[..., :L.in_channels].float().abs().max().item()
    assert torch.isfinite(da1).all() and 0 < m1 < 2 ** 14
    k = int(np.floor(np.log2(65000 / m1)))
    dak, dosk = grads(k)
    dak2, _ = grads(k + 2)
    torch.cuda.synchronize()
    assert 2 ** 15 <= m1 * 2 ** k < 2 ** 16
    assert torch.isfinite(dak).all() and torch.isfinite(dosk).all()
    a1, ak = da1[..., :L.in_channels].float() * 2 ** k, dak[..., :L.in_channels].float()
    assert torch.allclose(ak, a1, rtol=1e-3, atol=1e-3 * a1.abs().max().item()), (ak - a1).abs().max().item()
    assert torch.allclose(dosk, dos1 * 2 ** k, rtol=1e-3, atol=1e-3 * (dos1 * 2 ** k).abs().max().item())
    assert torch.isinf(dak2).any()   # a saturating store never produces inf
