"""The encoder's split-bf16 mode (precision='bf16x3', ic2ops.h IC2_BF16X3), op by op against fp64.

Each f32 operand v is carried as hi = bf16(v), lo = bf16(v - hi); a conv accumulates x_hi*w_hi + x_hi*w_lo + x_lo*w_hi
in f32 on bf16 MFMAs (the tripled-K GEMM), so a product is exact to ~2^-16 relative.  Reference functions:
VGGBlock.forward / HVAE_VGG_Encoder.forward, stylegan3_hvae_full.py:105-191.  The end-to-end bar (8-bit indices of
the fp32 reference) is tests/test_gpu_c2_parity.py and test_gpu_path.py::test_encoder_full_config_matches_reference.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from image_compression_2_amd import _native as nv
from image_compression_2_amd import stylegan3_hvae_full as shf

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _inference():
    with torch.no_grad():
        yield


def _split_pack(x, cuda):
    """NCHW f32 -> split-bf16 NHWC activation handle (ic2_nchw_to_nhwc, dtype IC2_BF16X3)."""
    n, c, h, w = x.shape
    c_p = nv.pad32(c)
    xd = x.to(cuda).contiguous()
    t = torch.empty([n, h, w, 2 * c_p], dtype=torch.bfloat16, device=cuda)
    nv.call("ic2_nchw_to_nhwc", nv.ptr(xd), nv.ptr(t), nv.BF16X3, n, c, h, w, c_p, None, nv.stream_of(xd))
    torch.cuda.synchronize()
    return shf._Act(t, c, x3=True)


def _unsplit(a):
    """split activation -> NCHW f32 (hi + lo) of its c logical channels ([hi | lo] layout, 2 * c_p channels)."""
    t = a.t.float().cpu()
    cp = a.c_p
    assert t.shape[-1] == 2 * cp
    hi, lo = t[..., :cp], t[..., cp:]
    return (hi.double() + lo.double())[..., :a.c].permute(0, 3, 1, 2)


def test_split_packing_is_hi_lo(cuda):
    x = torch.randn(2, 5, 7, 9, generator=torch.Generator().manual_seed(1)) * 3
    a = _split_pack(x, cuda)
    t = a.t.float().cpu()
    hi = x.to(torch.bfloat16).float().permute(0, 2, 3, 1)
    lo = (x - x.to(torch.bfloat16).float()).to(torch.bfloat16).float().permute(0, 2, 3, 1)
    assert t.shape[-1] == 64 and torch.equal(t[..., :5], hi) and torch.equal(t[..., 32:37], lo)
    assert (t[..., 5:32] == 0).all() and (t[..., 37:] == 0).all()
    assert (_unsplit(a) - x.double()).abs().max().item() <= 2 ** -16 * x.abs().max().item()


def test_split_weight_packing(cuda):
    conv = torch.nn.Conv2d(40, 20, 3, padding=1)
    a = shf._Act(torch.zeros(1, 4, 4, 2 * 64, dtype=torch.bfloat16, device=cuda), 40, x3=True)
    wp, bp = shf._packed(conv.to(cuda), a, torch.bfloat16, {}, nv.stream_of())
    torch.cuda.synchronize()
    assert wp.shape == (32, 3, 3, 192)
    w = conv.weight.detach().cpu().permute(0, 2, 3, 1)  # [o][ky][kx][i]
    hi = w.to(torch.bfloat16).float()
    lo = (w - hi).to(torch.bfloat16).float()
    got = wp.float().cpu()
    assert torch.equal(got[:20, ..., :40], hi) and torch.equal(got[:20, ..., 64:104], lo)
    assert torch.equal(got[:20, ..., 128:168], hi)
    assert (got[20:] == 0).all() and (got[..., 40:64] == 0).all()


# shapes reaching the launch plan's kernels at the tripled channel strides: hg4 (<= 256 in), the 8-phase
# kernels (384 / 768 / 1536 in), the small-grid igemm with split-K (the 16^2 .. 2^2 encoder blocks)
SPLIT_CONV_CASES = [(32, 64, 2, 150), (64, 64, 2, 129), (64, 128, 4, 64), (128, 128, 4, 64), (128, 256, 8, 32),
                    (256, 512, 8, 16), (512, 512, 8, 8), (512, 512, 16, 2), (40, 20, 2, 33)]


@pytest.mark.parametrize("cin,cout,n,size", SPLIT_CONV_CASES)
def test_split_conv_gn_matches_fp64(cuda, cin, cout, n, size):
    """_conv_gn in split mode: the f32 conv output within 2e-5 (relative to max |y|) of F.conv2d in fp64 on the
    unrounded f32 operands (a plain bf16 conv: ~1e-2), and the GroupNorm statistics of that output."""
    g = torch.Generator().manual_seed(cin * 7 + cout + size)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    norm = torch.nn.GroupNorm(min(32, cout), cout)
    x = torch.randn(n, cin, size, size, generator=g)
    a = _split_pack(x, cuda)
    y, st = shf._conv_gn(conv.to(cuda), norm.to(cuda), a, torch.bfloat16, {}, nv.stream_of())
    torch.cuda.synchronize()
    assert y.t.dtype == torch.float32 and not y.x3
    r = F.conv2d(x.double(), conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(), padding=1)
    got = y.t[..., :cout].cpu().double().permute(0, 3, 1, 2)
    err = (got - r).abs().max().item() / r.abs().max().item()
    print(f"[split conv {cin}->{cout} n{n} {size}^2] max rel err {err:.2e}")
    assert err < 2e-5
    assert (y.t[..., cout:] == 0).all()
    groups = norm.num_groups
    rg = r.reshape(n, groups, -1)
    mean, var = rg.mean(-1), rg.var(-1, unbiased=False)
    s = st[: n * groups * 2].view(n, groups, 2).cpu().double()
    assert torch.allclose(s[..., 0], mean, rtol=1e-4, atol=1e-5 * r.abs().max().item())
    assert torch.allclose(s[..., 1], 1 / torch.sqrt(var + 1e-5), rtol=1e-4)


@pytest.mark.parametrize("cin,cout,n,h,w", [(32, 64, 8, 126, 124), (64, 128, 8, 128, 128), (64, 128, 8, 126, 124),
                                             (64, 64, 8, 1024, 1024)])
def test_split_conv_gn_fused_epilogue(cuda, cin, cout, n, h, w):
    """64- / 128-wide split convs on the 4-wave halo GEMM take the GroupNorm statistics from its epilogue
    (ic2_conv3x3_gn_fwd, IC2_BF16X3): the same f32 output bits as the unfused call, statistics within 1e-6 of the
    separate pass and of fp64 on ragged 8 x 32 tiles (126 x 124: partial rows and columns masked out) and on the C4
    block-0 conv2 shape, whose 3.2 GB input runs as two launches of 4 images."""
    g = torch.Generator().manual_seed(cin + cout + h)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1 + 0.05)
    norm = torch.nn.GroupNorm(32, cout)
    x = torch.randn(n, cin, h, w, generator=torch.Generator(device=cuda).manual_seed(h), device=cuda)
    a = _split_pack(x, cuda)
    del x
    assert nv.query("ic2_conv3x3_gn_fuses", nv.BF16X3, n, h, w, a.k_p, cout, cout, 3, 3, 1, 32, -1) == 1
    assert nv.query("ic2_conv3x3_gn_fuses", nv.BF16X3, n, h, w, a.k_p, cout, cout, 3, 3, 1, 32, 0) == 0
    conv, norm = conv.to(cuda), norm.to(cuda)
    yf, sf = shf._conv_gn(conv, norm, a, torch.bfloat16, {}, nv.stream_of(), fuse=-1)
    yu, su = shf._conv_gn(conv, norm, a, torch.bfloat16, {}, nv.stream_of(), fuse=0)
    torch.cuda.synchronize()
    assert torch.equal(yf.t, yu.t)
    del yf
    k = n * 32 * 2
    sfd, sud = sf[:k].view(n, 32, 2).double(), su[:k].view(n, 32, 2).double()
    mean = torch.empty(n, 32, dtype=torch.float64, device=cuda)
    var = torch.empty_like(mean)
    for i in range(n):  # fp64 statistics of the f32 output, one image at a time
        r = yu.t[i, ..., :cout].double().reshape(-1, 32, cout // 32).transpose(0, 1).reshape(32, -1)
        mean[i], var[i] = r.mean(-1), r.var(-1, unbiased=False)
    rstd = 1 / torch.sqrt(var + norm.eps)
    scale = yu.t.abs().max().item()
    d_mean = max((sfd[..., 0] - sud[..., 0]).abs().max().item(), (sfd[..., 0] - mean).abs().max().item()) / scale
    d_rstd = max(((sfd[..., 1] - sud[..., 1]) / sud[..., 1]).abs().max().item(),
                 ((sfd[..., 1] - rstd) / rstd).abs().max().item())
    print(f"[split conv+GN fused {cin}->{cout} n{n} {h}x{w}] mean {d_mean:.2e} (of max|y|) rstd {d_rstd:.2e} rel")
    assert d_mean < 1e-6 and d_rstd < 1e-6


@pytest.mark.parametrize("pool", [False, True])
def test_split_gn_lrelu_pool(cuda, pool):
    """GroupNorm + lrelu (+ pool) in f32, stored split: hi + lo within 2^-16 (relative) of the fp64 result (the split
    keeps 16 significant bits: residual <= 2^-17 |v|; f32 statistics add ~1e-6)."""
    g = torch.Generator().manual_seed(3)
    n, c, h, w = 3, 96, 18, 14
    y = torch.randn(n, c, h, w, generator=g) * 2 + 0.3
    norm = torch.nn.GroupNorm(32, c)
    with torch.no_grad():
        norm.weight.copy_(torch.rand(c, generator=g) + 0.5)
        norm.bias.copy_(torch.randn(c, generator=g))
    stream = nv.stream_of()
    ya = shf._to_nhwc(y.to(cuda), torch.float32, stream)
    out = shf._group_norm_lrelu(norm.to(cuda), ya, pool, torch.bfloat16, stream, split=True)
    assert out.x3 and out.t.shape[-1] == 2 * 96
    r = F.leaky_relu(F.group_norm(y.double(), 32, norm.weight.detach().cpu().double(),
                                  norm.bias.detach().cpu().double(), 1e-5), 0.2)
    if pool:
        r = F.avg_pool2d(r, 2)
    got = _unsplit(out)
    assert (got - r).abs().max().item() < 2 ** -16 * (1 + r.abs().max().item())


@pytest.mark.parametrize("cin,cout,n,h,w", [(3, 32, 3, 67, 45), (3, 64, 2, 40, 33), (1, 32, 1, 9, 70), (3, 128, 2, 33, 40),
                                             (3, 20, 2, 16, 32)])
def test_from_rgb_split_exact(cuda, cin, cout, n, h, w):
    """ic2_from_rgb_conv_x3: exact f32 FMAs on the unrounded image, stored split -> within 2^-16 (relative) of fp64."""
    g = torch.Generator().manual_seed(cin * 100 + cout + h)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    x = torch.rand(n, cin, h, w, generator=g) * 2 - 1
    a = shf._from_rgb(conv.to(cuda), x.to(cuda), torch.bfloat16, {}, nv.stream_of(), split=True)
    torch.cuda.synchronize()
    assert a.x3 and a.c == cout
    r = F.conv2d(x.double(), conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(), padding=1)
    got = _unsplit(a)
    assert (got - r).abs().max().item() < 2 ** -16 * (1 + r.abs().max().item())


def test_from_rgb_split_generic_route(cuda):
    """from_rgb shapes without the direct kernel (5x5 here) take an exact f32 conv + split packing."""
    g = torch.Generator().manual_seed(9)
    conv = torch.nn.Conv2d(3, 32, 5, padding=2)
    x = torch.rand(2, 3, 21, 19, generator=g) * 2 - 1
    a = shf._from_rgb(conv.to(cuda), x.to(cuda), torch.bfloat16, {}, nv.stream_of(), split=True)
    r = F.conv2d(x.double(), conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(), padding=2)
    assert (_unsplit(a) - r).abs().max().item() < 2 ** -16 * (1 + r.abs().max().item())


def test_split_global_avg_pool(cuda):
    x = torch.randn(3, 40, 9, 11, generator=torch.Generator().manual_seed(2)) * 2
    a = _split_pack(x, cuda)
    got = shf._gap(a, nv.stream_of()).cpu().double()
    r = x.double().mean((2, 3))
    assert (got - r).abs().max().item() < 1e-5


# ------------------------------------------------------------------------------------------------
# The split-weight f16 mode of the encoder's first blocks (ic2ops.h IC2_F16X2): f16 activation x, f16 weights
# w_hi + w_lo, K over [x | x] -> x * w to the f32 accumulation's precision for the f16-rounded x.
def _h2_pack(x, cuda):
    """NCHW f32 -> f16 NHWC activation handle for a split-weight conv (ic2_nchw_to_nhwc, dtype IC2_F16)."""
    n, c, h, w = x.shape
    c_p = nv.pad32(c)
    xd = x.to(cuda).contiguous()
    t = torch.empty([n, h, w, c_p], dtype=torch.float16, device=cuda)
    nv.call("ic2_nchw_to_nhwc", nv.ptr(xd), nv.ptr(t), nv.F16, n, c, h, w, c_p, None, nv.stream_of(xd))
    torch.cuda.synchronize()
    return shf._Act(t, c, h2=True)


def test_f16x2_weight_packing(cuda):
    conv = torch.nn.Conv2d(40, 20, 3, padding=1)
    a = shf._Act(torch.zeros(1, 4, 4, 64, dtype=torch.float16, device=cuda), 40, h2=True)
    assert a.k_p == 128 and a.code == nv.F16X2
    cache = {}
    wp, bp = shf._packed(conv.to(cuda), a, torch.bfloat16, cache, nv.stream_of())
    mul = shf._out_mul(conv, cache)
    torch.cuda.synchronize()
    assert wp.shape == (32, 3, 3, 128) and wp.dtype == torch.float16
    # packed times 2^s = 1 / mul with max |w| 2^s in [2^12, 2^13); the bias likewise
    w = conv.weight.detach().cpu().permute(0, 2, 3, 1) / mul  # [o][ky][kx][i]
    assert 2 ** 12 <= w.abs().max().item() < 2 ** 13 and mul == 2.0 ** round(np.log2(mul))
    hi = w.to(torch.float16).float()
    lo = (w - hi).to(torch.float16).float()
    got = wp.float().cpu()
    assert torch.equal(got[:20, ..., :40], hi) and torch.equal(got[:20, ..., 64:104], lo)
    assert (got[20:] == 0).all() and (got[..., 40:64] == 0).all() and (got[..., 104:] == 0).all()
    assert torch.equal(bp[:20].cpu(), conv.bias.detach().cpu() / mul)


# hg4 (the fused-statistics instances and the plain ones), the generic 16-bit igemm with an odd count of stored
# 32-channel blocks (the 8-phase kernels need an even one), the 8-phase kernels, small grids with split-K; the
# last case scales the weights by 1e-3 (unscaled, w_hi itself would be an f16 subnormal: the packing's 2^s keeps it
# normal)
F16X2_CONV_CASES = [(32, 64, 2, 150, 1.0), (64, 64, 2, 129, 1.0), (64, 128, 4, 64, 1.0), (128, 128, 4, 64, 1.0),
                    (128, 256, 8, 32, 1.0), (256, 512, 8, 16, 1.0), (40, 20, 2, 33, 1.0), (32, 64, 1, 20, 1.0),
                    (64, 64, 2, 96, 1e-3)]


@pytest.mark.parametrize("cin,cout,n,size,wscale", F16X2_CONV_CASES)
def test_f16x2_conv_gn_matches_fp64(cuda, cin, cout, n, size, wscale):
    """_conv_gn on an f16 activation (IC2_F16X2): the f16 output within its rounding (2^-11 relative) plus 1e-5 of
    max |y| of F.conv2d in fp64 on the f16-rounded activation and the unrounded weights (the weight split carries ~22
    bits; before the output rounding the conv is within 1e-5), and the GroupNorm statistics of that output."""
    g = torch.Generator().manual_seed(cin * 5 + cout + size)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin) * wscale)
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1 * wscale)
    norm = torch.nn.GroupNorm(min(32, cout), cout)
    x = torch.randn(n, cin, size, size, generator=g)
    a = _h2_pack(x, cuda)
    plan = nv.conv_plan(nv.F16X2, nv.F32, nv.NHWC, n, size, size, a.k_p, nv.pad32(cout), cout, 3, 3, 1)
    y, st = shf._conv_gn(conv.to(cuda), norm.to(cuda), a, torch.bfloat16, {}, nv.stream_of())
    torch.cuda.synchronize()
    assert y.t.dtype == torch.float16 and not y.split
    r = F.conv2d(x.to(torch.float16).double(), conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(),
                 padding=1)
    got = y.t[..., :cout].cpu().double().permute(0, 3, 1, 2)
    ex = ((got - r).abs() - 2 ** -11 * r.abs()).max().item() / r.abs().max().item()
    print(f"[f16x2 conv {cin}->{cout} n{n} {size}^2 w*{wscale:g} plan {plan}] max err beyond f16 rounding {ex:.2e}")
    assert ex < 1e-5
    assert (y.t[..., cout:] == 0).all()
    groups = norm.num_groups
    rg = r.reshape(n, groups, -1)
    mean, var = rg.mean(-1), rg.var(-1, unbiased=False)
    s = st[: n * groups * 2].view(n, groups, 2).cpu().double()
    assert torch.allclose(s[..., 0], mean, rtol=1e-4, atol=1e-4 * r.abs().max().item())
    assert torch.allclose(s[..., 1], 1 / torch.sqrt(var + 1e-5), rtol=2e-4)


@pytest.mark.parametrize("cin,cout,n,h,w", [(32, 64, 8, 126, 124), (64, 128, 8, 126, 124), (64, 64, 8, 1024, 1024),
                                             (64, 128, 8, 512, 512)])
def test_f16x2_conv_gn_fused_epilogue(cuda, cin, cout, n, h, w):
    """The f16 instances of the statistics-epilogue halo GEMMs (hg4_*_gn_kernel_f16, tap-major hi / lo pairs): the
    unfused call's f16 output to an ulp, fp64 on a corner, statistics (of the stored f16 values) within 1e-5 of the
    separate pass, on ragged tiles and on the C4 block-0 / block-1 conv2 shapes."""
    g = torch.Generator().manual_seed(cin + cout + h + 1)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1 + 0.05)
    norm = torch.nn.GroupNorm(32, cout)
    x = torch.randn(n, cin, h, w, generator=torch.Generator(device=cuda).manual_seed(h), device=cuda)
    a = _h2_pack(x, cuda)
    del x
    assert nv.query("ic2_conv3x3_gn_fuses", nv.F16X2, n, h, w, a.k_p, cout, cout, 3, 3, 1, 32, -1) == 1
    assert nv.query("ic2_conv3x3_gn_fuses", nv.F16X2, n, h, w, a.k_p, cout, cout, 3, 3, 1, 32, 0) == 0
    conv, norm = conv.to(cuda), norm.to(cuda)
    yf, sf = shf._conv_gn(conv, norm, a, torch.bfloat16, {}, nv.stream_of(), fuse=-1)
    yu, su = shf._conv_gn(conv, norm, a, torch.bfloat16, {}, nv.stream_of(), fuse=0)
    torch.cuda.synchronize()
    # the fused kernels walk each tap's hi / lo K blocks together (hg4 PAIR), the unfused ones all hi then all lo:
    # the f32 sums differ in order, so the f16 outputs agree to an ulp
    d = (yf.t.float() - yu.t.float()).abs()
    assert (d <= 2 ** -10 * yu.t.float().abs() + 1e-6).all()
    # and the fused output against fp64 on image 0's top-left 64 x 64 (windows inside the 66 x 66 crop)
    xc = a.t[0, :66, :66, :cin].permute(2, 0, 1)[None].double().cpu()
    r = F.conv2d(xc, conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(), padding=1)[..., :64, :64]
    got = yf.t[0, :64, :64, :cout].permute(2, 0, 1)[None].double().cpu()
    ex = ((got - r).abs() - 2 ** -11 * r.abs()).max().item() / r.abs().max().item()
    assert ex < 1e-5
    del yf
    k = n * 32 * 2
    sfd, sud = sf[:k].view(n, 32, 2).double(), su[:k].view(n, 32, 2).double()
    scale = yu.t.abs().max().item()
    d_mean = (sfd[..., 0] - sud[..., 0]).abs().max().item() / scale
    d_rstd = ((sfd[..., 1] - sud[..., 1]) / sud[..., 1]).abs().max().item()
    print(f"[f16x2 conv+GN fused {cin}->{cout} n{n} {h}x{w}] vs fp64 {ex:.2e}; mean {d_mean:.2e} (of max|y|) "
          f"rstd {d_rstd:.2e} rel")
    assert d_mean < 1e-5 and d_rstd < 1e-5


@pytest.mark.parametrize("pool", [False, True])
def test_f16x2_gn_lrelu_pool_f16_out(cuda, pool):
    """GroupNorm + lrelu (+ pool) in f32 from the f32 conv output, rounded once to f16 (the next split-weight conv's
    operand): within half an f16 ulp (+ the f32 statistics' ~1e-6) of the fp64 result."""
    g = torch.Generator().manual_seed(4)
    n, c, h, w = 3, 64, 18, 14
    y = torch.randn(n, c, h, w, generator=g) * 2 + 0.3
    norm = torch.nn.GroupNorm(32, c)
    with torch.no_grad():
        norm.weight.copy_(torch.rand(c, generator=g) + 0.5)
        norm.bias.copy_(torch.randn(c, generator=g))
    stream = nv.stream_of()
    ya = shf._to_nhwc(y.to(cuda), torch.float32, stream)
    out = shf._group_norm_lrelu(norm.to(cuda), ya, pool, torch.bfloat16, stream, split=True, h2=True)
    assert out.h2 and not out.x3 and out.t.dtype == torch.float16 and out.t.shape[-1] == 64
    r = F.leaky_relu(F.group_norm(y.double(), 32, norm.weight.detach().cpu().double(),
                                  norm.bias.detach().cpu().double(), 1e-5), 0.2)
    if pool:
        r = F.avg_pool2d(r, 2)
    got = out.t.float().cpu().double().permute(0, 3, 1, 2)
    assert ((got - r).abs() <= 2 ** -11 * r.abs() + 1e-5 * (1 + r.abs().max().item())).all()


@pytest.mark.parametrize("cin,cout,n,h,w", [(3, 32, 3, 67, 45), (3, 64, 2, 40, 33), (3, 20, 2, 16, 32)])
def test_from_rgb_f16_out(cuda, cin, cout, n, h, w):
    """ic2_from_rgb_conv_f16: the exact-f32 from_rgb rounded once to f16 -> within half an f16 ulp of fp64."""
    g = torch.Generator().manual_seed(cin * 10 + cout + h)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(9 * cin))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    x = torch.rand(n, cin, h, w, generator=g) * 2 - 1
    a = shf._from_rgb(conv.to(cuda), x.to(cuda), torch.bfloat16, {}, nv.stream_of(), split=True, h2=True)
    torch.cuda.synchronize()
    assert a.h2 and a.c == cout and a.t.dtype == torch.float16
    r = F.conv2d(x.double(), conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double(), padding=1)
    got = a.t[..., :cout].float().cpu().double().permute(0, 3, 1, 2)
    assert ((got - r).abs() <= 2 ** -11 * r.abs() + 1e-6).all()
    assert (a.t[..., cout:] == 0).all()


def test_split_encoder_first_blocks_run_f16x2(cuda):
    """The benched split encoder ('bf16x3') runs its first IC2_SPLIT_F16_BLOCKS = 3 blocks' convs as split-weight f16
    (the f16 statistics-epilogue kernels) and the rest as split bf16."""
    import image_compression_2_amd as ic2
    calls = []
    orig = nv.call

    def rec(name, *args):
        convs = ("ic2_conv3x3_gn_fwd", "ic2_conv3x3_gn_fwd_scaled", "ic2_conv_igemm_ws")
        if name in convs + ("ic2_from_rgb_conv_f16", "ic2_from_rgb_conv_x3"):
            calls.append((name, args[3] if name in convs else None))
        return orig(name, *args)

    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision="bf16x3").to(cuda)
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1
    nv.call = rec
    try:
        enc(x.to(cuda))
    finally:
        nv.call = orig
    assert calls[0] == ("ic2_from_rgb_conv_f16", None)
    codes = [c for n, c in calls[1:]]
    assert len(codes) == 16 and codes[:6] == [nv.F16X2] * 6 and set(codes[6:]) == {nv.BF16X3}
