"""GPU: the training path's backward (BASELINE C5; reference train_hvae_encoder, stylegan3_hvae_full.py:655-707)
against torch.autograd through the fp64 oracle encoder (oracle/encoder.py, pinned to the reference's own
encoder by tests/golden): every parameter gradient and the input gradient, fp32 mode at the reference's
small golden config and at the full 1024-config on 256^2; bf16 mode within a relative-norm bound; plus the
individual backward kernels against torch on random shapes."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import image_compression_2_amd as ic2
from image_compression_2_amd import _native as nv
from image_compression_2_amd import autograd_ops as ao
from oracle import encoder as oe

pytestmark = pytest.mark.gpu

SMALL = dict(img_resolution=64, img_channels=3, w_dim=32, num_ws=16, block_split=(5, 12), channel_base=256,
             channel_max=32)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _grad_check(cuda, kw, x, precision, tol, seed=7):
    torch.manual_seed(seed)
    enc = ic2.HVAE_VGG_Encoder(precision=precision, **kw).to(cuda)
    xg = x.clone().to(cuda).requires_grad_(True)
    torch.manual_seed(seed + 1)
    w, m, lv = enc(xg)
    g = torch.Generator().manual_seed(3)
    r = [torch.randn(t.shape, generator=g) for t in (w, m, lv)]
    loss = sum((t * ri.to(cuda)).sum() for t, ri in zip((w, m, lv), r))
    loss.backward()
    # oracle: same weights (fp64 leaves), the fc1 this call drew, the eps this call drew
    named = dict(enc.named_parameters())
    sd = {k: v.detach().cpu().double().requires_grad_(True) for k, v in named.items()}
    fc1 = (sd["fine_projector.fc1.weight"], sd["fine_projector.fc1.bias"])
    eps_all = ((w - m) / torch.exp(0.5 * lv)).detach().cpu().double()
    nws = kw.get("num_ws", 16)
    bs = kw.get("block_split", (5, 12))
    eps = {"global": eps_all[:, :bs[0]], "medium": eps_all[:, bs[0]:bs[1]], "fine": eps_all[:, bs[1]:nws]}
    x64 = x.double().requires_grad_(True)
    ow, om, olv = oe.encoder_forward(sd, x64, num_ws=nws, block_split=bs, w_dim=kw.get("w_dim", 512), fine_fc1=fc1,
                                     eps=eps)
    oloss = sum((t * ri.double()).sum() for t, ri in zip((ow, om, olv), r))
    oloss.backward()
    pairs = {k: (p.grad, sd[k].grad) for k, p in named.items() if sd[k].grad is not None}
    for k, p in named.items():
        if sd[k].grad is None:  # blocks past the reference's 1x1 break (:129-131) take no part, in both
            assert p.grad is None, k
    pairs["x"] = (xg.grad, x64.grad)
    for k, (a, b) in pairs.items():
        assert a is not None, k
    gmax = max(b.norm().item() for _, b in pairs.values())
    worst = {}
    for k, (a, b) in pairs.items():
        a = a.detach().double().cpu()
        if b.norm().item() < 1e-8 * gmax:
            # exactly-zero true gradient (conv bias before a one-channel GroupNorm group): rounding noise only
            assert a.norm().item() < 1e-4 * gmax, k
            continue
        worst[k] = ((a - b).norm() / b.norm()).item()
    bad = {k: v for k, v in worst.items() if v > tol}
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:4]
    print(f"[train-{precision}] max relative grad error {max(worst.values()):.2e} over {len(worst)} tensors; "
          f"largest: {[(k, round(v, 4)) for k, v in top]}")
    assert not bad, bad


def test_encoder_backward_small_fp32(cuda):
    x = torch.rand(3, 3, 32, 32, generator=torch.Generator().manual_seed(8)) * 2 - 1
    _grad_check(cuda, SMALL, x, "fp32", 1e-4)


def test_encoder_backward_full_fp32(cuda):
    """HVAE_VGG_Encoder(img_resolution=1024) on 256^2 (blocks 0-7 run, 8-9 skipped as in the reference)."""
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1
    _grad_check(cuda, dict(img_resolution=1024), x, "fp32", 1e-3, seed=0)


def test_encoder_backward_full_bf16(cuda):
    """bf16 mode (activations, dy and MFMA operands in bf16; f32 accumulation and weight gradients).  The
    GroupNorm backward of the 8^2 .. 2^2 blocks (16 channels x <= 64 pixels per group) amplifies the bf16
    rounding of the pre-norm activations: measured <= 0.19 relative error there, 0.02-0.05 in the wide blocks
    (a wrong kernel shows O(1))."""
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1
    _grad_check(cuda, dict(img_resolution=1024), x, "bf16", 0.25, seed=0)


@pytest.mark.parametrize("cin,cout,size,pad,n", [(3, 32, 17, 1, 2), (32, 64, 20, 1, 3), (64, 96, 9, 1, 2),
                                                 (128, 32, 11, 2, 1), (96, 128, 13, 0, 2)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_backward_kernels(cuda, cin, cout, size, pad, n, dtype):
    """Conv2dNHWC backward (dx: the implicit GEMM on flipped / transposed weights; dW: ic2_conv_wgrad with the
    32-pixel K chunks split over workgroups; db) against torch autograd in fp64 on the same (rounded) operands."""
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn(n, cin, size, size, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(9 * cin)
    b = torch.randn(cout, generator=g)
    dy = torch.randn(n, cout, size + 2 * pad - 2, size + 2 * pad - 2, generator=g)
    cin_p, cout_p = nv.pad32(cin), nv.pad32(cout)
    xd = ao.ToNHWC.apply(x.to(cuda), dtype, cin_p).detach().requires_grad_(True)
    wd, bd = w.to(cuda).requires_grad_(True), b.to(cuda).requires_grad_(True)
    with torch.enable_grad():
        y = ao.Conv2dNHWC.apply(xd, wd, bd, pad, cout_p)
        dyd = F.pad(dy.permute(0, 2, 3, 1), (0, cout_p - cout)).to(cuda, dtype)
        y.backward(dyd)
    xr = x.to(dtype).double().requires_grad_(True)
    wr = w.to(dtype).double().requires_grad_(True) if dtype == torch.bfloat16 else w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    F.conv2d(xr, wr, br, padding=pad).backward(dy.to(dtype).double())
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    dx = xd.grad.float().cpu()[..., :cin].permute(0, 3, 1, 2)
    assert _rel(dx, xr.grad) < tol
    assert xd.grad.float()[..., cin:].abs().max().item() == 0.0 if cin < cin_p else True
    assert _rel(wd.grad, wr.grad) < tol
    assert _rel(bd.grad, br.grad) < tol


@pytest.mark.parametrize("n,c,groups,h,w,pool", [(2, 64, 32, 6, 8, True), (3, 32, 32, 9, 7, False),
                                                 (2, 128, 32, 5, 5, True), (1, 512, 32, 2, 2, True),
                                                 (2, 96, 32, 33, 17, False)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_group_norm_backward_kernel(cuda, n, c, groups, h, w, pool, dtype):
    g = torch.Generator().manual_seed(c + h)
    y = torch.randn(n, c, h, w, generator=g) * 2 + 0.3
    gam = torch.rand(c, generator=g) + 0.5
    bet = torch.randn(c, generator=g) * 0.3
    c_p = nv.pad32(c)
    yd = ao.ToNHWC.apply(y.to(cuda), dtype, c_p).detach().requires_grad_(True)
    gd, bd = gam.to(cuda).requires_grad_(True), bet.to(cuda).requires_grad_(True)
    with torch.enable_grad():
        out = ao.GroupNormLReluPoolNHWC.apply(yd, gd, bd, groups, 1e-5, 0.2, pool, c, dtype)
        dout = torch.randn(out.shape[0], out.shape[1], out.shape[2], c, generator=g)
        out.backward(F.pad(dout, (0, c_p - c)).to(cuda, dtype))
    yr = y.to(dtype).double().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    o = F.leaky_relu(F.group_norm(yr, groups, gr, br, 1e-5), 0.2)
    if pool:
        o = F.avg_pool2d(o, 2, 2)
    o.backward(dout.to(dtype).double().permute(0, 3, 1, 2))
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(yd.grad.float().cpu()[..., :c].permute(0, 3, 1, 2), yr.grad) < tol
    assert _rel(gd.grad, gr.grad) < tol and _rel(bd.grad, br.grad) < tol
