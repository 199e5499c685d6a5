"""The default launch plan picks only instances that a parity check here has run.

The benched workloads (bench.py C2 / C2g / C4, --precision bf16, bf16-all and f16) are run once with bench.CallTimer
recording every conv call; ic2_conv_plan (the dispatcher's own plan function) names the kernel instance of each.
For every distinct instance one of its own geometries (the batch reduced while the plan keeps the instance) is run
under the default plan and compared with the library's exact-fp32 MFMA conv (v_mfma_f32_16x16x4_f32, pinned to fp64
by test_gpu_kernels.py::test_conv_igemm[float32]) on the same bf16 (f16) operands: the two differ only in f32 summation
order.  Reference: the convs of HVAE_VGG_Encoder (stylegan3_hvae_full.py:62,175-176) and SG3 modulated_conv2d.
"""
import pytest
import torch

import bench
import image_compression_2_amd as ic2
from image_compression_2_amd import _native as nv

pytestmark = pytest.mark.gpu


def _record(cuda, res, gen_res, batch, enc_prec, gen_prec="bf16"):
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision=enc_prec).to(cuda).eval().requires_grad_(False)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=gen_res, precision=gen_prec).to(cuda).eval().requires_grad_(False)
    comp = ic2.StyleGAN3Compressor(enc, G)
    x = torch.rand(batch, 3, res, res, generator=torch.Generator().manual_seed(3)).to(cuda) * 2 - 1
    timer = bench.CallTimer(nv, bench.CONV_ENTRIES)
    timer.install()
    timer.enabled = True
    try:
        with torch.no_grad():
            comp.decompress(comp.compress(x))
    finally:
        timer.enabled = False
        timer.uninstall()
    return [(n, a) for n, a, _, _ in timer.calls(bench.CONV_ENTRIES)]


def _geometry(name, a):
    if name == "ic2_conv_igemm_ws":
        dt, odt, n, h, w, cin_p, cout_p, cv, kh, kw, pad = a[3:14]
        return dict(dt=dt, odt=odt, layout=a[23], n=n, h=h, w=w, cin_p=cin_p, cout_p=cout_p, cv=cv, kh=kh, kw=kw,
                    pad=pad)
    if name == "ic2_conv3x3_gn_fwd":
        n, h, w, cin_p, cout_p, cv, kh, kw, pad = a[4:13]
        odt = nv.F32 if a[3] == nv.BF16X3 else a[3]   # the split-bf16 conv writes f32
        return dict(dt=a[3], odt=odt, layout=nv.NHWC, n=n, h=h, w=w, cin_p=cin_p, cout_p=cout_p, cv=cv, kh=kh, kw=kw,
                    pad=pad)
    return None   # from_rgb: its own kernels, test_gpu_kernels.py / test_gpu_split.py


def _plan(g, n=None):
    return nv.conv_plan(g["dt"], g["odt"], g["layout"], n or g["n"], g["h"], g["w"], g["cin_p"], g["cout_p"], g["cv"],
                        g["kh"], g["kw"], g["pad"])


@pytest.fixture(scope="module")
def default_plan_instances(cuda):
    inst = {}
    for res, gen_res, batch in ((256, 256, 32), (1024, 1024, 8)):
        for enc_prec, gen_prec in (("bf16x3", "bf16"), ("bf16", "bf16"), ("bf16x3", "f16")):
            if res == 1024 and enc_prec == "bf16":
                continue
            for name, a in _record(cuda, res, gen_res, batch, enc_prec, gen_prec):
                g = _geometry(name, a)
                if g is None:
                    continue
                p = _plan(g)
                m = g["n"] * g["h"] * g["w"]
                if p not in inst or m < inst[p]["n"] * inst[p]["h"] * inst[p]["w"]:
                    inst[p] = g
    return inst


def test_default_plan_instances_listed(default_plan_instances):
    names = sorted(default_plan_instances)
    print("[plan] instances on the benched workloads:", names)
    assert "igemm8_og2" in names and any(n.startswith("hg4_") for n in names)
    assert "igemm8_og2_f16" in names and "torgb_f16" in names  # the synthesis's f16 mode


def _run_split(g, n, cuda):
    """A split-bf16 geometry (dtype IC2_BF16X3: input stored [hi | lo], K over [hi | hi | lo]): the conv of the [hi | lo]
    tensor equals, bit for bit, the plain bf16 conv of the same data tripled to [hi | hi | lo] (the round-3 storage,
    and the tripled conv agrees with the exact-fp32 conv of the same operands -> (max|diff|, max|err vs fp32|, tol)."""
    gen = torch.Generator().manual_seed(n * 7 + g["cin_p"])
    c = g["cin_p"] // 3
    ho, wo = g["h"] + 2 * g["pad"] - g["kh"] + 1, g["w"] + 2 * g["pad"] - g["kw"] + 1
    x2 = torch.randn(n, g["h"], g["w"], 2 * c, generator=gen).to(torch.bfloat16)
    x3 = torch.cat([x2[..., :c], x2[..., :c], x2[..., c:]], -1).contiguous()
    w = (torch.randn(g["cout_p"], g["kh"], g["kw"], g["cin_p"], generator=gen) / (g["kh"] * g["kw"] * c) ** 0.5)
    w = w.to(torch.bfloat16).to(cuda)
    bias = (torch.randn(g["cout_p"], generator=gen) * 0.1).to(cuda)
    outs = []
    for dt, x in ((nv.BF16X3, x2), (nv.BF16, x3), (nv.F32, x3.float())):
        xd = x.to(cuda)
        wd = w.float() if dt == nv.F32 else w
        y = torch.empty(n, ho, wo, g["cout_p"], dtype=torch.float32, device=cuda)
        nv.conv_igemm(nv.ptr(xd), nv.ptr(wd), nv.ptr(y), dt, nv.F32, n, g["h"], g["w"], g["cin_p"], g["cout_p"], g["cv"],
                      g["kh"], g["kw"], g["pad"], ho, wo, None, nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC,
                      nv.stream_of(xd), cuda)
        torch.cuda.synchronize()
        outs.append(y[..., :g["cv"]].cpu())
    tol = 1e-4 * (1 + outs[2].abs().max().item())
    return (outs[0] - outs[1]).abs().max().item(), (outs[1] - outs[2]).abs().max().item(), tol


def _run_conv(g, n, cuda, dt_in):
    gen = torch.Generator().manual_seed(n * 7 + g["cin_p"])
    ho, wo = g["h"] + 2 * g["pad"] - g["kh"] + 1, g["w"] + 2 * g["pad"] - g["kw"] + 1
    op = torch.float16 if dt_in == nv.F16 else torch.bfloat16
    x = (torch.randn(n, g["h"], g["w"], g["cin_p"], generator=gen)).to(op)
    w = (torch.randn(g["cout_p"], g["kh"], g["kw"], g["cin_p"], generator=gen) /
         (g["kh"] * g["kw"] * g["cin_p"]) ** 0.5).to(op)
    w[g["cv"]:] = 0
    bias = torch.randn(g["cout_p"], generator=gen) * 0.1
    outs = []
    for dt, odt, layout in ((dt_in, g["odt"], g["layout"]), (nv.F32, nv.F32, nv.NHWC)):
        tdt = op if dt == dt_in else torch.float32
        xd, wd, bd = x.to(tdt).to(cuda), w.to(tdt).to(cuda), bias.to(cuda)
        if layout == nv.NCHW:
            y = torch.empty(n, g["cv"], ho, wo, dtype=torch.float32, device=cuda)
        elif layout == nv.NHWC16:
            y = torch.empty(n, g["cout_p"] // 16, ho, wo, 16, dtype=torch.float16 if odt == nv.F16 else torch.bfloat16,
                            device=cuda)
        else:
            y = torch.empty(n, ho, wo, g["cout_p"], dtype={nv.F32: torch.float32, nv.BF16: torch.bfloat16,
                                                           nv.F16: torch.float16}[odt], device=cuda)
        nv.conv_igemm(nv.ptr(xd), nv.ptr(wd), nv.ptr(y), dt, odt, n, g["h"], g["w"], g["cin_p"], g["cout_p"], g["cv"],
                      g["kh"], g["kw"], g["pad"], ho, wo, None, nv.ptr(bd), 0, 0.0, 1.0, -1.0, 1.0, layout, nv.stream_of(xd),
                      cuda)
        torch.cuda.synchronize()
        if layout == nv.NCHW:
            y = y.permute(0, 2, 3, 1)
        elif layout == nv.NHWC16:
            y = y.permute(0, 2, 3, 1, 4).reshape(n, ho, wo, g["cout_p"])
        outs.append(y[..., :g["cv"]].float().cpu())
    return outs


def test_every_default_plan_instance_matches_fp32(cuda, default_plan_instances):
    for p, g in sorted(default_plan_instances.items()):
        n = 1
        while _plan(g, n) != p and n < g["n"]:
            n += 1
        assert _plan(g, n) == p
        if g["dt"] == nv.BF16X3:
            d, err, tol = _run_split(g, n, cuda)
            print(f"[plan] {p} (split-bf16 input): n={n} {g['h']}x{g['w']} {g['cin_p']}->{g['cout_p']} "
                  f"[hi | lo] vs tripled max|diff| {d:.2e}, vs fp32 {err:.2e}")
            assert d == 0.0 and err < tol, p
            continue
        got, ref = _run_conv(g, n, cuda, g["dt"])
        # f32 summation-order noise, plus one rounding of the stored output (bf16: 2^-8, f16: 2^-11 relative)
        rel = {nv.F32: 1e-4, nv.F16: 2 ** -10, nv.BF16: 2 ** -7}[g["odt"]]
        tol = rel * (1 + ref.abs().max().item())
        err = (got - ref).abs().max().item()
        print(f"[plan] {p}: n={n} {g['h']}x{g['w']} {g['cin_p']}->{g['cout_p']} max|err| {err:.2e}")
        assert err < tol, p


def test_batch_chunking_past_2gib(cuda):
    """A batch whose input exceeds the buffer descriptors' 2 GiB (the C4 encoder's split-bf16 block-0 conv2: 8 x 1024^2
    x 192 bf16 = 3.2 GB) runs in chunks of whole images, each on the halo GEMM, and equals the per-image launches."""
    n, h, cin_p, cout_p = 8, 1024, 192, 64
    assert nv.conv_plan(nv.BF16, nv.F32, nv.NHWC, n, h, h, cin_p, cout_p, cout_p, 3, 3, 1).startswith("hg4_o64")
    gen = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(n, h, h, cin_p, generator=gen, device=cuda).to(torch.bfloat16)
    w = (torch.randn(cout_p, 3, 3, cin_p, generator=gen, device=cuda) / (9 * cin_p) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(cout_p, generator=gen, device=cuda) * 0.1
    y = torch.empty(n, h, h, cout_p, device=cuda)
    st = nv.stream_of(x)
    nv.conv_igemm(nv.ptr(x), nv.ptr(w), nv.ptr(y), nv.BF16, nv.F32, n, h, h, cin_p, cout_p, cout_p, 3, 3, 1, h, h, None,
                  nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, st, cuda)
    y1 = torch.empty(1, h, h, cout_p, device=cuda)
    for i in (0, 3, 7):
        xi = x[i:i + 1].contiguous()
        nv.conv_igemm(nv.ptr(xi), nv.ptr(w), nv.ptr(y1), nv.BF16, nv.F32, 1, h, h, cin_p, cout_p, cout_p, 3, 3, 1, h,
                      h, None, nv.ptr(bias), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, st, cuda)
        err = (y[i] - y1[0]).abs().max().item()
        assert err < 1e-4 * (1 + y1.abs().max().item()), (i, err)
    del x, y
    torch.cuda.empty_cache()
