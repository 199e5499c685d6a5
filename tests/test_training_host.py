"""CPU: host logic of the training path (BASELINE C5) -- the upfirdn2d adjoint padding that every synthesis
backward uses (checked against torch.autograd through the oracle's upfirdn2d in fp64), the data-parallel
gradient average over gloo with world size 2, the KL term and the step's argument checks."""
import os

import numpy as np
import pytest
import torch

from image_compression_2_amd import distributed as icd
from image_compression_2_amd import training as ict
from image_compression_2_amd.sg3_ops import upfirdn2d_adjoint_padding
from oracle import sg3


CASES = [  # (h, w, taps, up, down, padding, flip)
    (12, 12, 12, 2, 1, [7, 6, 7, 6], False),          # an SG3 layer's up-FIR (up 2, 12 taps)
    (30, 30, 12, 1, 2, 0, False),                      # its down-FIR
    (9, 11, 24, 4, 1, [13, 11, 14, 10], False),        # up 4
    (40, 36, 24, 1, 4, 0, True),
    (10, 10, 5, 2, 2, [1, 3, 2, 0], False),            # up and down at once, odd taps, asymmetric padding
    (16, 16, 6, 1, 1, [-2, 1, 0, -1], True),           # crops
    (7, 9, 1, 3, 2, [0, 1, 1, 0], False),              # 1-tap filter
]


@pytest.mark.parametrize("h,w,taps,up,down,pad,flip", CASES)
def test_upfirdn2d_adjoint_padding_matches_autograd(h, w, taps, up, down, pad, flip):
    g = torch.Generator().manual_seed(h * 31 + taps)
    f = torch.rand(taps, generator=g, dtype=torch.float64) + 0.1
    x = torch.randn(2, 3, h, w, generator=g, dtype=torch.float64, requires_grad=True)
    gain = float(up * up)
    y = sg3.upfirdn2d(x, f, up=up, down=down, padding=pad, flip_filter=flip, gain=gain)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (ref,) = torch.autograd.grad(y, x, dy)
    p = upfirdn2d_adjoint_padding(x.shape[2:], y.shape[2:], f, up, down, pad)
    got = sg3.upfirdn2d(dy, f, up=down, down=up, padding=p, flip_filter=not flip, gain=gain)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() < 1e-10 * (1 + ref.abs().max().item())


def test_filtered_lrelu_backward_chain_on_oracle_ops():
    """The chain filtered_lrelu_backward runs (recompute U, adjoint down-FIR, lrelu' * gain with the clamp
    mask, adjoint up-FIR), restated on the oracle's upfirdn2d, equals autograd of the oracle's filtered_lrelu
    for an SG3-T layer geometry (up 2, down 2, 12 taps, clamp 256 reached)."""
    _, layers = sg3.layer_table(256)
    L = layers[5]
    g = torch.Generator().manual_seed(5)
    fu, fd = L["up_filter"].double(), L["down_filter"].double()
    n, c, s = 2, 4, L["in_size"] + 2
    z = (torch.randn(n, c, s, s, generator=g, dtype=torch.float64) * 150).requires_grad_(True)
    y = sg3.filtered_lrelu(z, fu, fd, up=L["up"], down=L["down"], padding=L["padding"], clamp=256)
    dout = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (ref,) = torch.autograd.grad(y, z, dout)
    u = sg3.upfirdn2d(z.detach(), fu, up=L["up"], padding=L["padding"], gain=L["up"] ** 2)
    v = sg3.bias_act(u, act="lrelu", alpha=0.2, gain=np.sqrt(2), clamp=256)
    assert (v.abs() >= 256).any()
    m = torch.where(v > 0, np.sqrt(2), 0.2 * np.sqrt(2)) * (v.abs() < 256)
    pd = upfirdn2d_adjoint_padding(u.shape[2:], dout.shape[2:], fd, 1, L["down"], 0)
    gv = sg3.upfirdn2d(dout, fd, up=L["down"], padding=pd, flip_filter=True)
    pu = upfirdn2d_adjoint_padding(z.shape[2:], u.shape[2:], fu, L["up"], 1, L["padding"])
    got = sg3.upfirdn2d(gv * m, fu, down=L["up"], padding=pu, flip_filter=True, gain=L["up"] ** 2)
    assert (got - ref).abs().max().item() < 1e-6 * (1 + ref.abs().max().item())


def _dp_worker(outq_path):
    import torch.distributed as dist
    rank, _, _ = icd.init("gloo")
    a = torch.nn.Parameter(torch.zeros(5, 3))
    b = torch.nn.Parameter(torch.zeros(1000))
    c = torch.nn.Parameter(torch.zeros(7))   # no gradient: skipped on every rank
    a.grad = torch.full((5, 3), float(rank + 1))
    b.grad = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    nb = icd.allreduce_gradients([a, b, c], bucket_bytes=32)   # tiny buckets: one per tensor
    res = torch.cat([a.grad.reshape(-1), b.grad, torch.tensor([float(nb), float(c.grad is None)])])
    torch.save(res, f"{outq_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_gradients_gloo_world2(tmp_path):
    out = str(tmp_path / "dp")
    icd.launch(2, _dp_worker, out)
    for r in range(2):
        res = torch.load(f"{out}.{r}", weights_only=True)
        assert torch.allclose(res[:15], torch.full((15,), 1.5))
        assert torch.allclose(res[15:1015], torch.arange(1000, dtype=torch.float32) * 1.5)
        assert res[1015].item() == 2 and res[1016].item() == 1


def test_allreduce_gradients_single_process_is_noop():
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    assert icd.allreduce_gradients([p], world=1) == 0 and p.grad.tolist() == [2.0, 2.0, 2.0]


def test_kl_divergence_formula():
    g = torch.Generator().manual_seed(0)
    m, lv = torch.randn(3, 16, 8, generator=g), torch.randn(3, 16, 8, generator=g) * 0.3
    w_avg = torch.randn(1, 1, 8, generator=g)
    ref = np.mean([0.5 * float(((m[i] - w_avg[0]) ** 2 + lv[i].exp() - lv[i] - 1).sum()) for i in range(3)])
    assert abs(ict.kl_divergence(m, lv, w_avg).item() - ref) < 1e-5 * abs(ref)


def test_train_step_requires_percep_for_perceptual_weight():
    with pytest.raises(ValueError, match="perceptual"):
        ict.train_step(None, None, None, None, perceptual_weight=0.8)


def _fc1_worker(out_path):
    """A data-parallel step's fine-projector path on one rank: the reference quirk re-creates fc1 from this
    process's CPU generator (seeded differently per rank here, as unsynchronised ranks would be), the training
    step's hook broadcasts it from rank 0, each rank backpropagates its own batch slice through it and the
    gradients are averaged."""
    import torch.distributed as dist
    import image_compression_2_amd as ic2
    rank, _, _ = icd.init("gloo")
    torch.manual_seed(100 + rank)
    proj = ic2.HierarchyProjector(64, 32, 4)
    proj.fc1_hook = icd.broadcast_params
    proj.refresh_fc1(128, torch.device("cpu"))
    pooled = torch.randn(3, 128, generator=torch.Generator().manual_seed(rank))   # this rank's batch slice
    loss = torch.nn.functional.leaky_relu(proj.fc1(pooled), 0.2).square().sum()
    loss.backward()
    icd.allreduce_gradients(list(proj.fc1.parameters()))
    torch.save({"w": proj.fc1.weight.detach(), "b": proj.fc1.bias.detach(), "gw": proj.fc1.weight.grad,
                "gb": proj.fc1.bias.grad, "pooled": pooled}, f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_fine_projector_fc1_consistent_across_ranks_gloo_world2(tmp_path):
    """SURVEY 8e pitfall / VERDICT r2: the re-created fine fc1 is broadcast from rank 0, so both ranks hold the
    same weights (rank 0's draw) and the averaged gradients are identical and equal the full-batch mean."""
    out = str(tmp_path / "fc1")
    icd.launch(2, _fc1_worker, out)
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    assert torch.equal(r0["w"], r1["w"]) and torch.equal(r0["b"], r1["b"])
    import image_compression_2_amd as ic2
    torch.manual_seed(100)
    ic2.HierarchyProjector(64, 32, 4)
    ref = torch.nn.Linear(128, 256)   # rank 0's draw after its construction: the reference's nn.Linear default init
    assert torch.equal(r0["w"], ref.weight.detach()) and torch.equal(r0["b"], ref.bias.detach())
    assert torch.equal(r0["gw"], r1["gw"]) and torch.equal(r0["gb"], r1["gb"])
    w = ref.weight.detach().clone().requires_grad_(True)
    b = ref.bias.detach().clone().requires_grad_(True)
    tot = sum(torch.nn.functional.leaky_relu(torch.nn.functional.linear(r["pooled"], w, b), 0.2).square().sum()
              for r in (r0, r1)) / 2
    tot.backward()
    assert torch.allclose(r0["gw"], w.grad, rtol=1e-5, atol=1e-6) and torch.allclose(r0["gb"], b.grad, rtol=1e-5)


def test_fix_fine_projector_builds_fc1_for_the_pooled_width():
    """fix_fine_projector=True (opt-in): every weight drawn as the reference draws it, then fc1 of the fine (and any
    other mismatched) projector rebuilt once for the width it pools -- no per-call re-creation."""
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    ref = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, fix_fine_projector=True)
    sd_r, sd_f = ref.state_dict(), enc.state_dict()
    for k in sd_r:
        if not k.startswith("fine_projector.fc1"):
            assert torch.equal(sd_r[k], sd_f[k]), k
    assert enc.fine_projector.fc1.weight.shape == (256, 128) and enc.fine_projector.in_channels == 128
    assert ref.fine_projector.fc1.weight.shape == (256, 64)
    assert enc.global_projector.in_channels == 512 and enc.medium_projector.in_channels == 512


def test_derived_cache_scope():
    """autograd_ops.derived_cache: inside the block a parameter's derived data (packed weights, padded bias) is
    built once per key and reused; outside it, and for non-parameter temporaries, it is rebuilt every call (a fused
    optimizer does not bump version counters, so the cache is scoped to the training step, not versioned)."""
    from image_compression_2_amd import autograd_ops as ao
    p = torch.nn.Parameter(torch.randn(4))
    calls = []

    def make():
        calls.append(1)
        return torch.zeros(1)
    ao._derived(p, ("k",), make)
    ao._derived(p, ("k",), make)
    assert len(calls) == 2                      # no block: no caching
    with ao.derived_cache():
        a = ao._derived(p, ("k",), make)
        b = ao._derived(p, ("k",), make)
        assert a is b and len(calls) == 3       # one build per key
        ao._derived(p, ("other",), make)
        assert len(calls) == 4
        t = p.detach() * 2                      # a temporary: never cached
        ao._derived(t, ("k",), make)
        ao._derived(t, ("k",), make)
        assert len(calls) == 6
    ao._derived(p, ("k",), make)
    assert len(calls) == 7                      # the block's entries are gone


class _ToyEncoder(torch.nn.Module):
    """A parameter used twice per step (as the training step's two encoder passes use every weight), one that gets
    no gradient, and a head re-created on every forward (the reference's fc1 quirk)."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(6, 6)
        self.b = torch.nn.Linear(6, 4)
        self.unused = torch.nn.Parameter(torch.zeros(3))
        self.head = torch.nn.Linear(4, 2)

    def forward(self, x):
        self.head = torch.nn.Linear(4, 2)   # fresh every call, like refresh_fc1
        with torch.no_grad():
            self.head.weight.fill_(0.5)
            self.head.bias.fill_(0.1)
        return self.head(torch.tanh(self.b(self.a(self.a(x)))))


def _reducer_worker(out_path):
    import torch.distributed as dist
    rank, world, _ = icd.init("gloo")
    torch.manual_seed(0)   # same weights on every rank
    m = _ToyEncoder()
    r = icd.GradReducer(m, world, bucket_bytes=64)   # several buckets
    res = {}
    for step in range(2):
        x = torch.randn(5, 6, generator=torch.Generator().manual_seed(10 * step + rank))   # this rank's slice
        m.zero_grad(set_to_none=True)
        loss = m(x).square().sum() + m(x).sum()   # two passes, as the training step
        r.start()
        loss.backward()
        launched = r.next_launch
        n = r.finish()
        got = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        # the same gradients reduced after backward
        m.zero_grad(set_to_none=True)
        torch.manual_seed(0)
        loss = m(x).square().sum() + m(x).sum()
        loss.backward()
        icd.allreduce_gradients(list(m.parameters()), world)
        ref = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        res[step] = {"got": got, "ref": ref, "launched": launched, "n": n, "unused": m.unused.grad is None}
    torch.save(res, f"{out_path}.{rank}")
    r.remove()
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_overlapped_matches_post_backward_allreduce(tmp_path):
    out = str(tmp_path / "gr")
    icd.launch(2, _reducer_worker, out)
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    for step in range(2):
        for rk in range(2):
            d = res[rk][step]
            assert set(d["got"]) == set(d["ref"]) == {"a.weight", "a.bias", "b.weight", "b.bias", "head.weight",
                                                      "head.bias"}
            for k in d["ref"]:
                assert torch.allclose(d["got"][k], d["ref"][k], atol=1e-6), (step, k)
                assert torch.allclose(d["got"][k], res[0][step]["got"][k]), "ranks disagree"
            assert d["launched"] >= 1, "no bucket launched during backward"
            assert d["unused"]


class _C5Encoder(torch.nn.Module):
    """BASELINE C5's encoder (HVAE_VGG_Encoder(img_resolution=1024), ref stylegan3_hvae_full.py:34-103) with the
    oracle's torch restatement of its forward (ref :105-167) over the live parameters, so it runs on the CPU: on a 256^2
    input the 1x1 break (ref :129-131) stops before blocks 8-9, which get no gradient.  The fine projector's fc1 is
    re-created per call as the reference does (:225-230), seeded the same on every rank (broadcast in the product)."""

    def __init__(self):
        super().__init__()
        import image_compression_2_amd as ic2
        self.enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)

    def forward(self, x):
        from oracle import encoder as oe
        sd = dict(self.enc.named_parameters())
        g = torch.Generator().manual_seed(7)
        fc1 = torch.nn.Linear(128, 256)
        with torch.no_grad():
            fc1.weight.copy_(torch.randn(256, 128, generator=g) * 0.05)
            fc1.bias.zero_()
        self.enc.fine_projector.fc1 = fc1
        return oe.encoder_forward(sd, x, fine_fc1=(fc1.weight, fc1.bias))


def _c5_reducer_worker(out_path):
    import torch.distributed as dist
    rank, world, _ = icd.init("gloo")
    torch.manual_seed(0)   # same weights on every rank
    m = _C5Encoder()
    r = icd.GradReducer(m, world)   # the training step's 25 MiB buckets
    res = {}
    for step in range(3):
        x = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(10 * step + rank)) * 2 - 1
        m.zero_grad(set_to_none=True)
        w, mean, lv = m(x)
        loss = w.square().mean() + 0.01 * (mean.square() + lv.exp() - lv).mean()
        r.start()
        loss.backward()
        launched, nb = r.next_launch, len(r.buckets)
        r.finish()
        got = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        m.zero_grad(set_to_none=True)
        w, mean, lv = m(x)
        (w.square().mean() + 0.01 * (mean.square() + lv.exp() - lv).mean()).backward()
        icd.allreduce_gradients(list(m.parameters()), world)
        ref = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        res[step] = {"got": got, "ref": ref, "launched": launched, "nb": nb}
    unused = [k for k, p in m.named_parameters() if p.grad is None]
    torch.save({"steps": res, "unused": unused, "n_buckets": len(r.buckets)}, f"{out_path}.{rank}")
    r.remove()
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_overlaps_at_c5_config(tmp_path):
    """at C5's own encoder config (1024 encoder on 256^2, blocks 8-9 unused) the first step's
    registration-order buckets cannot launch during backward (bucket 0 waits for blocks 8-9); after the rebuild from
    the hook order every bucket launches inside backward, and the gradients equal allreduce_gradients' on both ranks."""
    out = str(tmp_path / "c5")
    icd.launch(2, _c5_reducer_worker, out)
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    assert any(k.startswith("enc.blocks.8.") for k in res[0]["unused"])
    assert any(k.startswith("enc.blocks.9.") for k in res[0]["unused"])
    assert res[0]["n_buckets"] >= 5   # ~120 MB of used f32 gradients in 25 MiB buckets
    for rk in range(2):
        steps = res[rk]["steps"]
        for step in range(3):
            d = steps[step]
            assert set(d["got"]) == set(d["ref"])
            for k in d["ref"]:
                assert torch.allclose(d["got"][k], d["ref"][k], rtol=1e-5, atol=1e-8), (step, k)
                assert torch.equal(d["got"][k], res[0]["steps"][step]["got"][k]), ("ranks disagree", step, k)
        assert steps[0]["launched"] == 0   # registration order: bucket 0 holds blocks 8-9
        for step in (1, 2):
            assert steps[step]["launched"] == steps[step]["nb"] == res[0]["n_buckets"], steps[step]["launched"]


def _order_worker(out_path):
    import torch.distributed as dist
    rank, world, _ = icd.init("gloo")
    torch.manual_seed(0)
    m = _ToyEncoder()
    r = icd.GradReducer(m, world, bucket_bytes=64)
    x = torch.randn(5, 6, generator=torch.Generator().manual_seed(rank))
    m.zero_grad(set_to_none=True)
    r.start()
    m(x).sum().backward()
    if rank == 1:
        r._fired.reverse()   # a rank whose hooks fired in another order (the rebuild must not trust it)
    r.finish()
    names = {id(p): k for k, p in m.named_parameters()}
    names.update({id(p): f"param{i}" for i, p in enumerate(r.params) if id(p) not in names})
    torch.save({"buckets": [[names[id(p)] for p in b] for b in r.buckets]}, f"{out_path}.{rank}")
    r.remove()
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_rebuild_uses_rank0_order(tmp_path):
    """The rebuilt buckets come from rank 0's recorded hook order on every rank (broadcast), so ranks whose hooks fired
    in different orders still issue the same collective sequence; the parameter without a gradient is left out."""
    out = str(tmp_path / "ord")
    icd.launch(2, _order_worker, out)
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    assert r0["buckets"] == r1["buckets"] and r0["buckets"]
    flat = [k for b in r0["buckets"] for k in b]
    assert "unused" not in flat and len(flat) == len(set(flat))
    assert {"a.weight", "a.bias", "b.weight", "b.bias"} <= set(flat)


def test_grad_reducer_single_process_is_inert():
    m = _ToyEncoder()
    r = icd.GradReducer(m, world=1)
    r.start()
    m(torch.randn(2, 6)).sum().backward()
    assert r.finish() == 0 and not r._handles
