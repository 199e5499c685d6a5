"""Data-parallel training step on the GPU (BASELINE config 5's DDP, ref train_hvae_encoder :655-707 under
torch.distributed): two ranks, each with its own batch slice and its own device RNG stream, run the HIP training
step (encoder -> frozen synthesis -> loss -> backward) with the gradient all-reduce and the fine projector's fc1
broadcast.  RCCL refuses two ranks on one GPU, so the ranks share this box's GPU over gloo (which all-reduces device
tensors through host staging); the code path above the collective is the one RCCL runs on a multi-GPU node."""
import os

import numpy as np
import pytest
import torch

from image_compression_2_amd import distributed as icd

pytestmark = pytest.mark.gpu

ENC64 = dict(img_resolution=64, img_channels=3, w_dim=512, num_ws=16, block_split=(5, 12), channel_base=1024,
             channel_max=64)


C5ENC = dict(img_resolution=1024)   # BASELINE C5's encoder: on 256^2 input the 1x1 break skips blocks 8-9


def _ddp_worker(out, steps, overlap="1", c5=False):
    os.environ["IC2_OVERLAP_ALLREDUCE"] = overlap
    import torch.distributed as dist
    import image_compression_2_amd as ic2
    from image_compression_2_amd import training as ict
    rank, world, _ = icd.init("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)   # same initial weights on every rank
    enc = ic2.HVAE_VGG_Encoder(**(C5ENC if c5 else ENC64)).to(dev)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256).to(dev).eval().requires_grad_(False)
    res = 256 if c5 else 64
    comp = ic2.StyleGAN3Compressor(enc, G, training_resolution=res)
    opt = ict.make_optimizer(enc, lr=1e-3)
    w_avg = G.mapping.w_avg.view(1, 1, -1)
    x = (torch.rand(1, 3, res, res, generator=torch.Generator().manual_seed(9 + rank)) * 2 - 1).to(dev)  # own slice
    torch.manual_seed(100 + rank)   # unsynchronised RNG streams (fc1 draws, reparameterisation noise)
    before = {k: v.detach().clone() for k, v in enc.named_parameters()}
    losses, launched = [], []
    for _ in range(steps):
        out_l = ict.train_step(comp, x, opt, w_avg, perceptual_weight=0.0, sync_gradients=world)
        losses.append(float(out_l["total_loss"]))
        r = getattr(enc, "_grad_reducer", None)
        launched.append((r.next_launch, len(r.buckets)) if r is not None else None)
    torch.cuda.synchronize()
    moved = sum(int(not torch.equal(v.detach(), before[k])) for k, v in enc.named_parameters())
    torch.save({"params": {k: v.detach().cpu() for k, v in enc.named_parameters()}, "losses": losses,
                "launched": launched, "moved": moved, "n": len(before)}, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_train_step_ranks_agree(cuda, tmp_path):
    """After two data-parallel steps both ranks hold bit-identical encoder weights (the averaged gradients and the
    broadcast fc1 are the same on every rank, although each rank saw a different image and drew different noise),
    the weights moved, and the two ranks' losses differ (their slices differ)."""
    out = str(tmp_path / "ddp")
    icd.launch(2, _ddp_worker, out, 2)
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    assert r0["params"].keys() == r1["params"].keys()
    diff = [k for k in r0["params"] if not torch.equal(r0["params"][k], r1["params"][k])]
    assert not diff, diff[:5]
    assert r0["moved"] >= r0["n"] // 2 and r1["moved"] == r0["moved"]
    assert all(np.isfinite(r0["losses"])) and all(np.isfinite(r1["losses"]))
    assert r0["losses"][0] != r1["losses"][0]


def test_overlapped_gradient_allreduce_matches_post_backward(cuda, tmp_path):
    """distributed.GradReducer (bucket all_reduces launched from backward hooks, the default) and the post-backward
    allreduce_gradients (IC2_OVERLAP_ALLREDUCE=0) give bit-identical weights after two steps: a two-rank sum does
    not depend on the bucketing or the order, and the ranks run the same seeded step either way."""
    a, b = str(tmp_path / "ov"), str(tmp_path / "pb")
    icd.launch(2, _ddp_worker, a, 2, "1")
    icd.launch(2, _ddp_worker, b, 2, "0")
    for r in range(2):
        pa, pb = (torch.load(f"{o}.{r}", weights_only=True) for o in (a, b))
        diff = [k for k in pa["params"] if not torch.equal(pa["params"][k], pb["params"][k])]
        assert not diff, diff[:5]
        assert pa["losses"] == pb["losses"]


def test_data_parallel_train_step_at_c5_encoder_config(cuda, tmp_path):
    """the C5 encoder (img_resolution=1024) on 256^2 slices, where blocks 8-9 get no gradient.
    From the second step on every gradient bucket launches its all_reduce inside backward (the reducer rebuilt its
    buckets from the first step's hook order), the ranks end bit-identical, and the overlapped reduction gives the same
    weights as the post-backward one."""
    a, b = str(tmp_path / "c5ov"), str(tmp_path / "c5pb")
    icd.launch(2, _ddp_worker, a, 3, "1", True)
    icd.launch(2, _ddp_worker, b, 3, "0", True)
    r0, r1 = (torch.load(f"{a}.{r}", weights_only=True) for r in range(2))
    diff = [k for k in r0["params"] if not torch.equal(r0["params"][k], r1["params"][k])]
    assert not diff, diff[:5]
    for r in (r0, r1):
        assert r["launched"][0][0] == 0               # first step: registration-order buckets wait for blocks 8-9
        for nl, nb in r["launched"][1:]:
            assert nb >= 5 and nl == nb, r["launched"]
    for r in range(2):
        pa, pb = (torch.load(f"{o}.{r}", weights_only=True) for o in (a, b))
        diff = [k for k in pa["params"] if not torch.equal(pa["params"][k], pb["params"][k])]
        assert not diff, diff[:5]
        assert pa["losses"] == pb["losses"]
