"""Encoder training step: the body of the reference's ``train_hvae_encoder`` loop (BASELINE config C5,
/root/reference/stylegan3_hvae_full.py:383-707, step at :655-707), on the HIP autograd path.

Per batch, as the reference:
    optimizer.zero_grad()                                       :664
    reconstructed, w_plus = compressor(images)                  :669  encoder (HIP fwd/bwd) -> frozen G.synthesis
    rec_loss = F.mse_loss(images, reconstructed)                :672
    perceptual = percep(images, reconstructed).mean()           :675  (LPIPS; see below)
    _, means, logvars = encoder(images)                         :678  a second encoder pass, as the reference
    kl = 0.5 * mean_n sum_{ws, c} ((means - w_avg)^2 + exp(lv) - lv - 1)      :679-683
    loss = rec_weight * rec + perceptual_weight * perceptual + kl_weight * kl  :686-688
    loss.backward(); optimizer.step()                           :699-701  (Adam(lr, (0.9, 0.999)), :484)

Deviations, all explicit:
  * LPIPS(net='vgg') needs pretrained VGG weights that cannot be fetched here (no network): ``percep`` is a
    caller-supplied callable; with ``percep=None`` a non-zero ``perceptual_weight`` raises.
  * Without fp16 the reference runs its forward under ``torch.no_grad()`` (:668) and its loss.backward()
    then fails; this step always builds the graph.  Precision: ``precision='bf16'`` on the modules (no loss
    scaling needed), or the reference's fp16 branch (:487, :669, :693-696: autocast + GradScaler) as f16
    modules (encoder 'f16', generator 'f16' with ``synthesis.train_f16``) plus a ``torch.amp.GradScaler`` passed as
    ``scaler``: the loss is scaled before backward, the step is skipped and the scale backed off when a gradient
    overflowed (the f16 kernels store gradients IEEE, so an overflow arrives as inf), as the reference's scaler does.
  * Multi-GPU: data parallel, one process per GPU, gradients averaged by distributed.allreduce_gradients.  The
    fine projector's fc1, which the reference re-creates from the CPU generator on every call (:225-230), is
    broadcast from rank 0 after each re-creation, so every rank runs -- and averages the gradients of -- the same
    weights (or build the encoder with fix_fine_projector=True: no re-creation at all).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import autograd_ops as ao
from . import distributed as icd


def kl_divergence(means, logvars, w_avg):
    """KL(q(w | x) || N(w_avg, I)) summed over [num_ws, w_dim] and averaged over the batch (ref :679-683)."""
    return 0.5 * torch.mean(torch.sum(torch.pow(means - w_avg, 2) + torch.exp(logvars) - logvars - 1, dim=[1, 2]))


def make_optimizer(encoder, lr=1e-4):
    """The reference's optimizer (:484), as one fused multi-tensor kernel per step on the device (the same update
    rule; torch's per-parameter path launched ~8 elementwise kernels per encoder tensor)."""
    params = list(encoder.parameters())
    fused = all(p.is_cuda for p in params)
    return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), fused=fused or None)


def make_f16(compressor):
    """The reference's fp16 training (autocast + GradScaler, :487, :669, :693-696) on this path: f16 activations and
    MFMA operands in the encoder and the frozen synthesis (gradients too), f32 master weights and Adam state.
    -> the GradScaler to pass to train_step (torch's: init scale 2^16, growth 2 every 2000 clean steps, backoff 0.5)."""
    compressor.encoder.set_precision("f16")
    compressor.generator.set_precision("f16")
    compressor.generator.synthesis.train_f16 = True
    return torch.amp.GradScaler("cuda")


def train_step(compressor, images, optimizer, w_avg, rec_weight=1.0, perceptual_weight=0.8, kl_weight=0.01,
               percep=None, second_encoder_pass=True, sync_gradients=None, scaler=None, shared_trunk=True):
    """One optimisation step; returns the four losses as 0-d device tensors (no host sync).

    ``w_avg``: G.mapping.w_avg shaped [1, 1, w_dim] (ref :626).  ``second_encoder_pass=False`` reuses the
    first pass's means / logvars for the KL term (identical values unless the projector's fc1 quirk redraws
    fc1, ref :225-230) and skips one encoder forward.  ``sync_gradients``: world size for the data-parallel
    gradient average (default: the initialised process group's).  ``scaler``: a torch.amp.GradScaler for f16 training
    (make_f16): scaled backward, then unscale + overflow check + step + scale update, as the reference's :693-696.
    ``shared_trunk`` (with second_encoder_pass): the reference's two encoder calls on the same batch (:669, :678)
    share one trunk (from_rgb, blocks, global average pools: deterministic, so both calls compute the same values)
    and run the projector heads twice in the reference's order -- the second call's fc1 re-draw and
    reparameterisation draw included, so every value and RNG draw is the reference's.  Autograd then sums both heads'
    gradients into one trunk backward instead of running two (the same gradient up to summation order)."""
    if percep is None and perceptual_weight != 0:
        raise ValueError("perceptual_weight != 0 needs a perceptual loss callable (the reference's LPIPS(net='vgg') "
                         "weights are not available offline): pass percep=... or perceptual_weight=0")
    encoder = compressor.encoder
    optimizer.zero_grad()
    world = sync_gradients if sync_gradients is not None else (
        torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1)
    projectors = (encoder.global_projector, encoder.medium_projector, encoder.fine_projector)
    if world > 1:
        for proj in projectors:
            proj.fc1_hook = icd.broadcast_params
    try:
        return _train_step(compressor, encoder, images, optimizer, w_avg, rec_weight, perceptual_weight, kl_weight,
                           percep, second_encoder_pass, sync_gradients, scaler, shared_trunk)
    finally:
        for proj in projectors:
            proj.fc1_hook = None


def _decode(compressor, w_plus, images):
    """compressor.forward after the encoder: the frozen synthesis, resized to the batch's resolution (:669)."""
    img = compressor.generator.synthesis(w_plus, noise_mode="const")
    if compressor.training_resolution is not None and img.shape[2] != images.shape[2]:
        from .stylegan3_hvae_full import resize_bilinear
        img = resize_bilinear(img, (images.shape[2], images.shape[3]))
    return img


def _reducer(encoder, world):
    """The encoder's overlapped gradient reducer (distributed.GradReducer, built on the first data-parallel step),
    or None: single process, or IC2_OVERLAP_ALLREDUCE=0 (the post-backward allreduce_gradients, for A/B)."""
    import os
    if world is None:
        world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if world <= 1 or os.environ.get("IC2_OVERLAP_ALLREDUCE", "1") == "0":
        return None
    r = getattr(encoder, "_grad_reducer", None)
    if r is None or r.world != world:
        r = encoder._grad_reducer = icd.GradReducer(encoder, world)
    return r


def _train_step(compressor, encoder, images, optimizer, w_avg, rec_weight, perceptual_weight, kl_weight, percep,
                second_encoder_pass, sync_gradients, scaler=None, shared_trunk=True):
    with torch.enable_grad(), ao.derived_cache():
        if second_encoder_pass and shared_trunk:
            pooled = encoder.trunk_train(images)
            w_plus, _, _ = encoder.heads_train(pooled)          # compressor(images) (:669)
            reconstructed = _decode(compressor, w_plus, images)
            _, means, logvars = encoder.heads_train(pooled)     # encoder(images) (:678)
        elif second_encoder_pass:
            reconstructed, _ = compressor(images)
            _, means, logvars = encoder(images)
        else:
            w_plus, means, logvars = encoder(images)
            reconstructed = compressor.generator.synthesis(w_plus, noise_mode="const")
            if compressor.training_resolution is not None and reconstructed.shape[2] != images.shape[2]:
                from .stylegan3_hvae_full import resize_bilinear
                reconstructed = resize_bilinear(reconstructed, (images.shape[2], images.shape[3]))
        rec_loss = F.mse_loss(images, reconstructed)
        perceptual = percep(images, reconstructed).mean() if percep is not None else rec_loss.new_zeros(())
        kl = kl_divergence(means, logvars, w_avg)
        loss = rec_weight * rec_loss + perceptual_weight * perceptual + kl_weight * kl
        reducer = _reducer(encoder, sync_gradients)
        if reducer is not None:
            reducer.start()   # bucket all_reduces launched from backward as their gradients complete
        (scaler.scale(loss) if scaler is not None else loss).backward()
    # the average of scaled gradients is the scaled average: the scaler unscales after the all_reduce
    if reducer is not None:
        reducer.finish()
    else:
        icd.allreduce_gradients(list(encoder.parameters()), sync_gradients)
    if scaler is not None:
        scaler.step(optimizer)
        scaler.update()
    else:
        optimizer.step()
    return {"rec_loss": rec_loss.detach(), "kl_loss": kl.detach(), "perceptual_loss": perceptual.detach(),
            "total_loss": loss.detach()}
