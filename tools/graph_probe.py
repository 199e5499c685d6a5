"""Where does a graph-captured f16 C5 step go wrong?  Captures, on the f16 training path (make_f16 + GradScaler),
(A) the loss forward only, (B) forward + scaled backward, (C) the whole train_step (capturable Adam), each with the
fine projector fixed (fix_fine_projector=True, no per-call fc1) and -- (A) and (C) again -- with the reference's
per-call fc1 drawn on the device; replays each and compares with the eager value on the same weights and batch.
    python tools/graph_probe.py [batch]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(dev, n, fix):
    import image_compression_2_amd as ic2
    from image_compression_2_amd import training as ict
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, fix_fine_projector=fix).to(dev)
    G = ic2.Generator(img_resolution=256).to(dev).eval().requires_grad_(False)
    comp = ic2.StyleGAN3Compressor(enc, G)
    scaler = ict.make_f16(comp)
    if not fix:
        # the reverted GraphedTrainStep's fc1 draw: nn.Linear's kaiming-uniform init on the device generator (a host
        # draw through pinned memory cannot be captured)
        import types

        def refresh_fc1(self, in_features, device):
            self.fc1 = torch.nn.Linear(in_features, 256, device=device)
        for p in (enc.global_projector, enc.medium_projector, enc.fine_projector):
            p.refresh_fc1 = types.MethodType(refresh_fc1, p)
    x = (torch.rand(n, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1).to(dev)
    return comp, enc, G, scaler, x


def capture(fn, warm=2):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def main():
    from image_compression_2_amd import training as ict
    from image_compression_2_amd import autograd_ops as ao
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda", 0)
    for fix in (True, False):
        comp, enc, G, scaler, x = build(dev, n, fix)
        tag = "fixed fc1" if fix else "per-call fc1 (device draw)"

        def fwd():
            with torch.enable_grad(), ao.derived_cache():
                rec, _ = comp(x)
                return F.mse_loss(x, rec)
        eager = [float(fwd()) for _ in range(2)]
        g, out = capture(fwd)
        reps = []
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            reps.append(float(out))
        print(f"[A {tag}] forward loss eager {eager} replay {reps}", flush=True)
        del g, out

        if fix:
            def fwd_bwd():
                enc.zero_grad(set_to_none=False)
                with torch.enable_grad(), ao.derived_cache():
                    rec, _ = comp(x)
                    loss = F.mse_loss(x, rec)
                    scaler.scale(loss).backward()
                return loss.detach()
            for p in enc.parameters():
                p.grad = torch.zeros_like(p)
            le = float(fwd_bwd())
            ge = torch.sqrt(sum((p.grad.float() ** 2).sum() for p in enc.parameters())).item()
            g, out = capture(fwd_bwd)
            g.replay()
            torch.cuda.synchronize()
            gr = torch.sqrt(sum((p.grad.float() ** 2).sum() for p in enc.parameters())).item()
            print(f"[B {tag}] fwd+bwd loss eager {le:.5f} replay {float(out):.5f}; |grad| eager {ge:.4e} replay "
                  f"{gr:.4e}", flush=True)
            del g, out

        opt = torch.optim.Adam(list(enc.parameters()), lr=1e-4, betas=(0.9, 0.999), fused=True, capturable=True)
        w_avg = G.mapping.w_avg.view(1, 1, -1)

        def step():
            return ict.train_step(comp, x, opt, w_avg, perceptual_weight=0.0, sync_gradients=1, scaler=scaler)
        e = [float(step()["rec_loss"]) for _ in range(2)]
        g, out = capture(step)
        reps = []
        for _ in range(4):
            g.replay()
            torch.cuda.synchronize()
            reps.append(tuple(round(float(out[k]), 5) for k in ("rec_loss", "kl_loss", "total_loss")))
        after = float(step()["rec_loss"])
        print(f"[C {tag}] step rec_loss eager {e} replay {reps} eager-after {after:.5f} scale "
              f"{float(scaler.get_scale())}", flush=True)
        del g, out, comp, enc, G, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
