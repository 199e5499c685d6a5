"""Census of the C5 training step's leaf ATen ops (the small torch launches): torch.profiler over two steps of the
bench's C5 setup (f16 + loss scaler), counted per op name and, where the profiler recorded a Python stack, the
innermost package frame (ops issued from the autograd engine's backward thread carry none: "?").

    python tools/prof_c5_ops.py [--steps 2] [--top 40] [--mode profiler|dispatch]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--mode", choices=("profiler", "dispatch"), default="profiler")
    args = ap.parse_args()
    import image_compression_2_amd as ic2
    from image_compression_2_amd import training as ict
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision="f16").to(dev)
    torch.manual_seed(1)
    G = ic2.Generator(img_resolution=256, precision="f16").to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G, training_resolution=256)
    x = (torch.rand(16, 3, 256, 256, generator=torch.Generator().manual_seed(1000)) * 2 - 1).to(dev)
    opt = ict.make_optimizer(enc, lr=1e-4)
    w_avg = G.mapping.w_avg.view(1, 1, -1)
    scaler = ict.make_f16(comp)

    def step():
        return ict.train_step(comp, x, opt, w_avg, rec_weight=1.0, perceptual_weight=0.0, kl_weight=0.01,
                              scaler=scaler)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if args.mode == "dispatch":
        # TorchDispatchMode census: every ATen op that reaches the backend, attributed to the innermost package frame
        # of the Python stack of the thread that issued it (the autograd engine runs the package's Function.backward in
        # Python, so its ops carry their frame too)
        import traceback
        from torch.utils._python_dispatch import TorchDispatchMode
        counts = {}

        class Census(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args_=(), kwargs=None):
                fr = "?"
                for f in reversed(traceback.extract_stack()[:-1]):
                    if "image_compression_2_amd" in f.filename or "torch/amp" in f.filename or "torch/optim" in f.filename:
                        fr = f"{os.path.basename(f.filename)}:{f.lineno}"
                        break
                key = (str(func.overloadpacket.__name__), fr)
                counts[key] = counts.get(key, 0) + 1
                return func(*args_, **(kwargs or {}))
        with Census():
            for _ in range(args.steps):
                step()
        torch.cuda.synchronize()
        skip = {"view", "_unsafe_view", "as_strided", "detach", "t", "transpose", "permute", "expand", "slice", "select",
                "unsqueeze", "squeeze", "reshape", "alias", "split", "chunk", "unbind", "empty", "empty_like",
                "empty_strided", "is_same_size", "_to_copy_view", "lift_fresh"}
        rows = [(k, c) for k, c in counts.items() if k[0] not in skip]
        print(f"ops per step (views / empties excluded): {sum(c for _, c in rows) / args.steps:.0f}")
        for (name, frame), c in sorted(rows, key=lambda kv: -kv[1])[: args.top]:
            print(f"{c / args.steps:7.1f}  {name:32s} {frame}")
        return
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    # leaf ATen ops (the ones that launch), attributed to the innermost frame inside the package / torch.amp / optim
    counts = {}
    for e in prof.events():
        if not e.name.startswith("aten::") or e.cpu_children:
            continue
        frames = [f for f in (e.stack or []) if "image_compression_2_amd" in f or "torch/amp" in f or "torch/optim" in f
                  or "autograd" in f]
        key = (e.name, frames[0] if frames else "?")
        counts[key] = counts.get(key, 0) + 1
    total = sum(counts.values())
    print(f"leaf aten ops per step: {total / args.steps:.0f}")
    for (name, frame), c in sorted(counts.items(), key=lambda kv: -kv[1])[: args.top]:
        print(f"{c / args.steps:7.1f}  {name:32s} {frame}")


if __name__ == "__main__":
    main()
