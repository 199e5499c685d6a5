"""What the platform's own convolution library (MIOpen, through torch.nn.functional.conv2d with benchmark-mode
algorithm search) sustains on the SG3-T-256 synthesis conv shapes at batch 32 in f16: a reference point for the
hand-written kernels (direct implicit GEMM today, Winograd F(2x2,3x3) candidate), not a product path.

Run under `rocprofv3 --kernel-trace --stats` to see which solver's kernels MIOpen picked."""
import json
import sys

import torch
import torch.nn.functional as F

# (name, n, cin, cout, h): SG3-T-256 modulated-conv shapes (3x3, padding 2 -> output h + 2)
SHAPES = [("L8_148_512", 32, 512, 512, 148), ("L6_84_512", 32, 512, 512, 84), ("L11_276_256_192", 32, 256, 192, 276)]


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    out = {}
    for name, n, cin, cout, h in SHAPES:
        for layout in ("nhwc", "nchw"):
            x = torch.randn(n, cin, h, h, device=dev, dtype=torch.float16)
            w = torch.randn(cout, cin, 3, 3, device=dev, dtype=torch.float16) * (1.0 / (cin * 9) ** 0.5)
            if layout == "nhwc":
                x = x.contiguous(memory_format=torch.channels_last)
                w = w.contiguous(memory_format=torch.channels_last)
            for _ in range(3):
                y = F.conv2d(x, w, padding=2)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                y = F.conv2d(x, w, padding=2)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            ho = h + 2
            tf = 2 * n * ho * ho * cin * cout * 9 / (ms * 1e-3) / 1e12
            key = f"{name}_{layout}"
            out[key] = {"ms": round(ms, 4), "direct_equiv_tflops": round(tf, 1)}
            print(key, out[key], flush=True)
            del x, w, y
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
