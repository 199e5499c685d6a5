"""What the platform's own bf16 GEMM (hipBLASLt through torch.matmul) sustains on this MI355X on random data: the
practical ceiling the implicit-GEMM conv kernels are compared against, next to the 2.5 PF dense datasheet peak."""
import json
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for dt in (torch.bfloat16, torch.float16):
        for m, n, k in ((8192, 8192, 8192), (16384, 16384, 8192), (524288, 512, 4608), (131072, 384, 3456)):
            a = torch.randn(m, k, device=dev, dtype=dt)
            b = torch.randn(k, n, device=dev, dtype=dt)
            for _ in range(3):
                torch.matmul(a, b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                torch.matmul(a, b)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            tf = 2 * m * n * k / (ms * 1e-3) / 1e12
            key = f"{str(dt).split('.')[-1]}_{m}x{n}x{k}"
            out[key] = {"ms": round(ms, 4), "tflops": round(tf, 1)}
            print(key, out[key], flush=True)
            del a, b
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
