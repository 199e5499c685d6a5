"""Calibration: what the vendor bf16 GEMM (torch.matmul -> hipBLASLt) sustains on MI355X for GEMMs of the
synthesis conv shapes (M = batch-32 output pixels, N = cout, K = 9 cin), i.e. the practical MFMA ceiling the
implicit-GEMM conv is compared with.   python tools/gemm_calib.py"""
import json
import torch

SHAPES = [("s148", 32 * 150 * 150, 512, 4608), ("s84", 32 * 86 * 86, 512, 4608), ("s276a", 32 * 278 * 278, 192, 2304),
          ("s276c", 32 * 278 * 278, 128, 1152), ("sq8k", 8192, 8192, 8192)]


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for name, m, n, k in SHAPES:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            torch.matmul(a, b)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        out[name] = {"m": m, "n": n, "k": k, "ms": round(ms, 3), "tflops": round(2 * m * n * k / ms / 1e9, 1)}
        del a, b
    print(json.dumps(out))


if __name__ == "__main__":
    main()
