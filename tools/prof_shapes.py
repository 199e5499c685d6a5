"""Every bench conv shape (tools/sweep_igemm.SHAPES, batch 32 bf16) run `reps` times in a fixed order: the
target for per-shape rocprofv3 --pmc passes (aggregated by tools/pmc_shapes_agg.py).
    python tools/prof_shapes.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from sweep_igemm import SHAPES  # noqa: E402


def main():
    import torch
    from image_compression_2_amd import _native as nv
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    n = 32
    for name, ci, co, s, pad in SHAPES:
        cip, cop = nv.pad32(ci), nv.pad32(co)
        ho = s + 2 * pad - 2
        x = torch.randn(n, s, s, cip, device=dev).to(torch.bfloat16)
        w = (torch.randn(cop, 3, 3, cip, device=dev) / (9 * cip) ** 0.5).to(torch.bfloat16)
        b = torch.zeros(cop, device=dev)
        y = torch.empty(n, ho, ho, cop, device=dev, dtype=torch.bfloat16)
        for _ in range(reps):
            nv.conv_igemm(nv.ptr(x), nv.ptr(w), nv.ptr(y), nv.BF16, nv.BF16, n, s, s, cip, cop, co, 3, 3, pad, ho, ho,
                          None, nv.ptr(b), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(x), dev)
        torch.cuda.synchronize()
    print("ok", len(SHAPES), "shapes x", reps)


if __name__ == "__main__":
    main()
