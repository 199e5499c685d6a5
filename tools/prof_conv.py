"""Run one synthesis-layer implicit-GEMM conv (SG3-T-256 L8 shape by default, batch 32, bf16 or PC_DT=f16) a few
times: the target for rocprofv3 --pmc passes.   python tools/prof_conv.py [cin cout size reps]
PC_WINO=1: f16, and the same conv as ic2_conv_wino (Winograd F(2,3) along x) after the direct one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from image_compression_2_amd import _native as nv
    cin, cout, size, reps = [int(v) for v in (sys.argv[1:] + ["512", "512", "148", "5"][len(sys.argv) - 1:])]
    dev = torch.device("cuda", 0)
    n = 32
    conv = size + 2
    dt = torch.float16 if os.environ.get("PC_DT") == "f16" else torch.bfloat16
    cdt = nv.F16 if dt == torch.float16 else nv.BF16
    x = torch.randn(n, size, size, cin, device=dev).to(dt)
    w = (torch.randn(cout, 3, 3, cin, device=dev) / (9 * cin) ** 0.5).to(dt)
    b = torch.zeros(cout, device=dev)
    y = torch.empty(n, conv, conv, cout, device=dev, dtype=dt)
    for _ in range(reps):
        nv.call("ic2_conv_igemm", nv.ptr(x), nv.ptr(w), nv.ptr(y), cdt, cdt, n, size, size, cin, cout, cout,
                3, 3, 2, conv, conv, None, nv.ptr(b), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(x))
    if os.environ.get("PC_WINO") == "1":
        assert dt == torch.float16, "PC_WINO needs PC_DT=f16"
        w32 = torch.randn(cout, cin, 3, 3, device=dev)
        u = torch.empty(cout, 3, 4, cin, device=dev, dtype=dt)
        nv.call("ic2_pack_weight_wino", nv.ptr(w32), cout, cin, cout, cin, 1, 1.0, nv.ptr(u), nv.F16, nv.stream_of(x))
        for _ in range(reps):
            nv.call("ic2_conv_wino", nv.ptr(x), nv.ptr(u), nv.ptr(y), cdt, cdt, n, size, size, cin, cout, cout, 2, conv,
                    conv, None, nv.ptr(b), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(x))
    torch.cuda.synchronize()
    print("ok", float(y.float().abs().mean()))


if __name__ == "__main__":
    main()
