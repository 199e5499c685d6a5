"""Kernel microbenchmarks on the SG3-T-256 layer shapes (batch 32): FLR, implicit GEMM (bf16) and the f16 hg4
layers (L11-L13).

    python tools/bench_kernels.py [flr|igemm|hg4] [variant-env-value ...]

Each variant runs in a child process (the variant env var is read once per process).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(kind):
    import numpy as np
    import torch
    import image_compression_2_amd as ic2
    from image_compression_2_amd import _native as nv
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    # BK_RES / BK_N: another generator resolution / batch (e.g. 1024 / 8 for the C4 layers)
    G = ic2.Generator(img_resolution=int(os.environ.get("BK_RES", 256)), precision="bf16").to(dev)
    res = {}
    n = int(os.environ.get("BK_N", 32))
    for name in G.synthesis.layer_names[:-1]:
        L = getattr(G.synthesis, name)
        s_in = int(L.in_size[0])
        conv = s_in + 2
        s_out = int(L.out_size[0])
        if kind == "flr":
            # f16 input: what the synthesis conv epilogue hands the fused filtered lrelu
            # (channel-blocked NHWC16, as the synthesis path hands it over, unless IC2_FLR_BLOCKED=0)
            blocked = os.environ.get("IC2_FLR_BLOCKED", "1") != "0"
            y = (torch.randn(n, conv, conv, L.cout_p, device=dev) * 2).to(torch.float16)
            out = torch.empty(n, s_out, s_out, L.cout_p, device=dev, dtype=torch.bfloat16)
            fn = "ic2_flrelu_nhwc16" if blocked else "ic2_flrelu_nhwc"
            def run():
                nv.call(fn, nv.ptr(y), nv.ptr(out), nv.F16, nv.BF16, n, L.cout_p, conv, conv, s_out,
                        s_out, L._fu.ctypes.data_as(__import__("ctypes").c_void_p), L._fu.shape[0],
                        L._fd.ctypes.data_as(__import__("ctypes").c_void_p), L._fd.shape[0], None, L.up_factor,
                        L.down_factor, *L.padding, float(np.sqrt(2)), 0.2, 256.0, 0, None, nv.stream_of(y))
            work = 0
        else:
            # hg4: the f16 synthesis convs the launch plan runs on hg4 (<= 256 in, <= 192 out)
            if kind == "hg4" and not (L.cin_p <= 256 and L.cout_p <= 192):
                continue
            dt = torch.float16 if kind == "hg4" else torch.bfloat16
            cdt = nv.F16 if kind == "hg4" else nv.BF16
            x = torch.randn(n, s_in, s_in, L.cin_p, device=dev).to(dt)
            wp, _, bp = L.packed(dt)
            out = torch.empty(n, conv, conv, L.cout_p, device=dev, dtype=dt)
            def run():
                nv.call("ic2_conv_igemm", nv.ptr(x), nv.ptr(wp), nv.ptr(out), cdt, cdt, n, s_in, s_in,
                        L.cin_p, L.cout_p, L.out_channels, 3, 3, 2, conv, conv, None, nv.ptr(bp), 0, 0.0, 1.0, -1.0,
                        1.0, nv.NHWC, nv.stream_of(x))
            work = 2.0 * n * conv * conv * L.out_channels * 9 * L.in_channels
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        if kind == "flr":  # compulsory bytes (f16 in, bf16 out) at the achieved rate, TB/s
            nbytes = n * (conv * conv + s_out * s_out) * L.cout_p * 2
            res[name] = (round(ms * 1e3, 1), round(nbytes / (ms * 1e-3) / 1e12, 2))
        else:
            res[name] = (round(ms * 1e3, 1), round(work / (ms * 1e-3) / 1e12, 1) if work else None)
    print(json.dumps(res))


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "flr"
    variants = sys.argv[2:] or ["default"]
    table = {}
    for v in variants:
        # each variant: "default" or a comma list of ENV=value overrides (read once per child process)
        env = dict(os.environ)
        for kv in v.split(","):
            if "=" in kv:
                k, val = kv.split("=")
                env[k] = val
        r = subprocess.run([sys.executable, __file__, "--child", kind], env=env, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            print(f"variant {v} failed:\n{r.stderr[-2000:]}")
            continue
        table[v] = json.loads(r.stdout.strip().splitlines()[-1])
    names = list(next(iter(table.values())).keys()) if table else []
    print(f"{kind}: us ({'TB/s of compulsory bytes' if kind == 'flr' else 'TFLOP/s'}) per layer")
    print(f"{'layer':14s}" + "".join(f"{v[-15:]:>16s}" for v in table))
    for nm in names:
        print(f"{nm:14s}" + "".join(f"{str(table[v][nm]):>16s}" for v in table))
    print(f"{'total us':14s}" + "".join(f"{sum(x[0] for x in table[v].values()):16.1f}" for v in table))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
