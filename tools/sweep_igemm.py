"""Time ic2_conv_igemm_ws on the bench's conv shapes (batch 32, bf16) under launch-plan overrides.

    python tools/sweep_igemm.py [VAR=value,VAR=value ...]   (each argument = one variant, own child process)

Shapes: the 1024-config encoder on 256^2 input (pad 1) and the SG3-T-256 synthesis layers (pad 2).
Prints one JSON line per variant: {shape: [us, TFLOP/s]}.  SWEEP_DT=f16: f16 operands and output (the synthesis
precision of the bench's default mode).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, cin_valid, cout_valid, size_in, pad)
SHAPES = [("e_rgb", 3, 32, 256, 1), ("e0a", 32, 64, 256, 1), ("e0b", 64, 64, 256, 1), ("e1a", 64, 128, 128, 1),
          ("e1b", 128, 128, 128, 1), ("e2a", 128, 256, 64, 1), ("e2b", 256, 256, 64, 1), ("e3a", 256, 512, 32, 1),
          ("e3b", 512, 512, 32, 1), ("e4", 512, 512, 16, 1), ("e5", 512, 512, 8, 1),
          ("s36", 512, 512, 36, 2), ("s52", 512, 512, 52, 2), ("s84", 512, 512, 84, 2), ("s148", 512, 512, 148, 2),
          ("s148b", 512, 362, 148, 2), ("s148c", 362, 256, 148, 2), ("s276a", 256, 181, 276, 2),
          ("s276b", 181, 128, 276, 2), ("s276c", 128, 128, 276, 2)]
# SWEEP_SET=c4: the C4 workload's (batch 8) high-resolution shapes: encoder at 1024^2 / 512^2, SG3-T-1024 L8-L13
SHAPES_C4 = [("E_rgb", 3, 32, 1024, 1), ("E0a", 32, 64, 1024, 1), ("E0b", 64, 64, 1024, 1), ("E1a", 64, 128, 512, 1),
             ("E1b", 128, 128, 512, 1), ("T8", 323, 203, 276, 2), ("T9", 203, 128, 276, 2), ("T10", 128, 81, 532, 2),
             ("T11", 81, 51, 1044, 2), ("T12", 51, 32, 1044, 2), ("T13", 32, 32, 1044, 2)]
if os.environ.get("SWEEP_SET") == "c4":
    SHAPES = SHAPES_C4


def child(only):
    import torch
    from image_compression_2_amd import _native as nv
    dev = torch.device("cuda", 0)
    n = 8 if os.environ.get("SWEEP_SET") == "c4" else 32
    f16 = os.environ.get("SWEEP_DT") == "f16"
    tdt, code = (torch.float16, nv.F16) if f16 else (torch.bfloat16, nv.BF16)
    res = {}
    for name, ci, co, s, pad in SHAPES:
        if only and name not in only:
            continue
        cip, cop = (nv.pad_synth(ci), nv.pad_synth(co)) if name[0] in "sT" else (nv.pad32(ci), nv.pad32(co))
        ho = s + 2 * pad - 2
        x = torch.randn(n, s, s, cip, device=dev).to(tdt)
        w = (torch.randn(cop, 3, 3, cip, device=dev) / (9 * cip) ** 0.5).to(tdt)
        b = torch.zeros(cop, device=dev)
        y = torch.empty(n, ho, ho, cop, device=dev, dtype=tdt)

        def run():
            nv.conv_igemm(nv.ptr(x), nv.ptr(w), nv.ptr(y), code, code, n, s, s, cip, cop, co, 3, 3, pad, ho, ho,
                          None, nv.ptr(b), 0, 0.0, 1.0, -1.0, 1.0, nv.NHWC, nv.stream_of(x), dev)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        flops = 2.0 * n * ho * ho * co * 9 * ci
        res[name] = [round(us, 1), round(flops / us / 1e6, 1)]
    print(json.dumps(res), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else [])
        return
    only = os.environ.get("SWEEP_ONLY", "")
    for var in (sys.argv[1:] or [""]):
        env = dict(os.environ)
        for kv in filter(None, var.split(",")):
            k, v = kv.split("=")
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "--child", only], env=env, capture_output=True, text=True,
                           timeout=300)
        print(f"[{var or 'default'}]", r.stdout.strip() if r.returncode == 0 else ("FAILED " + r.stderr[-2000:]),
              flush=True)


if __name__ == "__main__":
    main()
