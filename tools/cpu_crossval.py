"""Cross-validates the CPU baseline (oracle/ restatement) against the REFERENCE's own CPU encoder, in the
build container only (needs /root/reference; SURVEY.md 8(d): the restatement must time within +-15 % of the
reference on the same box before it stands in as the CPU baseline).

    python tools/cpu_crossval.py [threads]      -> profiles/r2_cpu_crossval.json

Times HVAE_VGG_Encoder.forward of the reference (stylegan3_hvae_full.py:105-167, stdout silenced: the
reference prints shapes in every forward) and oracle.encoder.encoder_forward on the SAME weights and input,
B = 1 and B = 32 at 256^2, and the reference / oracle GumbelSoftmaxDiscretization forward at B = 32.
The reference's synthesis cannot run anywhere offline, so the oracle's synthesis time
stands in for it (labelled as such in bench.py's cpu_baseline).
"""
import contextlib
import io
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from make_golden import import_reference  # noqa: E402  (stubs the absent third-party modules)
from oracle import encoder as oe  # noqa: E402


def best_of(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(threads)
    ref_full, ref_gumbel = import_reference()
    torch.manual_seed(0)
    enc = ref_full.HVAE_VGG_Encoder(img_resolution=1024).eval()
    rows = {}
    for b, reps in ((1, 5), (32, 2)):
        x = torch.rand(b, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            torch.manual_seed(2)
            enc(x)  # warm-up; re-creates the fine fc1 (reference quirk, :225-230)
            t_ref = best_of(lambda: enc(x), reps)
        sd = {k: v.detach() for k, v in enc.state_dict().items()}
        fc1 = (sd["fine_projector.fc1.weight"], sd["fine_projector.fc1.bias"])
        with torch.no_grad():
            oe.encoder_forward(sd, x, fine_fc1=fc1)
            t_or = best_of(lambda: oe.encoder_forward(sd, x, fine_fc1=fc1), reps)
        rows[f"encoder_b{b}"] = {"reference_ms_per_img": round(t_ref / b * 1e3, 2),
                                 "oracle_ms_per_img": round(t_or / b * 1e3, 2), "ratio": round(t_or / t_ref, 3)}
    z = torch.rand(32, 16, 512, generator=torch.Generator().manual_seed(3)) * 2 - 1
    disc = ref_gumbel.GumbelSoftmaxDiscretization(512, 256).eval()
    with torch.no_grad():  # both draw their Gumbel noise inside the timed call
        t_ref = best_of(lambda: disc(z, hard=True), 3)
        t_or = best_of(lambda: oe.gumbel_forward(z, oe.gumbel_noise(5, z.numel()), disc.temperature, True), 3)
    rows["gumbel_b32"] = {"reference_ms": round(t_ref * 1e3, 1), "oracle_ms": round(t_or * 1e3, 1),
                          "ratio": round(t_or / t_ref, 3)}
    cpu = "unknown"
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
    # the gate covers the stages bench.py's cpu_baseline times (encoder; its quantizer is the uniform one);
    # the Gumbel row is informational
    out = {"threads": threads, "cpu_model": cpu, "rows": rows,
           "within_15pct": all(abs(r["ratio"] - 1) <= 0.15 for k, r in rows.items() if k.startswith("encoder"))}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r2_cpu_crossval.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    assert out["within_15pct"], "oracle timing differs from the reference's by more than 15 %"


if __name__ == "__main__":
    main()
