"""CPU baseline rows of SURVEY.md 8(d) on the GPU box's host cores: the oracle (pure-PyTorch fp32 CPU
restatement, cross-validated against the reference's own CPU encoder by tools/cpu_crossval.py) timed on
  B = 1 and B = 32 at 256^2 (1024-config encoder + 8-bit quantize + SG3-T-256 synthesis), and
  B = 1 at 1024^2 (1024-config encoder on a 1024^2 input + 8-bit quantize + SG3-T-1024 synthesis).

    python tools/cpu_baseline.py [rows]     -> gpurun_out/cpu_baseline.json (copied to profiles/)

rows: comma list of b1_256, b32_256, b1_1024 (default: all).  Threads: torch's default (OMP_NUM_THREADS,
16 on the GPU box).  The fine projector's fc1 is drawn as the reference re-creates it (nn.Linear(128, 256)).
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import cpu_model  # noqa: E402
from oracle import encoder as oe  # noqa: E402
from oracle import sg3  # noqa: E402


def row(name, b, res, gen_res):
    import image_compression_2_amd as ic2
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
    sd_e = {k: v.detach() for k, v in enc.state_dict().items()}
    sd_g = sg3.init_params(gen_res, seed=1)
    x = torch.rand(b, 3, res, res, generator=torch.Generator().manual_seed(1000)) * 2 - 1
    torch.manual_seed(5)
    lin = torch.nn.Linear(128, 256)
    fc1 = (lin.weight.detach(), lin.bias.detach())
    with torch.no_grad():
        t0 = time.perf_counter()
        _, m, _ = oe.encoder_forward(sd_e, x, fine_fc1=fc1)
        t1 = time.perf_counter()
        q = oe.quantize_uniform(m, 8)
        t2 = time.perf_counter()
        sg3.synthesis_forward(sd_g, gen_res, q)
        t3 = time.perf_counter()
    out = {"batch": b, "input": res, "generator": gen_res, "encoder_s": round(t1 - t0, 3),
           "quantize_s": round(t2 - t1, 4), "synthesis_s": round(t3 - t2, 3), "total_s": round(t3 - t0, 3),
           "images_per_s": round(b / (t3 - t0), 5)}
    print(name, json.dumps(out), flush=True)
    return out


def main():
    want = sys.argv[1].split(",") if len(sys.argv) > 1 else ["b1_256", "b32_256", "b1_1024"]
    spec = {"b1_256": (1, 256, 256), "b32_256": (32, 256, 256), "b1_1024": (1, 1024, 1024)}
    res = {"cpu_model": cpu_model(), "threads": torch.get_num_threads(), "kind": "port",
           "what": "oracle/ restatement, fp32, encode + 8-bit quantize + synthesis; the reference's synthesis "
                   "cannot run offline (SURVEY.md 8(c)), the restatement's stands in for it", "rows": {}}
    for name in want:
        res["rows"][name] = row(name, *spec[name])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "cpu_baseline.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
