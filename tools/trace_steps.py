"""Per-step kernel times from a rocprofv3 --kernel-trace CSV, timed steps only.

The bench's metric pass ends every step with one uint8_sse_partial_kernel dispatch; the dispatches up to and including
the i-th one are step i.  The first `--warmup` steps (bench --warmup, plus the one-time weight packing and first-touch
costs they carry) are dropped, and the conv-family / FLR / per-kernel times are averaged over the rest, so they can
be set against the bench's own per-call HIP events (roofline.conv_ms_per_step, roofline.flr.ms_per_step).
usage: python tools/trace_steps.py <run_kernel_trace.csv> --warmup 3 [--bench bench.json] [--out summary.txt]
"""
import argparse
import csv
import json
import re
from collections import defaultdict

CONV = ("igemm", "hg4_", "hconv_", "torgb_", "from_rgb", "wino_fx")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bench", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--step-end", default="uint8_sse_partial_kernel",
                    help="regex of the kernel that closes a step (C5: the fused Adam kernel)")
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rx = re.compile(args.step_end)
    ends = [i for i, r in enumerate(rows) if rx.search(r["Kernel_Name"])]
    steps = [(0 if k == 0 else ends[k - 1] + 1, e + 1) for k, e in enumerate(ends)]
    timed = steps[args.warmup:]
    per = defaultdict(float)
    calls = defaultdict(int)
    for a, b in timed:
        for r in rows[a:b]:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            calls[name] += 1
    n = len(timed)
    step_conv = sorted(sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows[a:b]
                           if any(c in r["Kernel_Name"] for c in CONV)) for a, b in timed)
    med_conv = step_conv[n // 2] if n % 2 else 0.5 * (step_conv[n // 2 - 1] + step_conv[n // 2])
    conv = sum(v for k, v in per.items() if any(c in k for c in CONV)) / n
    flr = sum(v for k, v in per.items() if "flrelu_mfma" in k) / n
    total = sum(per.values()) / n
    wall = sum((int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) * 1e-6 for a, b in timed) / n
    lines = [f"{args.trace}: {len(steps)} steps, {args.warmup} dropped, {n} timed",
             f"kernel time per step {total:.3f} ms (first dispatch to last of a step: {wall:.3f} ms)",
             f"conv family per step {conv:.3f} ms (every igemm*/hg4_*/hconv_*/wino_fx*/torgb_*/from_rgb* dispatch incl. the "
             f"split-K combine); median step {med_conv:.3f} ms (per-step conv ms: "
             f"{', '.join(f'{v:.2f}' for v in step_conv)})", f"filtered lrelu per step {flr:.3f} ms"]
    if args.bench:
        d = json.load(open(args.bench))
        r = d["roofline"]
        B = d["config"].get("global_batch", d["config"].get("batch"))
        fr = r["algorithmic_gflop_per_image"] * 1e9 * B / (conv * 1e-3) / (r["peak"] * 1e12)
        frm = r["algorithmic_gflop_per_image"] * 1e9 * B / (med_conv * 1e-3) / (r["peak"] * 1e12)
        lines += [f"bench: {d['value']} img/s, {d['ms_per_step']} ms/step, conv {r['conv_ms_per_step']} ms "
                  f"(frac {r['frac']}), FLR {r['flr']['ms_per_step']} ms",
                  f"recomputed from the trace: conv frac {fr:.4f} from the mean step "
                  f"({(fr / r['frac'] - 1) * 100:+.1f} % vs the bench), {frm:.4f} from the median step "
                  f"({(frm / r['frac'] - 1) * 100:+.1f} %); FLR {(flr / r['flr']['ms_per_step'] - 1) * 100:+.1f} %"]
    lines.append("per kernel (ms/step, calls/step):")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:args.top]:
        lines.append(f"  {v / n:8.3f}  {calls[k] / n:6.1f}  {k}")
    out = "\n".join(lines)
    print(out)
    if args.out:
        open(args.out, "w").write(out + "\n")


if __name__ == "__main__":
    main()
