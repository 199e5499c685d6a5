"""Summarise a rocprofv3 PC-sampling CSV (--pc-sampling-beta-enabled, stochastic or host_trap): samples per
instruction (and per stall reason / wave-issued flag when the CSV carries them), top N, with the kernel filter.
usage: python tools/pcs_summary.py <pc_sampling*.csv> [--kernel REGEX] [--top 60] [--out file]"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    lines = [f"{args.csv}: {len(rows)} samples; columns: {list(rows[0].keys()) if rows else []}"]
    if not rows:
        print("\n".join(lines))
        return
    cols = rows[0].keys()
    kcol = next((c for c in cols if "kernel" in c.lower() and "name" in c.lower()), None)
    icol = next((c for c in cols if c.lower() in ("instruction", "inst", "instruction_text")), None)
    pcol = next((c for c in cols if "pc" in c.lower() and ("offset" in c.lower() or c.lower() in ("pc", "pc_address"))),
                None)
    if args.kernel and kcol:
        rx = re.compile(args.kernel)
        rows = [r for r in rows if rx.search(r[kcol] or "")]
        lines.append(f"{len(rows)} samples in kernels matching {args.kernel!r}")
    extra = [c for c in cols if any(t in c.lower() for t in ("stall", "reason", "issued", "wave_issued", "inst_type"))]
    key = icol or pcol
    tot = len(rows)
    by = collections.Counter(r[key] for r in rows)
    lines.append(f"top instructions by samples (key {key!r}):")
    for k, v in by.most_common(args.top):
        lines.append(f"  {v:8d} {100.0 * v / max(tot, 1):6.2f} %  {k}")
    for c in extra:
        cnt = collections.Counter(r[c] for r in rows)
        lines.append(f"by {c}: " + ", ".join(f"{k}={100.0 * v / tot:.1f}%" for k, v in cnt.most_common(12)))
    out = "\n".join(lines)
    print(out)
    if args.out:
        open(args.out, "w").write(out + "\n")


if __name__ == "__main__":
    main()
