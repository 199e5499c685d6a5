"""Per-launch HBM traffic of the bench's kernel families from two rocprofv3 --pmc passes over bench.py.

    python tools/pmc_traffic.py 'gpurun_out/pmc_traffic/p*' out.json [bench args...]

Units and gfx950 corrections (MI355X_MICROARCH.md, "HBM"; cdna_hip_programming.md "Profile"):
FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read on gfx950 (the operand loads are 16-B-per-lane LDS-DMA), so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Families (round 3: the same launch set bench.py's roofline times):
  conv  -- every dispatch behind a conv entry point (igemm*, the split-K combine, hg4, the halo conv, ToRGB,
           from_rgb, the Winograd conv); per launch = bytes / conv-body dispatches (the split 384-wide layer's og2 + og1 pair and the
           split-K combine count as one launch), matching bench.py's per-call accounting;
  igemm8_og2 -- the dominant kernel alone (per dispatch; the og2 half of a split 384 pair included);
  flr   -- the fused filtered lrelu (flrelu_mfma*), per dispatch.
"""
import collections
import csv
import glob
import json
import sys

CONV = ("igemm", "hg4_", "hconv_kernel", "torgb_kernel", "from_rgb_kernel", "wino_fx")


def main():
    pat, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # family -> counter -> total
    calls = collections.defaultdict(collections.Counter)                    # family -> counter -> launches
    kinds = collections.Counter()
    for d in sorted(glob.glob(pat)):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            rows = list(csv.DictReader(open(f)))
            names = {int(r["Dispatch_Id"]): r["Kernel_Name"] for r in rows}
            for r in rows:
                k, c, v = r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])
                fams = []
                if any(t in k for t in CONV):
                    fams.append("conv")
                    split_tail = "igemm8_og1" in k and "igemm8_og2" in names.get(int(r["Dispatch_Id"]) - 1, "")
                    if "splitk_reduce" not in k and not split_tail:
                        calls["conv"][c] += 1
                        kinds[k.split("(")[0]] += 1
                if "igemm8_og2" in k:
                    fams.append("igemm8_og2")
                    calls["igemm8_og2"][c] += 1
                if "flrelu_mfma" in k:
                    fams.append("flr")
                    calls["flr"][c] += 1
                for fam in fams:
                    per[fam][c] += v
    if "FETCH_SIZE" not in per["conv"] or "WRITE_SIZE" not in per["conv"]:
        sys.exit(f"missing counters in {pat}: {sorted(per['conv'])}")
    rec = {"bench_args": sys.argv[3:],
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count, KiB units)"}
    for fam in ("conv", "igemm8_og2", "flr"):
        if not calls[fam]["FETCH_SIZE"]:
            continue
        fetch = 2.0 * per[fam]["FETCH_SIZE"] * 1024 / calls[fam]["FETCH_SIZE"]
        write = per[fam]["WRITE_SIZE"] * 1024 / calls[fam]["WRITE_SIZE"]
        rec[fam] = {"launches_profiled": calls[fam]["FETCH_SIZE"], "fetch_bytes_per_launch": round(fetch),
                    "write_bytes_per_launch": round(write), "hbm_bytes_per_launch": round(fetch + write)}
    # top-level fields kept for bench.py's roofline.traffic (the conv family)
    rec["kernel"] = "conv family (every conv entry point of the bench step)"
    rec.update(rec["conv"])
    rec["dispatches"] = dict(kinds)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
