"""Per-launch HBM traffic of the igemm kernels from two rocprofv3 --pmc passes over bench.py.

    python tools/pmc_traffic.py 'gpurun_out/pmc_traffic/p*' out.json [bench args...]

Units and gfx950 corrections (MI355X_MICROARCH.md, "HBM"; cdna_hip_programming.md "Profile"):
FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read on gfx950 (the igemm operand loads are 16-B-per-lane LDS-DMA), so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Per launch = the bytes of every dispatch behind ic2_conv_igemm (igemm*, the split-K combine, the halo conv
and the ToRGB kernel) / the number of ic2_conv_igemm calls (= conv-body dispatches), matching how bench.py
times the kernel.
"""
import collections
import csv
import glob
import json
import sys


def main():
    pat, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(float)     # counter -> total over igemm dispatches
    calls = collections.Counter()            # counter -> number of GEMM-body dispatches seen in that pass
    kinds = collections.Counter()
    for d in sorted(glob.glob(pat)):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            rows = [r for r in csv.DictReader(open(f))
                    if any(t in r["Kernel_Name"] for t in ("igemm", "hgemm", "hg4_", "hconv_kernel", "torgb_kernel"))]
            names = {int(r["Dispatch_Id"]): r["Kernel_Name"] for r in rows}
            for r in rows:
                k = r["Kernel_Name"]
                c = r["Counter_Name"]
                per[c] += float(r["Counter_Value"])
                # one ic2_conv_igemm call = one conv-body dispatch, except the split 384-wide layers (an 8-phase
                # 256-wide dispatch directly followed by a 128 x 512 one) and the split-K combine kernel
                split_tail = "igemm8_og1" in k and "igemm8_og2" in names.get(int(r["Dispatch_Id"]) - 1, "")
                if "splitk_reduce" not in k and not split_tail:
                    calls[c] += 1
                    kinds[k.split("(")[0]] += 1
    if "FETCH_SIZE" not in per or "WRITE_SIZE" not in per:
        sys.exit(f"missing counters in {pat}: {sorted(per)}")
    fetch = 2.0 * per["FETCH_SIZE"] * 1024 / calls["FETCH_SIZE"]
    write = per["WRITE_SIZE"] * 1024 / calls["WRITE_SIZE"]
    rec = {"kernel": "igemm (all ic2_conv_igemm calls of the bench step)", "bench_args": sys.argv[3:],
           "launches_profiled": calls["FETCH_SIZE"], "fetch_bytes_per_launch": round(fetch),
           "write_bytes_per_launch": round(write), "hbm_bytes_per_launch": round(fetch + write),
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count, KiB units)",
           "dispatches": dict(kinds)}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
