"""Per-shape PMC summary of tools/prof_shapes.py runs: conv dispatches (split-K reduce kernels excluded) are
assigned to shapes in launch order (reps per shape), counters averaged per shape over the pass directories.
    python tools/pmc_shapes_agg.py 'gpurun_out/pmcs/p*' reps > profiles/rX_pmc_shapes.json
Derived: hbm_bytes = FETCH_SIZE x 2 (gfx950 wide-read under-count) + WRITE_SIZE (KiB -> bytes);
mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from sweep_igemm import SHAPES  # noqa: E402


def is_conv(name):
    return ("igemm" in name or "hgemm" in name or "hg4" in name or "hconv" in name or "torgb" in name) and "splitk" not in name


def dispatches_per_call(ci, co, s, pad, n=32):
    """Conv-body dispatches of one ic2_conv_igemm call: 2 where the launch plan splits an odd multiple of 128
    output channels (> 128) over the 256-wide and the 128 x 512 8-phase tiles (igemm.hip, IC2_IGEMM_SPLIT)."""
    cop = (co + 31) // 32 * 32 if co <= 128 else (co + 63) // 64 * 64
    ho = s + 2 * pad - 2
    m = n * ho * ho
    return 2 if (cop % 256 == 128 and cop > 128 and -(-m // 256) >= 240 and ci > 256) else 1


def main():
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    kname = {}
    # dispatch index -> (shape, call): walk the shapes' calls, each of dispatches_per_call dispatches
    order = []
    for name, ci, co, s, pad in SHAPES:
        for _ in range(reps):
            order.append((name, dispatches_per_call(ci, co, s, pad)))

    def calls(ids):
        i = 0
        for name, dpc in order:
            if i + dpc > len(ids):
                return
            yield name, ids[i:i + dpc]
            i += dpc

    for d in sorted(glob.glob(sys.argv[1])):
        rows = {}
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if is_conv(r["Kernel_Name"]):
                    rows.setdefault(int(r["Dispatch_Id"]), []).append(r)
        for shape, dids in calls(sorted(rows)):
            kname[shape] = "+".join(rows[did][0]["Kernel_Name"].split("(")[0] for did in dids)
            tot = collections.defaultdict(float)
            for did in dids:
                for r in rows[did]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
            for k, v in tot.items():
                per[shape][k].append(v)
        trace = {}
        for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if is_conv(r["Kernel_Name"]):
                    trace[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for shape, dids in calls(sorted(trace)):
            dur[shape].append(sum(trace[did] for did in dids))
    out = {}
    for name, ci, co, s, pad in SHAPES:
        c = {k: sum(v) / len(v) for k, v in per[name].items()}
        ho = s + 2 * pad - 2
        flops = 2.0 * 32 * ho * ho * co * 9 * ci
        rec = {"kernel": kname.get(name), "us_profiled_median": round(sorted(dur[name])[len(dur[name]) // 2], 1)
               if dur[name] else None, "gflop": round(flops / 1e9, 2)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec["hbm_bytes"] = round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            rec["algorithmic_bytes"] = int(32 * (s * s * ((ci + 31) // 32 * 32) + ho * ho * ((co + 31) // 32 * 32)) * 2
                                           + ((co + 31) // 32 * 32) * 9 * ((ci + 31) // 32 * 32) * 2)
            rec["traffic_x"] = round(rec["hbm_bytes"] / rec["algorithmic_bytes"], 2)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"] > 0:
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            rec["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 4)
            if rec["us_profiled_median"]:
                rec["clock_ghz"] = round(cyc / (rec["us_profiled_median"] * 1e3), 3)
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", "SQ_LDS_BANK_CONFLICT",
                  "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS"):
            if k in c:
                rec[k] = round(c[k])
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
