"""Per-launch durations of the last complete bench step in a rocprofv3 kernel-trace CSV.
A step starts at the input packing kernel (nchw_to_nhwc).
usage: python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [min_us]"""
import collections
import csv
import sys

path = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r["Kernel_Name"]]
step = rows[starts[-2]:starts[-1]] if len(starts) >= 2 else rows
tot = 0.0
by = collections.defaultdict(float)
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("void ", "").replace("ic2::", "").replace("unsigned short", "bf16")
    by[name.split("<")[0].split("(")[0]] += d
    if d >= min_us:
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{name[:58]:58s} {d:8.1f}us wgs={grid:6d} thr={r['Workgroup_Size_X']:>4s} lds={r['LDS_Block_Size']:>6s} "
              f"vgpr={r['VGPR_Count']} agpr={r['Accum_VGPR_Count']}")
print(f"\nkernel time in one step: {tot / 1e3:.3f} ms")
for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
    print(f"  {k:40s} {v / 1e3:8.3f} ms  {100 * v / tot:5.1f} %")
