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
span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
busy, cur_end = 0.0, None
for r in step:  # union of the launch intervals (kernels may overlap)
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if cur_end is None or st > cur_end:
        busy += en - st
        cur_end = en
    elif en > cur_end:
        busy += en - cur_end
        cur_end = en
print(f"\nkernel time in one step: {tot / 1e3:.3f} ms; step span {span:.3f} ms, GPU busy {busy / 1e6:.3f} ms, "
      f"idle gaps {span - busy / 1e6:.3f} ms over {len(step)} launches")
for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
    print(f"  {k:40s} {v / 1e3:8.3f} ms  {100 * v / tot:5.1f} %")
