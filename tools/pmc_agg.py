"""Average PMC counters per dispatch of the kernels matching a name, over rocprofv3 --pmc pass directories.
usage: python tools/pmc_agg.py 'gpurun_out/pmcflr/p*' flrelu"""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(float)
cnt = collections.Counter()
dur = []
for d in sorted(glob.glob(sys.argv[1])):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sys.argv[2] not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sys.argv[2] in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / cnt[k]:18.0f}   (n={cnt[k]})")
if dur:
    print(f"profiled durations (us): min {min(dur):.1f} median {sorted(dur)[len(dur) // 2]:.1f}")
