"""Top kernels of a rocprofv3 --stats kernel_stats.csv.  usage: python tools/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:5s} "
          f"avg={float(r['AverageNs']) / 1e3:8.1f}us {r['Name'][:100]}")
print(f"total {tot / 1e6:.2f} ms")
