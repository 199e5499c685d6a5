"""Summarise a rocprofv3 kernel-trace database: per-kernel totals and the per-launch sequence of the last step."""
import glob
import sqlite3
import sys


def short(name, n=70):
    name = name.replace("void ", "")
    base = name.split("(")[0]
    return base[-n:]


def main(path, last=0):
    db = glob.glob(f"{path}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    print(f"{'kernel':72s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>6s}")
    for r in rows[:25]:
        print(f"{short(r[0]):72s} {r[1]:6d} {r[2]/1e6:9.3f} {r[3]/1e3:9.2f} {r[4]:6.2f}")
    if last:
        seq = list(c.execute("select name, duration, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count from kernels order by start"))
        for r in seq[-last:]:
            print(f"{short(r[0], 60):60s} {r[1]/1e3:10.2f} us  wg={r[2]//max(r[3],1):7d} lds={r[4]} vgpr={r[5]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
