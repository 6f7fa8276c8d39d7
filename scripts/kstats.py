"""Per-kernel summary (calls, total/avg/min/max ns, share) from a rocprofv3 results .db,
written as CSV like rocprofv3's --stats kernel_stats.csv.  Usage: kstats.py <db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = con.execute("select %s, end - start from kernels" % name).fetchall()
    agg = {}
    for n, d in rows:
        a = agg.setdefault(n, [0, 0, None, 0])
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values()) or 1
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, (c, t, mn, mx) in out:
        w.writerow([n, c, t, t / c, 100.0 * t / tot, mn, mx])


if __name__ == "__main__":
    main()
