"""Kernel dispatch sequence (name, grid, workgroup, LDS, duration) from a rocprofv3 results
.db -- the kernels view kstats.py aggregates.  Usage: ktrace.py <db> [first] [count]"""
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    want = [c for c in ("grid_size_x", "grid_size_y", "workgroup_size_x", "group_segment_size") if c in cols]
    q = "select %s, start, end - start%s from kernels order by start" % (name, "".join(", " + c for c in want))
    rows = con.execute(q).fetchall()
    t0 = rows[0][1] if rows else 0
    for i, r in enumerate(rows[first:first + count], first):
        n = r[0] if len(r[0]) < 70 else r[0][:67] + "..."
        print("%5d %10.3f ms %9.1f us  %-70s %s" % (i, (r[1] - t0) / 1e6, r[2] / 1e3, n, " ".join(str(x) for x in r[3:])))


if __name__ == "__main__":
    main()
