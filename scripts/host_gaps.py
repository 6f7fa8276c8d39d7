"""Idle gaps on the GPU and the host API calls that span them, from a rocprofv3 .db taken
with --kernel-trace --hip-runtime-trace.  For the last `window_ms` of the run: every gap
between consecutive kernels longer than `min_gap_us`, and every HIP API call longer than
`min_call_us` that overlaps it (a blocking call the host sat in while the GPU went idle).
Usage: host_gaps.py <db> [window_ms=70] [min_gap_us=40] [min_call_us=20]"""
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 70.0
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 40.0
    min_call = float(sys.argv[4]) if len(sys.argv) > 4 else 20.0
    ks = con.execute("select name, start, end from kernels order by start").fetchall()
    calls = con.execute("select name, start, end from regions order by start").fetchall()
    if not ks:
        print("no kernels")
        return
    t_end = max(k[2] for k in ks)
    t_lo = t_end - window * 1e6
    ks = [k for k in ks if k[1] >= t_lo]
    t0 = ks[0][1]
    busy_end = ks[0][2]
    prev = ks[0][0]
    total = 0.0
    for name, s, e in ks[1:]:
        if s - busy_end > min_gap * 1e3:
            g = (s - busy_end) / 1e3
            total += g
            print("gap %8.1f us at %9.3f ms  after %-40s before %s" % (g, (busy_end - t0) / 1e6, prev[:40], name[:50]))
            for cn, cs, ce in calls:
                if ce - cs >= min_call * 1e3 and cs < s and ce > busy_end:
                    print("      %-32s %9.1f us  (%9.3f .. %9.3f ms)" % (cn[:32], (ce - cs) / 1e3, (cs - t0) / 1e6,
                                                                        (ce - t0) / 1e6))
        if e > busy_end:
            busy_end = e
            prev = name
    print("total gap %.1f us over %.1f ms" % (total, (busy_end - t0) / 1e6))


if __name__ == "__main__":
    main()
