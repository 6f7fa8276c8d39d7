"""Kernel times per (stage, probe) of an ab_stage2.py run under
`rocprofv3 --kernel-trace --output-format csv`: the stage-2 launches of the trace in order,
split by the counts ab_stage2.py issues (reps x 8 timed + 1 readback per probe).
  python scripts/ab_trace.py <kernel_trace.csv> <ab log> [--reps=7]"""
import csv
import re
import statistics
import sys

trace, log = sys.argv[1], sys.argv[2]
reps = int(next((a[7:] for a in sys.argv[3:] if a.startswith("--reps=")), "7"))
rows = []
with open(trace) as f:
    for r in csv.DictReader(f):
        if "k_stage2" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
runs = [l for l in open(log) if re.match(r"stage \d+ probe", l)]
per = reps * 8 + 1
i = 0
for l in runs:
    m = re.match(r"stage (\d+) probe\s+(\d+).*?(identical|DIFFERENT|ref)", l)
    seg = rows[i:i + per]
    i += per
    d = [(e - s) / 1e6 for s, e, _ in seg]
    print("stage %s probe %3s: kernel min %.3f med %.3f ms  (%s)  %s" % (m.group(1), m.group(2), min(d),
          statistics.median(d), seg[0][2].split("(")[0].replace("void hd::", ""), m.group(3)))
