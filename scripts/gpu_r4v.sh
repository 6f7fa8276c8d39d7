#!/bin/bash
# Session r4v: where a 16-bit beam's time goes (bench --nbits 16, kernel stats).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16 -o run -- python3 bench.py --nbits 16 \
    --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof16.log 2>&1 \
    || { echo prof16 failed; tail -20 gpurun_out/prof16.log; exit 1; }
python3 scripts/benchline.py gpurun_out/prof16.log || exit 1
f=$(find gpurun_out/prof16 -name "*kernel_stats.csv" | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-70s calls %5s ms/step %8.3f" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6 / 4))
PY
