#!/bin/bash
# k_sp_hits device time per HD_SP_PROBE (0 full, 1 no walk, 8 no true chain, 4 no bitmask,
# 2 no width-1 hits) over one beam's single-pulse leg, from rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/spprobe.txt
for pr in ${PROBES:-0 1 8 16 4}; do
  HD_SP_PROBE=$pr timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/spp_$pr -o run -- python3 bench.py \
      --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --sp-beams 1 > gpurun_out/spp_$pr.log 2>&1 \
      || { echo "probe $pr failed"; tail -20 gpurun_out/spp_$pr.log; exit 1; }
  f=$(find gpurun_out/spp_$pr -name "*kernel_stats.csv" | sort | tail -n 1)
  python3 - "$pr" "$f" >> gpurun_out/spprobe.txt <<'PY' || exit 1
import csv, sys
pr, f = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f)):
    if "k_sp_" in r["Name"]:
        print("probe %s %-28s calls %4s total %9.2f ms avg %7.3f ms max %7.3f ms" % (pr, r["Name"].split("(")[0][-28:], r["Calls"],
              float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
PY
done
cat gpurun_out/spprobe.txt
echo "spprobe done"
