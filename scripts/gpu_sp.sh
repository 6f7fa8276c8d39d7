#!/bin/bash
# Single-pulse: its GPU tests, then the bench's SP leg (2 beams) with HD_SP_TIMING=1 (collect
# waits / copies / host prune wall times) under each HD_SP_PROBE (0 full, 1 no prune walk, 8 no
# true chain, 4 no boxcar bitmask) and with the 4-wave k_sp_hits (HD_SP_NW=4), then the
# per-kernel device times of one full leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/sp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sp_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/sp_tests.log; exit 1; }
tail -2 gpurun_out/sp_tests.log
B="python3 bench.py --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --sp-beams 2"
: > gpurun_out/sp_split.txt
for pr in 0 1 8 4 nw4; do
  e="HD_SP_PROBE=$pr"; [ "$pr" = nw4 ] && e="HD_SP_NW=4"
  env HD_SP_TIMING=1 $e timeout -k 10 300 $B > gpurun_out/sp_$pr.log 2>&1 || { echo "bench failed (probe $pr)"; tail -20 gpurun_out/sp_$pr.log; exit 1; }
  python3 - "$pr" >> gpurun_out/sp_split.txt <<'PY' || { echo "no line"; exit 1; }
import json, sys
pr = sys.argv[1]
txt = open("gpurun_out/sp_%s.log" % pr).read().splitlines()
line = next(json.loads(l) for l in txt if l.startswith("{"))
tim = [l for l in txt if l.startswith("hd_single_pulse:")]
print("probe %s: %.3f s/beam, %d candidates/beam | %s" % (pr, line["single_pulse"]["s_per_beam"],
      line["single_pulse"]["candidates_per_beam"], tim[-1] if tim else "no timing"))
PY
done
cat gpurun_out/sp_split.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu \
    --e2e-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --sp-beams 1 > gpurun_out/prof_sp.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_sp.log; exit 1; }
for f in $(find gpurun_out/prof_sp -name "*kernel_stats.csv"); do cp "$f" gpurun_out/sp_kernel_stats.csv; done
echo "sp done"
