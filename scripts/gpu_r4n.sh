#!/bin/bash
# Session r4n: single-pulse per-workgroup phase clocks and walk counters (HD_SP_STATS) over
# one beam's SP leg, and the SP probe-0 timing with the instrumentation compiled in (off).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
HD_SP_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 --sp-beams 1 > gpurun_out/spstats.log 2> gpurun_out/spstats.err \
    || { echo "stats run failed"; tail -20 gpurun_out/spstats.err; exit 1; }
grep -c sp_stats gpurun_out/spstats.err
PROBES="0" HD_SP_NOSTATS=1 bash scripts/gpu_spprobe.sh || exit 1
echo "r4n done"
