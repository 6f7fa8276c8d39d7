#!/bin/bash
# round-6 session L: where k_sp_hits' time goes after the bitmask change (HD_SP_PROBE bits: 1 no
# prune walk, 4 no boxcar hits, 8 no true chain, 16 no emission; per-phase workgroup clocks with
# HD_SP_STATS=1), and the default bench line with the committed PMC traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_sp.sh "" HD_SP_PROBE=1 HD_SP_PROBE=4 HD_SP_PROBE=8 HD_SP_PROBE=16 > gpurun_out/r6l_probe.txt 2>&1 \
    || { echo "probe failed"; exit 1; }
HD_SP_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 1 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 > gpurun_out/r6l_stats.log 2>&1 || { echo "stats failed"; exit 2; }
timeout -k 10 600 python3 bench.py > gpurun_out/r6l_bench.log 2>&1 || { echo "bench failed"; exit 3; }
cat gpurun_out/r6l_probe.txt
