#!/bin/bash
# A/B of bench.py arguments in the bench context (no legs), 2 reps each:
#   bash scripts/ab_args.sh "" "--streams 2" ...
cd "$GRAFT_REPO_ROOT" || exit 1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
for x in "$@"; do
  for rep in 1 2; do
    timeout -k 10 300 $B $x > gpurun_out/aba.log 2>&1 || { echo "bench failed ($x)"; exit 1; }
    s=$(python3 scripts/benchline.py gpurun_out/aba.log) || { echo "no bench line ($x)"; exit 1; }
    echo "[$x] $s"
  done
done
