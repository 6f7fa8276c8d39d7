#!/bin/bash
# A/B of an environment switch in the bench context: bench.py (no legs) with and without it,
# ms per step and stage-1 / stage-2 kernel ms.   bash scripts/ab_env.sh VAR=value [...]
cd "$GRAFT_REPO_ROOT" || exit 1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
for e in "" "$@"; do
  for rep in 1 2; do
    env $e timeout -k 10 300 $B > gpurun_out/abe.log 2>&1 || { echo "bench failed ($e)"; exit 1; }
    s=$(python3 scripts/benchline.py gpurun_out/abe.log) || { echo "no bench line ($e)"; exit 1; }
    echo "[$e] $s"
  done
done
