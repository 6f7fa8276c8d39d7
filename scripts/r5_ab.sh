#!/bin/bash
# Round-5 A/B: the quarter-layout stage 2 (HD_S2_QP=1) against the pair kernel in the bench
# context, ms per step, then per-kernel stats of both; the in-library communicator at world 1.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/ab_env.sh HD_S2_QP=1 || exit 1
WORDS="stage2 q8m fix8" bash scripts/ab_envk.sh "" HD_S2_QP=1 || exit 1
timeout -k 10 300 python3 bench.py --mode slices --comm hd --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 \
    --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/r5_commhd.log 2>&1 || { echo "comm hd failed"; tail -5 gpurun_out/r5_commhd.log; exit 1; }
echo "comm hd: $(python3 scripts/benchline.py gpurun_out/r5_commhd.log)"
