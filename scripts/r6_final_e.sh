#!/bin/bash
# round-6 closing, call 5: the PMC passes of the final build (-> profiles/pmc_r06.json) and the
# 4-bit bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 300 python3 bench.py --nbits 4 --steps 5 --warmup 2 $L > gpurun_out/fin5_4bit.log 2>&1 || { echo "4-bit failed"; exit 3; }
COMMIT=$(cat COMMIT_ID 2>/dev/null) bash scripts/gpu_pmc.sh > gpurun_out/fin5_pmc.txt 2>&1 || { echo "pmc failed"; exit 4; }
echo "final e done"
