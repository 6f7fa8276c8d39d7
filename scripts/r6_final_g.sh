#!/bin/bash
# round-6 closing, call 7: one rank's time slice alone (0/8, 7/8) on the final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
rm -f gpurun_out/fin7_simslice.jsonl
for s in 0/8 7/8; do
  timeout -k 10 300 python3 bench.py --mode slices --sim-slice $s --steps 5 --warmup 2 $L > gpurun_out/fin7_sim.log 2>&1 || exit 3
  tail -1 gpurun_out/fin7_sim.log >> gpurun_out/fin7_simslice.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/fin7_simslice.jsonl'):
    j=json.loads(l); print(j['ms_per_step'], j.get('kernel_ms_per_step'))"
