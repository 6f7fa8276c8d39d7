#!/bin/bash
# Round-5 session k: the q8m float-fold probe; one rank's time slice alone (--sim-slice) at G = 2 / 8 for the per-rank
# fixed costs, plus its kernel stats at 0/8.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5k_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5k_q8m_probe.txt; exit 1; }
cat gpurun_out/r5k_q8m_probe.txt
for s in 0/2 0/8 7/8; do
  timeout -k 10 300 python3 bench.py --mode slices --sim-slice $s --steps 5 --warmup 2 $L > gpurun_out/r5k_sim.log 2>&1 \
      || { echo "sim-slice $s failed"; tail -5 gpurun_out/r5k_sim.log; exit 1; }
  echo "sim-slice $s: $(python3 scripts/benchline.py gpurun_out/r5k_sim.log)"
  tail -1 gpurun_out/r5k_sim.log >> gpurun_out/r5k_simslice.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k_prof -o run -- python3 bench.py --mode slices \
    --sim-slice 0/8 --steps 3 --warmup 1 $L > gpurun_out/r5k_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/r5k_prof -name '*.db' | head -1)" gpurun_out/r5k_kstats.csv
head -30 gpurun_out/r5k_kstats.csv
