#!/bin/bash
# Closing measurements of a round: the default bench line (the driver's command), kernel stats of
# the bench step, the 4-bit beam, and one rank's time slice alone at G = 2 / 8 (ranks 0 and 7).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 600 python3 bench.py > gpurun_out/fin_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/fin_bench.log; exit 1; }
tail -1 gpurun_out/fin_bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run -- python3 bench.py --steps 3 --warmup 1 $L \
    > gpurun_out/fin_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/fin_prof.log; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/fin_prof -name '*.db' | head -1)" gpurun_out/fin_kstats.csv
head -20 gpurun_out/fin_kstats.csv | cut -c1-150
timeout -k 10 300 python3 bench.py --nbits 4 --steps 5 --warmup 2 $L > gpurun_out/fin_4bit.log 2>&1 \
    || { echo "4-bit failed"; tail -5 gpurun_out/fin_4bit.log; exit 1; }
echo "4-bit: $(python3 scripts/benchline.py gpurun_out/fin_4bit.log)"
rm -f gpurun_out/fin_simslice.jsonl
for s in 0/2 0/8 7/8; do
  timeout -k 10 300 python3 bench.py --mode slices --sim-slice $s --steps 5 --warmup 2 $L > gpurun_out/fin_sim.log 2>&1 \
      || { echo "sim-slice $s failed"; tail -5 gpurun_out/fin_sim.log; exit 1; }
  echo "sim-slice $s: $(python3 scripts/benchline.py gpurun_out/fin_sim.log)"
  tail -1 gpurun_out/fin_sim.log >> gpurun_out/fin_simslice.jsonl
done
echo "final done"
