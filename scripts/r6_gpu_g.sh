#!/bin/bash
# round-6 session G: reversed expand order (HD_QP_LOADER=2) parity + A/B; one rank's time slice
# alone (0/8, 7/8) with kernel stats (the per-slice fixed cost).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
HD_QP_LOADER=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    > gpurun_out/r6g_tests.log 2>&1 || exit 1
bash scripts/ab_env.sh HD_QP_LOADER=2 > gpurun_out/r6g_ab.txt 2>&1 || exit 2
rm -f gpurun_out/r6g_simslice.jsonl
for s in 0/8 7/8; do
  n=$(echo $s | tr / o)
  timeout -k 10 300 python3 bench.py --mode slices --sim-slice $s --steps 5 --warmup 2 $L > gpurun_out/r6g_sim.log 2>&1 || exit 3
  tail -1 gpurun_out/r6g_sim.log >> gpurun_out/r6g_simslice.jsonl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6g_prof_$n -o run -- python3 bench.py --mode slices \
      --sim-slice $s --steps 3 --warmup 1 $L > gpurun_out/r6g_prof_$n.log 2>&1 || exit 4
  python3 scripts/kstats.py "$(find gpurun_out/r6g_prof_$n -name '*.db' | head -1)" gpurun_out/r6g_kstats_$n.csv
done
