#!/bin/bash
# One GPU session: smoke, the -m gpu tests, bench (default legs), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first crash or timeout.
#   TESTS=<pytest paths/-k args> BENCH=0|1 PROF=0|1 bash scripts/gpu_session.sh
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof.log 2>&1 || { echo prof failed; exit 1; }
  python3 scripts/kstats.py "$(find gpurun_out/prof -name '*.db' | head -1)" gpurun_out/kstats.csv
fi
if [ "${PROF_SP:-1}" = 1 ]; then   # kernel times of the single-pulse leg (one beam)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 1 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_sp.log 2>&1 || { echo prof_sp failed; exit 1; }
  python3 scripts/kstats.py "$(find gpurun_out/prof_sp -name '*.db' | head -1)" gpurun_out/kstats_sp.csv
fi
echo "session done"
