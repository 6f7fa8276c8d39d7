#!/bin/bash
# One parameterised GPU session (replaces the per-session one-off scripts): smoke, -m gpu
# tests, bench, rocprofv3 kernel stats, optional A/B and extra commands.  Every GPU step has
# its own time limit; the script stops at the first failure, crash or timeout.
#
#   TAG=r5a                 prefix of the logs under gpurun_out/ (default: session)
#   TESTS="tests/x.py -k y" pytest paths/args, or "none" (default: tests)
#   TEST_TIMEOUT=900        wall limit of the pytest step (seconds)
#   SMOKE=0|1               __graft_entry__.smoke() first (default 1)
#   BENCH=0|1               default bench line (default 1); BENCH_ARGS="..." extra arguments
#   PROF=0|1                rocprofv3 kernel stats of 3 bench steps (default 1)
#   PROF_SP=0|1             kernel stats of the single-pulse leg (default 0)
#   EXTRA="cmd"             one more command, run last under its own 600 s limit
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${TAG:-session}
TESTS=${TESTS:-tests}
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
    || { echo smoke failed; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -1 gpurun_out/${T}_smoke.log
fi
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/${T}_tests.log
  tail -3 gpurun_out/${T}_tests.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/${T}_tests.log | head -20; exit 1; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/${T}_bench.log 2>&1 \
    || { echo bench failed; tail -20 gpurun_out/${T}_bench.log; exit 1; }
  tail -1 gpurun_out/${T}_bench.log | cut -c1-400
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 3 --warmup 1 \
    --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 ${BENCH_ARGS} \
    > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${T}_prof.log; exit 1; }
  python3 scripts/kstats.py "$(find gpurun_out/${T}_prof -name '*.db' | head -1)" gpurun_out/${T}_kstats.csv
  head -12 gpurun_out/${T}_kstats.csv
fi
if [ "${PROF_SP:-0}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_sp -o run -- python3 bench.py --steps 1 --warmup 1 \
    --no-cpu --e2e-beams 0 --sp-beams 1 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/${T}_prof_sp.log 2>&1 \
    || { echo prof_sp failed; exit 1; }
  python3 scripts/kstats.py "$(find gpurun_out/${T}_prof_sp -name '*.db' | head -1)" gpurun_out/${T}_kstats_sp.csv
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/${T}_extra.log 2>&1 || { echo extra failed; tail -30 gpurun_out/${T}_extra.log; exit 1; }
  tail -30 gpurun_out/${T}_extra.log
fi
echo "session $T done"
