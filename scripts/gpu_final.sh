#!/bin/bash
# Round-end session: smoke, every -m gpu test, the default bench (all legs + CPU baseline),
# kernel stats of the bench's timed steps (CSV) and of one single-pulse leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_final.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/gpu_tests_final.log; exit 1; }
tail -2 gpurun_out/gpu_tests_final.log
echo "final tests done"
