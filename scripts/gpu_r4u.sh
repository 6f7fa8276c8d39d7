#!/bin/bash
# Session r4u: the crafted-subband single-pulse test (ties, zero-std blocks, negatives).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_pulse.py -m gpu -x -v --timeout 500 --timeout-method thread \
    > gpurun_out/r4u_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4u_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4u_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r4u_tests.log | cut -c1-150
tail -2 gpurun_out/r4u_tests.log
