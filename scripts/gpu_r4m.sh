#!/bin/bash
# Session r4m: single-pulse normalisation with the window's block coefficients in LDS and
# the sample loads issued before the arithmetic; SP tests and SP probes 0/1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4m_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4m_tests.log; exit 1; }
tail -2 gpurun_out/r4m_tests.log
PROBES="0 1" bash scripts/gpu_spprobe.sh || exit 1
echo "r4m done"
