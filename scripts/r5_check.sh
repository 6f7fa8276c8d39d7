#!/bin/bash
# Validate a stage-2 change: qp / whole-beam / parity GPU tests, then two short bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_qp.py tests/test_gpu_wholebeam.py tests/test_gpu_parity.py > gpurun_out/chk_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/chk_tests.log; exit 1; }
tail -2 gpurun_out/chk_tests.log
bash scripts/ab_env.sh
