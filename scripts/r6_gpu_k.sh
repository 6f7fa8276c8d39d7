#!/bin/bash
# round-6 session K: k_stage1_q8 / k_stage1_q8m int16 outputs as paired dword stores (neighbour
# lanes swap one half: 256-byte store instructions) -- stage-1 parity (q8m, parity, whole beam)
# and the bench A/B against the short stores (HD_Q8_NARROW=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_q8m.py \
    tests/test_gpu_parity.py tests/test_gpu_wholebeam.py > gpurun_out/r6k_tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash scripts/ab_env.sh HD_Q8_NARROW=1 > gpurun_out/r6k_ab.txt 2>&1 || { echo "ab failed"; exit 2; }
cat gpurun_out/r6k_ab.txt
