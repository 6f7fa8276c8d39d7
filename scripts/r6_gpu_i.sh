#!/bin/bash
# round-6 session I: the barrier-free k_stage2_qp (HD_QP_SYNC=1: three expanded sets, LDS
# progress counters instead of the per-chunk barrier) at 3 pairs per chunk -- parity (qp tests;
# the ppc-shape asserts of the odd-chunk / merged tests expect 4 pairs per chunk and may fail
# under HD_QP_PPC=3) and the bench A/B against plain 3 and the default 4 pairs per chunk.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
HD_QP_SYNC=1 HD_QP_PPC=3 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_qp.py > gpurun_out/r6i_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit 1
bash scripts/ab_env.sh HD_QP_PPC=3 "HD_QP_SYNC=1 HD_QP_PPC=3" > gpurun_out/r6i_ab.txt 2>&1 || exit 2
cat gpurun_out/r6i_ab.txt
