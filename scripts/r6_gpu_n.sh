#!/bin/bash
# round-6 session N: stage-1 subband stores non-temporal (k_stage1_q8 / q8m) in the in-tree
# build -- stage-1 parity (q8m, parity, whole beams, slices, qp), smoke, the default bench line
# and kernel stats of the bench step.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6n TESTS="tests/test_gpu_q8m.py tests/test_gpu_parity.py tests/test_gpu_wholebeam.py tests/test_gpu_slices.py tests/test_gpu_qp.py" \
    TEST_TIMEOUT=700 BENCH=1 PROF=1 bash scripts/gpu_session.sh
