#!/bin/bash
# round-6 session M: the bulk output stores with the non-temporal hint (k_stage1_q8 / q8m int16
# subbands, k_stage2_qp series; a second build through HD_LIB) -- qp / q8m parity of that build
# and the bench A/B against the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
NT=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_nt.so
HD_LIB=$NT timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    tests/test_gpu_q8m.py > gpurun_out/r6m_tests.log 2>&1 || { echo "nt tests failed"; exit 1; }
bash scripts/ab_env.sh HD_LIB=$NT > gpurun_out/r6m_ab.txt 2>&1 || { echo "ab failed"; exit 2; }
cat gpurun_out/r6m_ab.txt
