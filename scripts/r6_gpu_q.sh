#!/bin/bash
# round-6 session Q: raised wave priority over k_stage2_qp's DMA issue + expand (vd) and over the
# fill of k_stage1_q8 / q8m (vf), two builds through HD_LIB -- qp / q8m parity and the bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
D=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_vd.so
F=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_vf.so
HD_LIB=$D timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    > gpurun_out/r6q_tests_d.log 2>&1 || { echo "tests failed (vd)"; exit 1; }
HD_LIB=$F timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_q8m.py \
    > gpurun_out/r6q_tests_f.log 2>&1 || { echo "tests failed (vf)"; exit 1; }
tail -1 gpurun_out/r6q_tests_d.log gpurun_out/r6q_tests_f.log
bash scripts/ab_env.sh HD_LIB=$D HD_LIB=$F > gpurun_out/r6q_ab.txt 2>&1 || { echo "ab failed"; exit 2; }
cat gpurun_out/r6q_ab.txt
