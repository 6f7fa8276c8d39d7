#!/bin/bash
# round-6 session P: k_stage2_qp wave priority (s_setprio 2) around the expand (prx) or around
# the sums (prs), two builds through HD_LIB -- qp parity of both and the bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
A=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_prx.so
B=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_prs.so
for L in $A $B; do
  HD_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qp.py \
      > gpurun_out/r6p_tests.log 2>&1 || { echo "tests failed ($L)"; exit 1; }
  tail -1 gpurun_out/r6p_tests.log
done
bash scripts/ab_env.sh HD_LIB=$A HD_LIB=$B > gpurun_out/r6p_ab.txt 2>&1 || { echo "ab failed"; exit 2; }
cat gpurun_out/r6p_ab.txt
