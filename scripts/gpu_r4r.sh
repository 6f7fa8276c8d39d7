#!/bin/bash
# Session r4r: stage 1's special-tile float launches on the aux stream beside k_stage1_q8 /
# k_stage1_q8m (default now; HD_S1_SPECIAL_AUX=0 puts them back on the main stream).  Stage-1
# tests, then the bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py tests/test_gpu_q8m.py tests/test_gpu_c4.py \
    -m gpu -x -v --timeout 600 --timeout-method thread -k "stage1 or int8 or c2 or q8m or c4" > gpurun_out/r4r_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4r_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4r_tests.log; exit 1; }
tail -2 gpurun_out/r4r_tests.log
bash scripts/ab_env.sh HD_S1_SPECIAL_AUX=0 > gpurun_out/ab_r4r.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4r.txt; exit 1; }
cat gpurun_out/ab_r4r.txt
echo "r4r done"
