#!/bin/bash
# Session r4q: k_stage1_q8 at ds 1 with 2 outputs per lane per quarter (HD_Q8_M1=2: half the
# tile, ~5 workgroups per CU instead of 3) -- its stage-1 tests with the switch on, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
HD_Q8_M1=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py -m gpu -x -v \
    --timeout 600 --timeout-method thread -k "stage1 or int8 or c2" > gpurun_out/r4q_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4q_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4q_tests.log; exit 1; }
tail -2 gpurun_out/r4q_tests.log
bash scripts/ab_env.sh HD_Q8_M1=2 > gpurun_out/ab_r4q.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4q.txt; exit 1; }
cat gpurun_out/ab_r4q.txt
echo "r4q done"
