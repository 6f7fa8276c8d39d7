#!/bin/bash
# Session r4t: k_stage2_pair with each chunk's expand parameters prefetched a chunk ahead
# (HD_S2_XPF=0 turns the prefetch off in the same kernel).  Stage-2 tests, bench A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py tests/test_gpu_c4.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4t_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4t_tests.log; exit 1; }
tail -2 gpurun_out/r4t_tests.log
bash scripts/ab_env.sh HD_S2_XPF=0 > gpurun_out/ab_r4t.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4t.txt; exit 1; }
cat gpurun_out/ab_r4t.txt
echo "r4t done"
