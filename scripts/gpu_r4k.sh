#!/bin/bash
# Session r4k: fix8 fold two steps in flight, one launch zeroing the plans' max words --
# tests and bench (+ --streams 3 A/B); the hd-comm slice phases timed.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_clip.py tests/test_gpu_q8m.py tests/test_gpu_c2.py tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 900 --timeout-method thread -k "clip or q8m or fused or c2 or stage1 or int8 or 4bit" > gpurun_out/r4k_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4k_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4k_tests.log; exit 1; }
tail -2 gpurun_out/r4k_tests.log
bash scripts/ab_args.sh "" "--streams 3" > gpurun_out/ab_r4k.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4k.txt; exit 1; }
cat gpurun_out/ab_r4k.txt
timeout -k 10 300 python3 scripts/probe_hdcomm.py > gpurun_out/hdcomm_probe.txt 2>&1 || { echo "hdcomm probe failed"; tail -20 gpurun_out/hdcomm_probe.txt; exit 1; }
grep -v "^\[W\|amdgpu" gpurun_out/hdcomm_probe.txt
echo "r4k done"
