#!/bin/bash
# Session r4g: fix8 pads preloaded, the single-pulse true chain walked by the whole wave --
# tests, bench, the SP probes, then the PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_clip.py tests/test_gpu_q8m.py tests/test_gpu_c2.py -m gpu -x -v \
    --timeout 900 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4g_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4g_tests.log; exit 1; }
tail -2 gpurun_out/r4g_tests.log
bash scripts/ab_env.sh > gpurun_out/ab_r4g.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4g.txt; exit 1; }
cat gpurun_out/ab_r4g.txt
bash scripts/gpu_spprobe.sh || exit 1
bash scripts/gpu_pmc.sh || exit 1
echo "r4g done"
