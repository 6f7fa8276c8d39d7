#!/bin/bash
# Session r4i: single-pulse survivors' partners as successive hits (no rank search per
# survivor); SP tests, bench, SP probes (16: no emission), k_stage1_q8 store probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4i_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
bash scripts/ab_env.sh > gpurun_out/ab_r4i.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4i.txt; exit 1; }
cat gpurun_out/ab_r4i.txt
bash scripts/gpu_spprobe.sh || exit 1
timeout -k 10 300 python3 scripts/probe_q8_stores.py > gpurun_out/q8_stores.txt 2>&1 || { echo "q8 probe failed"; tail -5 gpurun_out/q8_stores.txt; exit 1; }
cat gpurun_out/q8_stores.txt
echo "r4i done"
