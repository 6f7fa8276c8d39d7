#!/bin/bash
# Session r4k: smoke + every -m gpu test (fix8 fold two steps in flight, one launch zeroing
# the plans' max words, ...), bench A/B of --streams 3, the hd-comm slice phases timed.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/gpu_tests_r4k.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r4k.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/gpu_tests_r4k.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r4k.log
bash scripts/ab_args.sh "" "--streams 3" > gpurun_out/ab_r4k.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4k.txt; exit 1; }
cat gpurun_out/ab_r4k.txt
timeout -k 10 300 python3 scripts/probe_hdcomm.py > gpurun_out/hdcomm_probe.txt 2>&1 || { echo "hdcomm probe failed"; tail -20 gpurun_out/hdcomm_probe.txt; exit 1; }
grep -v "^\[W\|amdgpu" gpurun_out/hdcomm_probe.txt
echo "r4k done"
