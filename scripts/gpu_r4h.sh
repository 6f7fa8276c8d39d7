#!/bin/bash
# Session r4h: padded single-pulse prefix array (no 64-way bank conflicts in the lanes'
# walks), pipelined ballot phase, k_stage1_q8m's rotated steps for even ds -- tests, bench,
# the SP kernel times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_q8m.py tests/test_gpu_c2.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 900 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4h_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4h_tests.log; exit 1; }
tail -2 gpurun_out/r4h_tests.log
bash scripts/ab_env.sh > gpurun_out/ab_r4h.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4h.txt; exit 1; }
cat gpurun_out/ab_r4h.txt
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --sp-beams 2 \
    > gpurun_out/sp_r4h.log 2>&1 || { echo "sp leg failed"; tail -20 gpurun_out/sp_r4h.log; exit 1; }
grep -o '"single_pulse": {[^}]*}' gpurun_out/sp_r4h.log | cut -c1-140
sed -i 's/for pr in 0 1 8 4 2; do/for pr in 0 1; do/' scripts/gpu_spprobe.sh
bash scripts/gpu_spprobe.sh || exit 1
echo "r4h done"
