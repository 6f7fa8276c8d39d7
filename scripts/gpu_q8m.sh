#!/bin/bash
# Fused multi-stage stage 1 (k_stage1_q8m): its parity tests, the stage-1 / C2 tests, then an
# A/B of the bench with one stage-1 call per DDplan stage, and the kernel stats of the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_q8m.py tests/test_gpu_parity.py tests/test_gpu_clip.py tests/test_gpu_4bit.py tests/test_gpu_c2.py -m gpu -x -v \
    --timeout 600 --timeout-method thread -k "q8m or fused or stage1 or clip or 4bit or c2 or int8" > gpurun_out/q8m_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/q8m_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/q8m_tests.log; exit 1; }
tail -2 gpurun_out/q8m_tests.log
bash scripts/ab_args.sh "" "--s1-per-stage" > gpurun_out/ab_q8m.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_q8m.txt; exit 1; }
bash scripts/ab_env.sh HD_FIX8M=0 >> gpurun_out/ab_q8m.txt 2>&1 || { echo "ab env failed"; cat gpurun_out/ab_q8m.txt; exit 1; }
cat gpurun_out/ab_q8m.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8m -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu \
    --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_q8m.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_q8m.log; exit 1; }
for f in $(find gpurun_out/prof_q8m -name "*kernel_stats.csv"); do cp "$f" gpurun_out/q8m_kernel_stats.csv; done
echo "q8m done"
