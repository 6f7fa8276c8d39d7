#!/bin/bash
# Session r4d: fused stage 1 at 3 workgroups per CU + the batched series sums + the relaxed
# stage-2 store wait (tests, A/Bs), then the single-pulse tests and split.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_q8m.py tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_c2.py -m gpu -x -v \
    --timeout 900 --timeout-method thread -k "q8m or fused or stage1 or stage2 or multipass or dual or own_stream or slices or c2 or clip_stats or int8" \
    > gpurun_out/r4d_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4d_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
bash scripts/ab_env.sh HD_S2_SWAIT=0 HD_Q8M=0 > gpurun_out/ab_r4d.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_r4d.txt; exit 1; }
cat gpurun_out/ab_r4d.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4d -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu \
    --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_r4d.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_r4d.log; exit 1; }
for f in $(find gpurun_out/prof_r4d -name "*kernel_stats.csv"); do cp "$f" gpurun_out/r4d_kernel_stats.csv; done
bash scripts/gpu_sp.sh || exit 1
echo "r4d done"
