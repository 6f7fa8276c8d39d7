#!/bin/bash
# Session r4f: stage-2 expand over one item range, width-1 hits batched per wave -- their
# tests, the bench (2 runs), the SP leg with its kernel stats, then the PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py tests/test_gpu_single_pulse.py tests/test_gpu_clip.py tests/test_gpu_q8m.py -m gpu -x -v \
    --timeout 900 --timeout-method thread -k "stage2 or multipass or dual or own_stream or c2 or single_pulse or candidate or clip or stage1 or fused or q8m or int8 or 4bit" \
    > gpurun_out/r4f_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4f_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
bash scripts/ab_env.sh > gpurun_out/ab_r4f.txt 2>&1 || { echo "bench failed"; cat gpurun_out/ab_r4f.txt; exit 1; }
cat gpurun_out/ab_r4f.txt
HD_SP_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp2 -o run -- python3 bench.py \
    --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --sp-beams 2 > gpurun_out/prof_sp2.log 2>&1 \
    || { echo "sp prof failed"; tail -20 gpurun_out/prof_sp2.log; exit 1; }
for f in $(find gpurun_out/prof_sp2 -name "*kernel_stats.csv"); do cp "$f" gpurun_out/sp2_kernel_stats.csv; done
python3 scripts/benchline.py gpurun_out/prof_sp2.log || exit 1
grep -h "hd_single_pulse:\|single_pulse" gpurun_out/prof_sp2.log | cut -c1-300
bash scripts/gpu_spprobe.sh || exit 1
bash scripts/gpu_pmc.sh || exit 1
echo "r4f done"
