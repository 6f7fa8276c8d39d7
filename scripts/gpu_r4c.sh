#!/bin/bash
# Session r4c: stage-2 and slice tests after the relaxed store wait and the batched series
# sums, an A/B of the store wait in the bench, and one rank's slice timed at G = 2, 4, 8.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_c2.py -m gpu -x -v \
    --timeout 900 --timeout-method thread -k "stage2 or multipass or dual or own_stream or slices or c2 or clip_stats" \
    > gpurun_out/r4c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4c_tests.log; exit 1; }
tail -2 gpurun_out/r4c_tests.log
bash scripts/ab_env.sh HD_S2_SWAIT=0 > gpurun_out/ab_swait.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_swait.txt; exit 1; }
cat gpurun_out/ab_swait.txt
for g in 2 4 8; do
  timeout -k 10 200 python bench.py --mode slices --sim-slice 0/$g --steps 5 --warmup 2 --no-cpu > gpurun_out/simslice_$g.log 2>&1 \
      || { echo "sim-slice $g failed"; exit 1; }
  python3 scripts/benchline.py gpurun_out/simslice_$g.log || exit 1
done
echo "r4c done"
