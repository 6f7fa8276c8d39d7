#!/bin/bash
# Session r4w: 16-bit data -- zero-DM and channel-sum kernels on int16 pairs, and the float
# stage-1 kernel keeping two-block tiles in its main launch.  Clip / stage-1 tests, then
# the 16-bit beam's kernel split (gpu_r4v.sh) and the 8-bit bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_clip.py tests/test_gpu_parity.py -m gpu -x -v --timeout 600 \
    --timeout-method thread -k "clean_state or 16bit or stage1 or psrfits_stream" > gpurun_out/r4w_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4w_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4w_tests.log; exit 1; }
tail -2 gpurun_out/r4w_tests.log
bash scripts/gpu_r4v.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 \
    --stream-beams 0 > gpurun_out/abe.log 2>&1 || { echo "bench failed"; exit 1; }
python3 scripts/benchline.py gpurun_out/abe.log || exit 1
echo "r4w done"
