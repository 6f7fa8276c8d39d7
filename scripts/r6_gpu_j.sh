#!/bin/bash
# round-6 session J: k_sp_hits' boxcar-bitmask loop with contiguous item ranges per wave (width
# parameters hoisted, four boxcars' reads in flight) -- SP parity tests, kernel times against the
# previous build (HD_LIB), and the SP leg wall time of both builds (2 beams each).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_single_pulse.py \
    > gpurun_out/r6j_tests.log 2>&1 || { echo "sp tests failed"; exit 1; }
bash scripts/ab_sp.sh "" "HD_LIB=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_sp0.so" > gpurun_out/r6j_absp.txt 2>&1 \
    || { echo "ab_sp failed"; exit 2; }
L="--steps 1 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 2 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
for e in "" "HD_LIB=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_sp0.so"; do
  env $e timeout -k 10 300 python3 bench.py $L > gpurun_out/r6j_leg.log 2>&1 || { echo "leg failed"; exit 3; }
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/r6j_leg.log').read().strip().split('\n')[-1])['single_pulse']; print('[$e]', j['s_per_beam'], j['candidates_per_beam'])" >> gpurun_out/r6j_absp.txt
done
cat gpurun_out/r6j_absp.txt
