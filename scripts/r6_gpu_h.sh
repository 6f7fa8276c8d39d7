#!/bin/bash
# round-6 session H: quarter sub-tiles of the merged special launch (parity: q8m, slices, whole
# beams), the scalar-load stage 2 against the round-6 LDS one (HD_LIB A/B), slices re-timed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_q8m.py \
    tests/test_gpu_slices.py tests/test_gpu_wholebeam.py tests/test_gpu_qp.py > gpurun_out/r6h_tests.log 2>&1 || exit 1
bash scripts/ab_env.sh HD_LIB=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_s2d.so > gpurun_out/r6h_ab.txt 2>&1 || exit 2
rm -f gpurun_out/r6h_simslice.jsonl
for s in 0/8 7/8; do
  timeout -k 10 300 python3 bench.py --mode slices --sim-slice $s --steps 5 --warmup 2 $L > gpurun_out/r6h_sim.log 2>&1 || exit 3
  tail -1 gpurun_out/r6h_sim.log >> gpurun_out/r6h_simslice.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6h_prof_0o8 -o run -- python3 bench.py --mode slices \
    --sim-slice 0/8 --steps 3 --warmup 1 $L > gpurun_out/r6h_prof_0o8.log 2>&1 || exit 4
python3 scripts/kstats.py "$(find gpurun_out/r6h_prof_0o8 -name '*.db' | head -1)" gpurun_out/r6h_kstats_0o8.csv
