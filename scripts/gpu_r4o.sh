#!/bin/bash
# Session r4o: single-pulse walk as one flat loop per lane (batches of 8 hits tested against
# the moving pivot); SP tests, per-workgroup phase clocks (HD_SP_STATS), SP timing, SQ counters.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4o_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
HD_SP_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 --sp-beams 1 > gpurun_out/spstats.log 2> gpurun_out/spstats.err \
    || { echo "stats run failed"; tail -20 gpurun_out/spstats.err; exit 1; }
PROBES="0 1" bash scripts/gpu_spprobe.sh || exit 1
bash scripts/gpu_pmc_sp.sh || exit 1
cat gpurun_out/pmcsp_summary.txt
echo "r4o done"
