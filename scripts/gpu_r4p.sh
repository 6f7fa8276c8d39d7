#!/bin/bash
# Session r4p: k_sp_blocks sort on int keys, fully unrolled (med3 across lanes, complemented
# keys for descending lanes); k_sp_hits bitmask four ballots per trip.  SP tests, SP leg
# timing (2 beams), phase clocks, SP probes 0/1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_candidates.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4p_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 --sp-beams 2 > gpurun_out/r4p_spleg.log 2>&1 \
    || { echo "sp leg failed"; tail -20 gpurun_out/r4p_spleg.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r4p_spleg.log"):
    if l.startswith("{"):
        print("single_pulse", json.dumps(json.loads(l).get("single_pulse"))[:300])
PY
HD_SP_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 --sp-beams 1 > gpurun_out/spstats.log 2> gpurun_out/spstats.err \
    || { echo "stats run failed"; tail -20 gpurun_out/spstats.err; exit 1; }
PROBES="0 1" bash scripts/gpu_spprobe.sh || exit 1
echo "r4p done"
