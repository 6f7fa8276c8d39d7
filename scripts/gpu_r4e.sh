#!/bin/bash
# Session r4e: single-pulse tests with the pooled search buffers and the SP leg timing, then
# the fused fixup kernel's split (HD_FIX8_PROBE 1: no folds, 2: no windows, 3: neither) in
# the bench context (stage-1 ms; the probe runs' outputs are not valid).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_single_pulse.py tests/test_gpu_slices.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4e_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
for b in 2 3; do
  HD_SP_TIMING=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --fft-beams 0 --rfi-beams 0 \
      --stream-beams 0 --sp-beams $b > gpurun_out/sp_b$b.log 2>&1 || { echo "sp bench failed"; tail -20 gpurun_out/sp_b$b.log; exit 1; }
  python3 -c "
import json,sys
t=open('gpurun_out/sp_b$b.log').read().splitlines()
d=next(json.loads(l) for l in t if l.startswith('{'))
print('sp beams $b:', d['single_pulse'], [l for l in t if l.startswith('hd_single_pulse:')])" || exit 1
done
bash scripts/ab_env.sh HD_FIX8_PROBE=1 HD_FIX8_PROBE=2 HD_FIX8_PROBE=3 > gpurun_out/ab_fix8probe.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_fix8probe.txt; exit 1; }
cat gpurun_out/ab_fix8probe.txt
echo "r4e done"
