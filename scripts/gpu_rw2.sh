#!/bin/bash
# Round-4 stage-2 session 2: the GPR-index probe, then the register-window kernel's tests,
# the bench and the per-stage probes of variants 7 and 8.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/gi_probe > gpurun_out/gi_probe.txt 2>&1; echo "gi_probe rc=$?" >> gpurun_out/gi_probe.txt
cat gpurun_out/gi_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "stage2 or multipass or dual or own_stream or shorter or c1_config" > gpurun_out/rw_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rw_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -40 gpurun_out/rw_tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/rw_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/rw_bench.log; exit 1; }
python3 scripts/benchline.py gpurun_out/rw_bench.log
for v in 7 8; do
  timeout -k 10 200 python scripts/probe_stage2.py 0 1 2 3 4 5 --variant=$v --probes=0,1,8,9,15 > gpurun_out/rw_probe_$v.txt 2>&1 || { echo "probe $v failed"; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/rw_c2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rw_c2.log
[ $rc -eq 0 ] || { echo "c2 rc=$rc"; tail -40 gpurun_out/rw_c2.log; exit 1; }
echo "rw2 done"
