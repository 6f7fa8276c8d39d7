#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace (+stats).
# Every GPU step has its own time limit; the script stops at the first crash or timeout.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-3}
TESTS=${TESTS:-tests}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit 1; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1
echo "done rc=$? pytest_rc=$rc"
