#!/bin/bash
# round-6 closing, call 2: the qp parity tests and smoke of this build, the default bench line, kernel stats of the bench step, the 4-bit
# beam, and the PMC passes of the final kernels (-> profiles/pmc_r06.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    > gpurun_out/fin_qp_tests.log 2>&1 || { echo "qp tests failed"; exit 5; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { echo "smoke failed"; exit 6; }
timeout -k 10 600 python3 bench.py > gpurun_out/fin_bench.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run -- python3 bench.py --steps 3 --warmup 1 $L \
    > gpurun_out/fin_prof.log 2>&1 || { echo "prof failed"; exit 2; }
python3 scripts/kstats.py "$(find gpurun_out/fin_prof -name '*.db' | head -1)" gpurun_out/fin_kstats.csv
timeout -k 10 300 python3 bench.py --nbits 4 --steps 5 --warmup 2 $L > gpurun_out/fin_4bit.log 2>&1 || { echo "4-bit failed"; exit 3; }
COMMIT=$(cat COMMIT_ID 2>/dev/null) bash scripts/gpu_pmc.sh > gpurun_out/fin_pmc.txt 2>&1 || { echo "pmc failed"; exit 4; }
echo "final b done"
