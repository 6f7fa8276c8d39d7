# Full GPU session: smoke, every -m gpu test, bench (default legs), rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 > gpurun_out/prof.log 2>&1 || { echo prof failed; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/prof -name '*.db' | head -1)" gpurun_out/kstats.csv
echo "done pytest_rc=$rc"
