cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fft.py "tests/test_gpu_parity.py::test_search_stage_dedisperse_job" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t11.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t11.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/fft_time.py > gpurun_out/fft11.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o fft -- python scripts/fft_time.py > gpurun_out/fft11p.log 2>&1
