cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_slices.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "slices or stream" > gpurun_out/t7.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t7.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --streams 1 > gpurun_out/bs1.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --streams 3 > gpurun_out/bs3.log 2>&1
