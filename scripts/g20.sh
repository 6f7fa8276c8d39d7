cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_parity.py -k "fft or dedisperse_job" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t20.log 2>&1 &&
timeout -k 10 500 python bench.py --no-cpu --e2e-beams 0 --sp-beams 0 > gpurun_out/b20.log 2>&1
