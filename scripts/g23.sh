cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t23.log 2>&1 &&
timeout -k 10 300 python scripts/fft_time.py > gpurun_out/fft23.log 2>&1
