cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_clip.py tests/test_gpu_4bit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t24.log 2>&1 &&
timeout -k 10 500 python bench.py --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 > gpurun_out/b24.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof24 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 > gpurun_out/prof24.log 2>&1
