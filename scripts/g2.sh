cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_4bit.py tests/test_gpu_clip.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --nbits 4 > gpurun_out/b4.log 2>&1
