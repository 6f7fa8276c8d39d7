cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_clip.py tests/test_gpu_4bit.py tests/test_gpu_c2.py tests/test_gpu_slices.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t9.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t9.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/probe_fixup.py > gpurun_out/pfix2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 > gpurun_out/b9.log 2>&1
