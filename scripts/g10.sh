cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rfifind.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t10.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t10.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/rfi_time.py > gpurun_out/rfi10.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o rfi -- python scripts/rfi_time.py > gpurun_out/rfi10p.log 2>&1
