cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_single_pulse.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t6.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python scripts/sp_time.py > gpurun_out/sp_time.log 2>&1
