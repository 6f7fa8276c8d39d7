cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mock.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "mock or gap or dedisperse_job or psrfits or stream" > gpurun_out/t12.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t12.log
[ $rc -eq 0 ]
