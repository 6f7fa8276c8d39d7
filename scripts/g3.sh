cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stage2" > gpurun_out/t5.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t5.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/probe_stage2.py 0 3 --variant=6 --probes=0,1,8,9 > gpurun_out/pr6.log 2>&1 &&
timeout -k 10 300 python scripts/probe_stage2.py 0 3 --variant=7 --probes=0,1,8,9 > gpurun_out/pr7.log 2>&1
