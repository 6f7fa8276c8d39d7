#!/bin/bash
# round-6 session F: the merged special-tile launch (parity), one-loader-wave DMA (parity + A/B),
# the no-DMA probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_q8m.py \
    tests/test_gpu_qp.py tests/test_gpu_wholebeam.py -k "q8m or qp or 8bit" > gpurun_out/r6f_tests.log 2>&1 || exit 1
HD_QP_LOADER=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    > gpurun_out/r6f_tests_loader.log 2>&1 || exit 2
bash scripts/ab_env.sh HD_QP_LOADER=1 HD_S1_SPMERGE=0 > gpurun_out/r6f_ab.txt 2>&1 || exit 3
timeout -k 10 120 python scripts/probe_stage2.py 0 --variant=9 --probes=0,2,1,8 > gpurun_out/r6f_probe.txt 2>&1 || exit 4
HD_QP_LOADER=1 timeout -k 10 120 python scripts/probe_stage2.py 0 --variant=9 --probes=0,2,1,8 > gpurun_out/r6f_probe_loader.txt 2>&1 || exit 5
