#!/bin/bash
# round-6 session C: the 12-wave x 7-DM stage-2 variant (HD_QP_W12=1): parity, A/B, probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
HD_QP_W12=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_qp.py > gpurun_out/r6c_tests.log 2>&1 || exit 1
bash scripts/ab_env.sh HD_QP_W12=1 > gpurun_out/r6c_ab.txt 2>&1 || exit 2
HD_QP_W12=1 timeout -k 10 120 python scripts/probe_stage2.py 0 1 --variant=9 > gpurun_out/r6c_probe_w12.txt 2>&1 || exit 3
