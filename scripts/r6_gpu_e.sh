#!/bin/bash
# round-6 session E: scalar-cache pair-table loads in k_stage2_qp: parity, bench, stamps, probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_qp.py \
    tests/test_gpu_wholebeam.py -k "qp or 8bit" > gpurun_out/r6e_tests.log 2>&1 || exit 1
bash scripts/ab_env.sh > gpurun_out/r6e_ab.txt 2>&1 || exit 2
HD_S2_STAMPS=gpurun_out/stamps1.bin timeout -k 10 120 python scripts/probe_stage2.py 0 --variant=9 --probes=0 > gpurun_out/r6e_probe1.txt 2>&1 || exit 3
python3 scripts/qp_stamps.py gpurun_out/stamps1.bin > gpurun_out/r6e_stamps.txt 2>&1
timeout -k 10 120 python scripts/probe_stage2.py 0 1 --variant=9 > gpurun_out/r6e_probe.txt 2>&1 || exit 4
