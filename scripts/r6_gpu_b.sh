#!/bin/bash
# round-6 session B: staging-ring depth A/B in the bench context, stage-0 probes at NS=4,
# then the PMC passes of one bench beam.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/ab_env.sh HD_QP_NS=4 > gpurun_out/r6b_ab.txt 2>&1 || exit 1
HD_QP_NS=4 timeout -k 10 120 python scripts/probe_stage2.py 0 --variant=9 > gpurun_out/r6b_probe_ns4.txt 2>&1 || exit 2
COMMIT=$(cat COMMIT_ID 2>/dev/null) bash scripts/gpu_pmc.sh > gpurun_out/r6b_pmc.txt 2>&1 || exit 3
