#!/bin/bash
# Stage-1 split probe per DDplan stage, then an A/B of non-temporal series stores in stage 2.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/probe_s1_split.py > gpurun_out/s1_split.txt 2>&1 || { echo "s1 probe failed"; tail gpurun_out/s1_split.txt; exit 1; }
bash scripts/ab_env.sh HD_S2_NT=1 > gpurun_out/ab_nt.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_nt.txt; exit 1; }
cat gpurun_out/ab_nt.txt
echo "s1probe done"
