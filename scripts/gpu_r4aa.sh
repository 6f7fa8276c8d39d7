#!/bin/bash
# Session r4aa: stage-2 stream overlap A/B in the bench context (--streams 1 / 2 / 3).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_args.sh "" "--streams 2" "--streams 3" > gpurun_out/ab_r4aa.txt 2>&1 || { cat gpurun_out/ab_r4aa.txt; exit 1; }
cat gpurun_out/ab_r4aa.txt
