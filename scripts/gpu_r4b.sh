#!/bin/bash
# Session r4b: the fused stage-1 tests + A/B + kernel stats, then the single-pulse split.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_q8m.sh || exit 1
bash scripts/gpu_sp.sh || exit 1
echo "r4b done"
