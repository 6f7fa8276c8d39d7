#!/bin/bash
# Session r4s: PMC refresh of the bench's kernels at the round's final code commit.
cd "$GRAFT_REPO_ROOT" || exit 1
COMMIT=6660531 bash scripts/gpu_pmc.sh || exit 1
head -60 gpurun_out/pmc_summary.txt
