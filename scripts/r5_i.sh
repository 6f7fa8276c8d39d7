#!/bin/bash
# Round-5 session i (after the tests): bench A/B context, kernel stats, then the PMC passes of
# one bench beam (scripts/gpu_pmc.sh) for profiles/pmc_r05.json.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_env.sh || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
COMMIT=${COMMIT:-unknown} bash scripts/gpu_pmc.sh || exit 1
head -60 gpurun_out/pmc_summary.txt
