#!/bin/bash
# Round-end session: smoke + the whole -m gpu suite (gpu_final.sh), then the default bench
# line and kernel stats (gpu_final2.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_final.sh || exit 1
bash scripts/gpu_final2.sh || exit 1
