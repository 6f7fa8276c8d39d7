#!/bin/bash
# One GPU call: bench (no CPU leg) under rocprofv3 kernel trace; summary CSV via kstats.py.
# usage: scripts/gpu_prof.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu "$@" \
    > gpurun_out/p_$tag.log 2>&1 || { echo "rocprof rc=$?" >> gpurun_out/p_$tag.log; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/prof_$tag -name '*.db' | head -1)" gpurun_out/k_$tag.csv
