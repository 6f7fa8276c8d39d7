#!/bin/bash
# Round-5 session j (after the tests): software-pipelined q8m reads -- timing, kernel stats and
# the stage-1 phase probes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_env.sh || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5j_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5j_q8m_probe.txt; exit 1; }
cat gpurun_out/r5j_q8m_probe.txt
