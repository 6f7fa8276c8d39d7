#!/bin/bash
# Round-5 session m (after the tests): q8m unrolled float fold (default read2 vs HD_Q8M_B64=1),
# k_stage2_qp with host-built expand items -- timing, kernel stats, probes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_env.sh HD_Q8M_B64=1 || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5m_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5m_q8m_probe.txt; exit 1; }
cat gpurun_out/r5m_q8m_probe.txt
timeout -k 10 300 python3 scripts/probe_stage2.py 0 --variant=9 --probes=0,1,2,4,8,6,14,13,11,7,15 \
    > gpurun_out/r5m_qp_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r5m_qp_probe.txt; exit 1; }
cat gpurun_out/r5m_qp_probe.txt
