#!/bin/bash
# Round-5 session f: k_stage2_qp with the two-iteration DMA lookahead (default) bit-exact, timed
# against HD_QP_DEEP=0; the stage-0 qp probe sweep; the stage-1 q8 / q8m phase probes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_qp.py tests/test_gpu_wholebeam.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r5f_qp.log 2>&1 || { echo "qp tests failed"; tail -20 gpurun_out/r5f_qp.log; exit 1; }
echo "qp + whole beam: $(tail -1 gpurun_out/r5f_qp.log)"
bash scripts/ab_env.sh HD_QP_DEEP=0 || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 scripts/probe_stage2.py 0 --variant=9 --probes=0,1,2,4,8,6,9,14,13,11,7,15 \
    > gpurun_out/r5f_qp_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r5f_qp_probe.txt; exit 1; }
cat gpurun_out/r5f_qp_probe.txt
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5f_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5f_q8m_probe.txt; exit 1; }
cat gpurun_out/r5f_q8m_probe.txt
