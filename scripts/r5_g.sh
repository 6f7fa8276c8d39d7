#!/bin/bash
# Round-5 session g: stage-1 pass delays through scalar loads (the pass loop no longer waits on
# the previous pass's stores): stage-1 parity, bench A/B of the qp DMA lookahead, q8/q8m probes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_q8m.py tests/test_gpu_wholebeam.py tests/test_gpu_qp.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r5g_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r5g_tests.log)"
bash scripts/ab_env.sh HD_QP_DEEP=0 || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5g_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5g_q8m_probe.txt; exit 1; }
cat gpurun_out/r5g_q8m_probe.txt
