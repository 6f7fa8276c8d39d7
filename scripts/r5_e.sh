#!/bin/bash
# Round-5 session e: the float4-store qp flush (HD_QP_FQ=1) bit-exact, then timed against the
# default and the pair kernel (HD_S2_QP=0); kernel stats; --comm hd at world 1 after the
# clip-stats copy fix; the qp probe sweep (stage-0 pass).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
HD_QP_FQ=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_qp.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r5e_qpvar.log 2>&1 || { echo "qp FQ failed"; tail -20 gpurun_out/r5e_qpvar.log; exit 1; }
echo "HD_QP_FQ=1: $(tail -1 gpurun_out/r5e_qpvar.log)"
bash scripts/ab_env.sh HD_S2_QP=0 HD_QP_FQ=1 || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 bench.py --mode slices --comm hd --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 \
    --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/r5e_commhd.log 2>&1 || { echo "comm hd failed"; tail -5 gpurun_out/r5e_commhd.log; exit 1; }
echo "comm hd: $(python3 scripts/benchline.py gpurun_out/r5e_commhd.log)"
timeout -k 10 300 python3 scripts/probe_stage2.py 0 --variant=9 --probes=0,1,2,4,8,6,9,14,13,11,7,15 \
    > gpurun_out/r5e_qp_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r5e_qp_probe.txt; exit 1; }
cat gpurun_out/r5e_qp_probe.txt
