#!/bin/bash
# Round-5 session d: default vs HD_S2_QP=0 (per-ppc qp tables, q8m reverted), kernel stats,
# --comm hd at world 1 after the clip-stats copy fix, the qp probe sweep (stage-0 pass), the
# 8-wave qp (HD_QP_NW=8) and the restructured k_stage1_fix8.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
# the two qp variants must be bit-exact before they are timed
for e in HD_QP_NW=8 HD_QP_FQ=1; do
  env $e timeout -k 10 400 python -u -m pytest tests/test_gpu_qp.py -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/r5d_qpvar.log 2>&1 || { echo "qp variant $e failed"; tail -20 gpurun_out/r5d_qpvar.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/r5d_qpvar.log)"
done
bash scripts/ab_env.sh HD_S2_QP=0 HD_QP_NW=8 HD_QP_FQ=1 || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 bench.py --mode slices --comm hd --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 \
    --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/r5d_commhd.log 2>&1 || { echo "comm hd failed"; tail -5 gpurun_out/r5d_commhd.log; exit 1; }
echo "comm hd: $(python3 scripts/benchline.py gpurun_out/r5d_commhd.log)"
timeout -k 10 300 python3 scripts/probe_stage2.py 0 --variant=9 --probes=0,1,2,4,8,6,9,14,13,11,7,15 \
    > gpurun_out/r5d_qp_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r5d_qp_probe.txt; exit 1; }
cat gpurun_out/r5d_qp_probe.txt
