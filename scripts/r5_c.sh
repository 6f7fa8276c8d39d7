#!/bin/bash
# Round-5 session c: default (k_stage2_qp, q8m b64 reads) vs HD_S2_QP=0 in the bench context,
# per-kernel stats of the default, and a kernel trace of --mode slices --comm hd (world 1).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_env.sh HD_S2_QP=0 || exit 1
WORDS="stage2 q8m fix8 q8< transpose clip" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c_commhd -o run -- python3 bench.py --mode slices \
    --comm hd --steps 1 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 \
    > gpurun_out/r5c_commhd.log 2>&1 || { echo "comm hd trace failed"; tail -5 gpurun_out/r5c_commhd.log; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/r5c_commhd -name '*.db' | head -1)" gpurun_out/r5c_commhd.csv
head -8 gpurun_out/r5c_commhd.csv | cut -c1-150
echo "comm hd: $(python3 scripts/benchline.py gpurun_out/r5c_commhd.log)"
