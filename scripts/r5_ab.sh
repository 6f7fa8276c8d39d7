#!/bin/bash
# Round-5 A/B: the quarter-layout stage 2 (HD_S2_QP=1) against the pair kernel in the bench
# context, ms per step, then per-kernel stats of both; the in-library communicator at world 1.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/ab_env.sh HD_S2_QP=1 || exit 1
WORDS="stage2 q8m fix8" bash scripts/ab_envk.sh "" HD_S2_QP=1 || exit 1
timeout -k 10 300 python3 bench.py --mode slices --comm hd --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 \
    --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/r5_commhd.log 2>&1 || { echo "comm hd failed"; tail -5 gpurun_out/r5_commhd.log; exit 1; }
echo "comm hd: $(python3 scripts/benchline.py gpurun_out/r5_commhd.log)"
# configs[4] rehearsal: 2 beams on 3 gloo ranks sharing this GPU (2 home ranks, 1 helper), union check
HD_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --mode pointing --beams 2 --nspec 1048576 --check-union \
    --steps 2 --warmup 1 > gpurun_out/r5_pointing_w3.log 2>&1 || { echo "pointing rehearsal failed"; tail -20 gpurun_out/r5_pointing_w3.log; exit 1; }
grep -o '"union_check": {[^}]*}' gpurun_out/r5_pointing_w3.log | cut -c1-200
# the production 4-bit beam at HEAD
timeout -k 10 300 python3 bench.py --nbits 4 --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 \
    --rfi-beams 0 --stream-beams 0 > gpurun_out/r5_bench4.log 2>&1 || { echo "4-bit bench failed"; exit 1; }
echo "4-bit: $(python3 scripts/benchline.py gpurun_out/r5_bench4.log)"
