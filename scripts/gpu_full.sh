#!/bin/bash
# Full GPU session: gpu_session.sh (smoke, every -m gpu test, bench, kernel stats), then a
# 2-rank gloo rehearsal of the multi-rank bench path on the one GPU (the node runs RCCL).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_session.sh || exit 1
HD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/b_w2.log 2>&1 \
    || { echo "2-rank rehearsal failed"; exit 1; }
tail -1 gpurun_out/b_w2.log | cut -c1-300
echo "full done"
