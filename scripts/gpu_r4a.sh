#!/bin/bash
# Round-4 first session: the new parity tests, then the multi-rank slice driver rehearsed
# (2 gloo ranks on one GPU, union checked against a whole-beam run), then one rank's slice
# timed alone at G = 2, 4, 8 (per-rank compute behind DESIGN §7's prediction).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 1100 python -u -m pytest ${TESTS:-tests/test_bary.py tests/test_gpu_candidates.py tests/test_gpu_slices.py tests/test_gpu_prefetch.py tests/test_gpu_c4.py} \
    -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/gpu_tests_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r4a.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests_r4a.log; exit 1; }
HD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --mode slices --steps 2 --warmup 1 --check-union \
    > gpurun_out/slices_w2.log 2>&1 || { echo "slices rehearsal failed"; tail -20 gpurun_out/slices_w2.log; exit 1; }
for g in 2 4 8; do
  timeout -k 10 200 python bench.py --mode slices --sim-slice 0/$g --steps 5 --warmup 2 --no-cpu > gpurun_out/simslice_$g.log 2>&1 \
      || { echo "sim-slice $g failed"; exit 1; }
  timeout -k 10 200 python bench.py --mode slices --sim-slice $((g-1))/$g --steps 5 --warmup 2 --no-cpu > gpurun_out/simslice_last_$g.log 2>&1 \
      || { echo "sim-slice last $g failed"; exit 1; }
done
timeout -k 10 200 python scripts/probe_stage2.py 0 --probes=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 > gpurun_out/probe_s2_r4.txt 2>&1 || { echo probe failed; exit 1; }
echo "r4a done"
