#!/bin/bash
# Session r4j: in-library RCCL communicator (world 1) + slices through it; the sliced rank's
# time alone at G = 2 / 4 / 8 with the batched padding sums.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_slices.py tests/test_gpu_parity.py -m gpu -x -v -k "slices or comm or clip_stats" \
    --timeout 600 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4j_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4j_tests.log; exit 1; }
tail -2 gpurun_out/r4j_tests.log
timeout -k 10 300 python3 bench.py --mode slices --comm hd --steps 3 --warmup 1 --no-cpu > gpurun_out/slices_hdcomm.log 2>&1 \
    || { echo "slices hd comm failed"; tail -20 gpurun_out/slices_hdcomm.log; exit 1; }
python3 scripts/benchline.py gpurun_out/slices_hdcomm.log || exit 1
grep -o '"slice_exchanges": "[^"]*"' gpurun_out/slices_hdcomm.log
for g in 2 4 8; do
  timeout -k 10 200 python3 bench.py --mode slices --sim-slice 0/$g --steps 5 --warmup 2 --no-cpu > gpurun_out/simslice_$g.log 2>&1 \
      || { echo "sim-slice $g failed"; exit 1; }
  echo "G=$g: $(python3 scripts/benchline.py gpurun_out/simslice_$g.log)"
done
echo "r4j done"
