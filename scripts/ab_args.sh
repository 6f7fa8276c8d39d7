#!/bin/bash
# A/B of bench.py arguments in the bench context (no legs), 2 reps each:
#   bash scripts/ab_args.sh "" "--streams 2" ...
cd "$GRAFT_REPO_ROOT" || exit 1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
for x in "$@"; do
  for rep in 1 2; do
    timeout -k 10 300 $B $x > gpurun_out/aba.log 2>&1 || { echo "bench failed ($x)"; exit 1; }
    echo "[$x] $(tail -1 gpurun_out/aba.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f ms/step, stage1 %.2f, stage2 %.2f" % (d["ms_per_step"], d["kernel_ms_per_step"]["stage1"], d["kernel_ms_per_step"]["stage2"]))')"
  done
done
