#!/bin/bash
# A/B of hd_plan_set_variant values in the bench's own context (one beam, all 57 passes): each
# value under rocprofv3 --kernel-trace --stats, per-kernel averages into gpurun_out/abb_<v>.csv.
#   bash scripts/ab_bench.sh <variant> [<variant> ...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/abb_$v -o run -- python3 bench.py --steps 2 --warmup 1 \
      --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 --variant $v > gpurun_out/abb_$v.log 2>&1 \
      || { echo "variant $v failed"; exit 1; }
  python3 scripts/kstats.py "$(find gpurun_out/abb_$v -name '*.db' | head -1)" gpurun_out/abb_$v.csv
  echo "== variant $v"
  python3 scripts/kstats_grep.py gpurun_out/abb_$v.csv stage2 stage1 fix8
done
