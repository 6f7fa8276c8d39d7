#!/bin/bash
# Single-pulse leg kernel times under environment settings (e.g. HD_SP_PROBE bits: 1 no
# prune walk, 2 no width-1 hits, 4 no boxcar hits; results invalid under a probe).
#   bash scripts/ab_sp.sh "" HD_SP_PROBE=1 ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  d=gpurun_out/absp_$i
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 1 --warmup 1 \
      --no-cpu --e2e-beams 0 --sp-beams 1 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > $d.log 2>&1 \
      || { echo "setting [$e] failed"; exit 1; }
  python3 scripts/kstats.py "$(find $d -name '*.db' | head -1)" $d.csv
  echo "== [$e]"
  python3 scripts/kstats_grep.py $d.csv k_sp
done
