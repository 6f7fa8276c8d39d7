#!/bin/bash
# Per-kernel A/B of environment switches in the bench context: each setting under rocprofv3
# --kernel-trace --stats (bench.py, no legs), kernel averages matching the grep words.
#   WORDS="fix8 q8" bash scripts/ab_envk.sh "" "HD_FIX8_PROBE=1" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  d=gpurun_out/abk_$i
  env $e timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 2 --warmup 1 \
      --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > $d.log 2>&1 \
      || { echo "setting [$e] failed"; exit 1; }
  python3 scripts/kstats.py "$(find $d -name '*.db' | head -1)" $d.csv
  s=$(python3 scripts/benchline.py $d.log ms) || { echo "no bench line [$e]"; exit 1; }
  echo "== [$e] $s"
  python3 scripts/kstats_grep.py $d.csv ${WORDS:-fix8 transpose}
done
