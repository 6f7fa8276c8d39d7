cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/ab17.log
for w in 0 1 0 1; do
  echo "HD_Q8_WIDE_STORES=$w" >> gpurun_out/ab17.log
  HD_Q8_WIDE_STORES=$w timeout -k 10 200 python scripts/ab_fix8.py >> gpurun_out/ab17.log 2>&1 || exit 1
done
