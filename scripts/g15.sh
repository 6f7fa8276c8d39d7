cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/ab15.log
for kb in 40; do
  HD_FIX8_LDS_KB=$kb timeout -k 10 200 python scripts/ab_fix8.py >> gpurun_out/ab15.log 2>&1 || exit 1
done
