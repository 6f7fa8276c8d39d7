cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in 5 6 7; do timeout -k 10 300 python scripts/probe_stage2.py 0 1 2 3 4 5 --variant=$v --probes=0 || exit 1; done > gpurun_out/pr_all.log 2>&1
