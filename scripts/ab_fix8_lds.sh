#!/bin/bash
# A/B of k_stage1_fix8's LDS cap (HD_FIX8_LDS_KB) in the bench context: per-stage fixup times.
cd "$GRAFT_REPO_ROOT" || exit 1
for kb in "$@"; do
  HD_FIX8_LDS_KB=$kb bash scripts/ab_bench.sh 0 > gpurun_out/abf_$kb.txt 2>&1 || exit 1
  echo "== $kb KiB"; grep fix8 gpurun_out/abf_$kb.txt
done
