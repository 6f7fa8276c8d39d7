#!/bin/bash
# round-6 session O: the channel-major copy's stores (k_raw_transpose) and k_stage1_q8's fill
# loads with the non-temporal hint (a second build through HD_LIB) -- q8m / parity tests of that
# build and the bench A/B against the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
NT=$GRAFT_REPO_ROOT/pipeline2.0_amd/ab/libhipdedisp_nt2.so
HD_LIB=$NT timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_q8m.py \
    > gpurun_out/r6o_tests.log 2>&1 || { echo "nt2 tests failed"; exit 1; }
bash scripts/ab_env.sh HD_LIB=$NT > gpurun_out/r6o_ab.txt 2>&1 || { echo "ab failed"; exit 2; }
cat gpurun_out/r6o_ab.txt
