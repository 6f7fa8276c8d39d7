#!/bin/bash
# round-6 closing, call 4: smoke, the whole -m gpu suite and the default bench line on the final
# build (non-temporal stage-1 stores).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6fin3 TEST_TIMEOUT=950 BENCH=1 PROF=0 bash scripts/gpu_session.sh
