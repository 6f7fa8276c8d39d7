#!/bin/bash
# round-6 closing, call 6: smoke, the whole -m gpu suite, the default bench line and kernel stats
# on the final build (expand at raised wave priority).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6fin4 TEST_TIMEOUT=900 BENCH=1 PROF=1 bash scripts/gpu_session.sh
