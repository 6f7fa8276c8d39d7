#!/bin/bash
# round-6 closing, call 1: smoke + the whole -m gpu suite (the driver's round-end check).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6fin TEST_TIMEOUT=1100 BENCH=0 PROF=0 bash scripts/gpu_session.sh
