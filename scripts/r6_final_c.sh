#!/bin/bash
# round-6 closing, call 3: smoke, the whole -m gpu suite and the default bench line on the
# closing build (its roofline traffic from the committed profiles/pmc_r06.json).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6fin2 TEST_TIMEOUT=950 BENCH=1 PROF=0 bash scripts/gpu_session.sh
