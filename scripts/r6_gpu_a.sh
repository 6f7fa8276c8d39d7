#!/bin/bash
# round-6 session A: the new qp / teardown tests, whole-beam 8- and 4-bit parity, bench,
# stage-2 probes.  Each GPU step under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
    tests/test_gpu_qp.py tests/test_gpu_teardown.py tests/test_gpu_wholebeam.py > gpurun_out/r6a_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r6a_bench.log 2>&1 || exit 2
timeout -k 10 120 python scripts/probe_stage2.py 0 1 --variant=9 > gpurun_out/r6a_probe.txt 2>&1 || exit 3
