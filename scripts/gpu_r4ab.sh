#!/bin/bash
# Session r4ab: k_stage1_fix8 with each subband's delays on a 32-byte LDS boundary (the merged
# 10-delay ds_read_b128 was misaligned).  Stage-1 tests, bench x2, fixup kernel times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py tests/test_gpu_q8m.py tests/test_gpu_c4.py \
    tests/test_gpu_clip.py -m gpu -x -v --timeout 600 --timeout-method thread -k "stage1 or int8 or c2 or q8m or c4 or fix" \
    > gpurun_out/r4ab_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4ab_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r4ab_tests.log; exit 1; }
tail -2 gpurun_out/r4ab_tests.log
bash scripts/ab_args.sh "" > gpurun_out/ab_r4ab.txt 2>&1 || { cat gpurun_out/ab_r4ab.txt; exit 1; }
cat gpurun_out/ab_r4ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu \
    --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_ab.log 2>&1 || { echo prof failed; exit 1; }
f=$(find gpurun_out/prof_ab -name "*kernel_stats.csv" | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fix8" in r["Name"]:
        print("%-60s calls %4s ms/step %7.3f" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e6 / 7))
PY
echo "r4ab done"
