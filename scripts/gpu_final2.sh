#!/bin/bash
# Round-end session, part 2: the default bench line, rocprofv3 kernel stats of the bench's
# timed steps and of one single-pulse leg (CSV).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python bench.py > gpurun_out/bench_final.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu \
    --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_final.log 2>&1 || { echo prof failed; exit 1; }
for f in $(find gpurun_out/prof_final -name "*kernel_stats.csv"); do cp "$f" gpurun_out/kernel_stats_final.csv; done
python3 scripts/benchline.py gpurun_out/prof_final.log || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final_sp -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu \
    --e2e-beams 0 --sp-beams 1 --fft-beams 0 --rfi-beams 0 --stream-beams 0 > gpurun_out/prof_final_sp.log 2>&1 || { echo prof sp failed; exit 1; }
for f in $(find gpurun_out/prof_final_sp -name "*kernel_stats.csv"); do cp "$f" gpurun_out/kernel_stats_final_sp.csv; done
echo "final2 done"
