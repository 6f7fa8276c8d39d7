#!/bin/bash
# Round-5 session l (after the tests): q8m with register-resident float folds and all-b64 even-ds
# reads -- timing, kernel stats, phase probes, the last time slice's kernel stats, then the PMC
# passes (profiles/pmc_r05.json).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_env.sh || exit 1
WORDS="stage2 q8m fix8 q8<" bash scripts/ab_envk.sh "" || exit 1
timeout -k 10 300 python3 scripts/probe_q8m.py > gpurun_out/r5l_q8m_probe.txt 2>&1 \
    || { echo "q8m probe failed"; tail -5 gpurun_out/r5l_q8m_probe.txt; exit 1; }
cat gpurun_out/r5l_q8m_probe.txt
L="--no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5l_prof78 -o run -- python3 bench.py --mode slices \
    --sim-slice 7/8 --steps 1 --warmup 1 $L > gpurun_out/r5l_prof78.log 2>&1 || { echo "prof 7/8 failed"; exit 1; }
python3 scripts/kstats.py "$(find gpurun_out/r5l_prof78 -name '*.db' | head -1)" gpurun_out/r5l_kstats78.csv
head -12 gpurun_out/r5l_kstats78.csv | cut -c1-150
COMMIT=${COMMIT:-unknown} bash scripts/gpu_pmc.sh || exit 1
grep -A30 "k_stage1_q8m" gpurun_out/pmc_summary.txt | head -32
