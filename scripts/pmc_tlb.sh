#!/bin/bash
# Address-translation (UTCL1) and TA/TCP stall counters of the bench beam and of the
# single-plan A/B script (scripts/ab_stage2.py, stage 0), each pass its own rocprofv3 run.
#   bash scripts/pmc_tlb.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/tlb && mkdir -p gpurun_out/tlb
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
A="python3 scripts/ab_stage2.py 0 --probes=0 --reps=1"
run() {  # dir cmd counters...
  local n=$1 cmd=$2; shift 2
  timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlb/$n -o $n --pmc "$@" -- $cmd \
    > gpurun_out/tlb/$n.log 2>&1 || { echo "pmc pass $n failed"; exit 1; }
}
for w in bench ab; do
  if [ $w = bench ]; then cmd=$B; else cmd=$A; fi
  run ${w}_1 "$cmd" TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum
  run ${w}_2 "$cmd" TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
  run ${w}_3 "$cmd" TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
  mkdir -p gpurun_out/tlb/sum_$w && cp -r gpurun_out/tlb/${w}_* gpurun_out/tlb/sum_$w/ 2>/dev/null
  python3 scripts/pmc_summary.py gpurun_out/tlb/sum_$w > gpurun_out/tlb/summary_$w.txt
done
echo "tlb done"
