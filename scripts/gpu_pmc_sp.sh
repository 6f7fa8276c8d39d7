#!/bin/bash
# PMC passes (SQ counters) over one beam's single-pulse leg: gpurun_out/pmcsp_summary.txt and
# gpurun_out/pmcsp.json.   COMMIT=<sha> bash scripts/gpu_pmc_sp.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/pmcsp && mkdir -p gpurun_out/pmcsp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --e2e-beams 0 --sp-beams 1 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcsp/$n -o $n --pmc "$@" -- $B \
    > gpurun_out/pmcsp/$n.log 2>&1 || { echo "pmc pass $n failed"; exit 1; }
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
run sq2 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM
run sq3 SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_ANY SQ_INSTS_VALU_ADD_F32 SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH
python3 scripts/pmc_summary.py gpurun_out/pmcsp --json gpurun_out/pmcsp.json --commit "${COMMIT:-unknown}" > gpurun_out/pmcsp_summary.txt
echo "pmcsp done"
