#!/bin/bash
# SQ counter passes over the stage-0 stage-1 launch (scripts/probe_stage1.py), one
# rocprofv3 run per counter group (--kernel-trace only beside --pmc).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
B="python3 scripts/probe_stage1.py 0"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc1/$n -o $n --pmc "$@" -- $B \
    > gpurun_out/pmc1/$n.log 2>&1 || { echo "pmc pass $n failed"; exit 1; }
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
run b SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM
run c SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_ADD_F32
echo "pmc2 done"
