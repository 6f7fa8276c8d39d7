#!/bin/bash
# PMC passes (each its own rocprofv3 run; counters only with --kernel-trace, never with sys/runtime traces).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/sq -o sq \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  -- $B > gpurun_out/pmc/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/sq2 -o sq2 \
  --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM \
  -- $B > gpurun_out/pmc/sq2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/fetch -o fetch --pmc FETCH_SIZE \
  -- $B > gpurun_out/pmc/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/write -o write --pmc WRITE_SIZE \
  -- $B > gpurun_out/pmc/write.log 2>&1
echo "pmc rc=$?"
