#!/bin/bash
# SQ instruction-mix / stall counters per kernel (two passes, one rocprofv3 run each, own kill timers)
TAG=${1:-sq}
export TMPDIR=/tmp
O=gpurun_out/pmcsq_$TAG
mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --segments 1 --sync-pictures > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run b SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
