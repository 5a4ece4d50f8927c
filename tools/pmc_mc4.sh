#!/bin/bash
# r04: counters of the MC kernels in isolation (tools/mc_bench.py), one rocprofv3 --pmc pass per group
TAG=${1:-mc}
STREAM=${2:-ra2160l_q27}
export TMPDIR=/tmp
O=gpurun_out/pmcmc_$TAG
mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 tools/mc_bench.py --stream $STREAM --reps 2 > $O/$n.log 2>&1
}
rocprofv3 --list-avail > $O/avail.txt 2>&1
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run b SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_SMEM SQ_WAVES &&
run c GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum &&
run d TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_BUSY_avr TCP_PENDING_STALL_CYCLES_sum
python3 tools/pmc_dump.py $O/a $O/b $O/c $O/d > $O/summary.txt
