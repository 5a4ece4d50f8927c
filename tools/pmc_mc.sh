#!/bin/bash
# SQ counters of the MC kernels in isolation (tools/mc_bench.py, 4K): one rocprofv3 --pmc run per pass,
# each under its own kill timer; VVCR_LIB selects an A/B library.
TAG=${1:-mc}
STREAM=${2:-ra2160_q32}
export TMPDIR=/tmp
O=gpurun_out/pmcmc_$TAG
mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 tools/mc_bench.py --stream $STREAM --reps 3 > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run b SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU &&
run c GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum
[ "$EXTRA" = "1" ] && run d SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INSTS_SALU &&
[ "$EXTRA" = "1" ] && run e SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES
