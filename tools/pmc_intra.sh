#!/bin/bash
# SQ counters of k_intra in isolation (tools/intra_bench.py): one rocprofv3 --pmc run per pass.
TAG=${1:-intra}
STREAM=${2:-ra1080_q32}
export TMPDIR=/tmp
O=gpurun_out/pmcin_$TAG
mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 tools/intra_bench.py --stream $STREAM --reps 3 > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run b SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU &&
run c SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_WAVE32
[ "$ICACHE" = "1" ] && run d SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES
