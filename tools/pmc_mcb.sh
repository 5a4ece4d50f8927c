#!/bin/bash
# PMC passes over tools/mc_bench.py (the MC kernels alone): instruction-cache and wait counters.
# Usage: bash tools/pmc_mcb.sh STREAM TAG
S=${1:-ra2160l_q27}; TAG=${2:-a}
export TMPDIR=/tmp
O=gpurun_out/pmcb_$TAG
mkdir -p $O
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 -u tools/mc_bench.py --stream $S --reps 2 > $O/$n.log 2>&1
}
run ic SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM
