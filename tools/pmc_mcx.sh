#!/bin/bash
# Instruction-fetch and issue counters of the MC kernels in isolation (tools/mc_bench.py, fused path, 4K
# QP32 stream): is a wave waiting for instructions (code size vs the instruction cache) or for issue?
# One rocprofv3 run per pass, each under its own kill timer; the available counters listed first.
TAG=${1:-mcx}
export TMPDIR=/tmp
O=gpurun_out/pmcx_$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 tools/mc_bench.py --stream ra2160l_q32 --reps 1 --all-stages > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU &&
run b SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
