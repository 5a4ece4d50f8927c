#!/bin/bash
# VALU issue counters of the MC kernels alone (tools/mc_bench.py): cycles per VALU instruction, busy cycles.
S=${1:-ra2160l_q27}; TAG=${2:-a}
export TMPDIR=/tmp
O=gpurun_out/pmcb2_$TAG
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -f csv -d $O/v -o run -- python3 -u tools/mc_bench.py --stream $S --reps 2 > $O/v.log 2>&1
