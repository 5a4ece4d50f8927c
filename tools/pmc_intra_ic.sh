#!/bin/bash
# Instruction-cache and issue counters of k_intra on the 4K intra picture (tools/intra_bench.py).
export TMPDIR=/tmp
O=gpurun_out/pmci_${1:-a}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -f csv -d $O/ic -o run -- python3 -u tools/intra_bench.py --stream ra2160l_q27 --reps 2 > $O/ic.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -f csv -d $O/sq -o run -- python3 -u tools/intra_bench.py --stream ra2160l_q27 --reps 2 > $O/sq.log 2>&1
