#!/bin/bash
# Texture-path counters of the MC kernels in isolation (tools/mc_bench.py, fused path, 4K QP32 stream):
# are k_mc's waves waiting on the address / data path (TA, TD, vector L1) rather than on HBM?
# One rocprofv3 run per pass (<= 2 TA, 2 TD, 4 TCP, 4 TCC, 8 SQ counters each), each under its own kill timer.
TAG=${1:-mcta}
export TMPDIR=/tmp
O=gpurun_out/pmcta_$TAG
mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 tools/mc_bench.py --stream ra2160l_q32 --reps 1 --all-stages > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_LATENCY &&
run b TA_ADDR_STALLED_BY_TD_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS TCP_TCC_READ_REQ_LATENCY TCC_HIT TCC_MISS &&
run c TA_TOTAL_WAVEFRONTS TA_FLAT_READ_WAVEFRONTS TD_LOAD_WAVEFRONT TD_COALESCABLE_WAVEFRONT TCP_TOTAL_READ TCP_TA_TCP_STATE_READ TCP_LFIFO_STALL_CYCLES TCP_RFIFO_STALL_CYCLES
python tools/pmc_table.py $O k_mc > $O/table.txt && cat $O/table.txt
