#!/bin/bash
# The bench's kernel table (median of synced one-segment steps) of the headline stream and the
# north-star stream, then the same steps under rocprofv3, one kernel trace per stream with marker kernels
# around the steps (VVCR_TRACE_MARKERS=1): tools/kt_trace.py cuts exactly the kernel-table launches out
# of the trace, so its per-kernel averages check the table's medians. SYNC=picture|step (KT_ARGS: more).
set -o pipefail
TAG=${1:-kt}
SYNC=${SYNC:-picture}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 --kernel-table-sync $SYNC $KT_ARGS > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  P=gpurun_out/prof_kt_${TAG}_$S
  VVCR_TRACE_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $P -o run -- python3 -u bench.py --kernel-table-only --kernel-table-reps 7 --kernel-table-sync $SYNC $KT_ARGS --stream $S --north-star-stream "" > $P.json 2> $P.err || exit 1
  python tools/kt_trace.py $P/run_kernel_trace.csv --alg $P.json > $P.summary.json || exit 1
done
