#!/bin/bash
# The bench's kernel table (median of synced one-segment steps) of the headline stream and the
# north-star stream, then the same steps under rocprofv3 with --selected-regions, one trace per stream:
# each trace holds exactly the kernel-table steps, so its per-kernel averages check the table's medians.
set -o pipefail
TAG=${1:-kt}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err &&
for S in ra2160l_q27 ra2160l_q32; do
  VVCR_ROCTX_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --selected-regions -f csv -d gpurun_out/prof_kt_${TAG}_$S -o run -- python3 -u bench.py --kernel-table-only --kernel-table-reps 7 --stream $S --north-star-stream "" > gpurun_out/prof_kt_${TAG}_$S.json 2> gpurun_out/prof_kt_${TAG}_$S.err || exit 1
done
