#!/bin/bash
# End-to-end sweep at steady state (steps >> segments): bench.py --stream S --segments N for each pair
# "S:N" given; one JSON line per run under gpurun_out/. Each run has its own time limit; the first
# failure ends the call.   tools/gpu_e2e.sh TAG ra1080l_q32:12 ra2160_q27:12 ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for sn in "$@"; do
  s=${sn%%:*}; n=${sn##*:}
  timeout -k 10 300 python -u bench.py --stream $s --steps ${STEPS:-10} --warmup ${WARMUP:-2} --segments $n --resident-steps 0 --no-cpu \
    --shard-steps 0 > gpurun_out/e2e_${TAG}_${s}_s$n.json 2> gpurun_out/e2e_${TAG}_${s}_s$n.err || exit 1
done
