#!/bin/bash
# Sweep of execution lanes (total:intra) x segments in flight for the 1080p bench line (one bench run
# each), with HQW hardware queues (default 16: every lane stream on its own queue).
set -o pipefail
HQW=${HQW:-16}
for cfg in ${CFGS:-"7:3:4" "8:4:4" "8:4:5" "9:5:5" "9:4:5" "10:5:6"}; do
  IFS=: read L I S <<< "$cfg"
  GPU_MAX_HW_QUEUES=$HQW VVCR_LANES=$L VVCR_INTRA_LANES=$I timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --shard-steps 0 --e2e-threads 0 --segments $S > gpurun_out/seg_${L}_${I}_${S}.json 2> gpurun_out/seg_${L}_${I}_${S}.err || exit 1
done
