#!/bin/bash
# Bench-line sweep of hardware queues x lanes (total:intra) x segments x intra workgroups; one run each.
set -o pipefail
for cfg in ${CFGS:-"8:8:4:12:48" "8:8:4:12:32" "12:10:5:12:32" "12:10:6:12:32" "12:12:6:12:24"}; do
  IFS=: read Q L I S G <<< "$cfg"
  GPU_MAX_HW_QUEUES=$Q VVCR_LANES=$L VVCR_INTRA_LANES=$I VVCR_INTRA_WG=$G timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --shard-steps 0 --e2e-threads 0 --segments $S > gpurun_out/lan_${Q}_${L}_${I}_${S}_${G}.json 2> gpurun_out/lan_${Q}_${L}_${I}_${S}_${G}.err || exit 1
done
