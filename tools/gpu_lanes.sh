#!/bin/bash
# Bench-line sweep of hardware queues x lanes (total:intra) x segments; one run each.
set -o pipefail
for cfg in ${CFGS:-"8:7:3:6" "8:7:3:8" "8:7:3:12" "8:8:4:8" "8:8:4:12" "12:10:5:12"}; do
  IFS=: read Q L I S <<< "$cfg"
  GPU_MAX_HW_QUEUES=$Q VVCR_LANES=$L VVCR_INTRA_LANES=$I timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --shard-steps 0 --e2e-threads 0 --segments $S > gpurun_out/lan_${Q}_${L}_${I}_${S}.json 2> gpurun_out/lan_${Q}_${L}_${I}_${S}.err || exit 1
done
