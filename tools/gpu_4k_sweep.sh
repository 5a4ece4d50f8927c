#!/bin/bash
# 4K (and 1080p) bench-line sweep of lanes : intra lanes : segments : k_intra workgroups (0 = the library's
# default), one run each; then the default bench (with the 8K shard pass) at 32 intra workgroups.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-8:5:12:32:ra2160_q32 10:6:12:32:ra2160_q32 12:7:12:32:ra2160_q32 10:6:12:24:ra2160_q32 10:6:12:32:ra1080_q32 12:7:12:32:ra1080_q32}; do
  IFS=: read L I S G ST <<< "$cfg"
  VVCR_LANES=$L VVCR_INTRA_LANES=$I VVCR_INTRA_WG=$G timeout -k 10 200 python -u bench.py --stream $ST --steps 10 --warmup 2 --no-cpu --shard-steps 0 --e2e-threads 0 --segments $S > gpurun_out/k4_${ST}_${L}_${I}_${S}_${G}.json 2> gpurun_out/k4_${ST}_${L}_${I}_${S}_${G}.err || exit 1
done
