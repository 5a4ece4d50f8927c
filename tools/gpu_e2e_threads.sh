#!/bin/bash
# End-to-end sweep of host parser threads x decodes in flight on the default stream (20 steps each).
set -o pipefail
mkdir -p gpurun_out
for cfg in "16 16" "32 16" "32 24" "16 24"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --e2e-threads $1 --segments $2 --resident-steps 0 --no-cpu --shard-steps 0 \
    > gpurun_out/e2e_thr_t$1_s$2.json 2> gpurun_out/e2e_thr_t$1_s$2.err || exit 1
done
