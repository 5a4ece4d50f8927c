#!/bin/bash
# Bench-line A/B: the default bench (no CPU baseline, no e2e / shard passes) under each setting of AB_ENVS
# (VAR=VALUE[,VAR=VALUE...], "base" = unchanged), interleaved twice. One JSON line per run into gpurun_out/bab_<tag>_<i>.json.
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
i=0
for pass in 1 2; do
  for e in base $AB_ENVS; do
    i=$((i + 1))
    if [ "$e" = base ]; then
      timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --shard-steps 0 --e2e-threads 0 > gpurun_out/bab_${TAG}_$i.json 2>/dev/null || exit 1
    else
      env ${e//,/ } timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --shard-steps 0 --e2e-threads 0 > gpurun_out/bab_${TAG}_$i.json 2>/dev/null || exit 1
    fi
    echo "$e" > gpurun_out/bab_${TAG}_$i.env
  done
done
