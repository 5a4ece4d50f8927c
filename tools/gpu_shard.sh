#!/bin/bash
# Sharding pass: sharded-decode parity (emulated ranks) and the tiled streams unsharded, then the bench
# line (1080p replicas + end-to-end + the 8K sharded pass at this node's GPU count).
set -o pipefail
TAG=${1:-sh}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_decode_gpu.py -x -v --timeout 300 --timeout-method thread -k "shard or ratile" > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
