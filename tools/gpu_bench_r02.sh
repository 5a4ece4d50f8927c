#!/bin/bash
# Round-2 evidence run: default bench (1080p headline, cpu baseline, e2e, shard pass), the 4K QP32 line, and a
# rocprofv3 kernel-trace of a short bench; each step under its own limit, the first failure ends the call.
set -o pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 300 python -u bench.py --stream ra2160_q32 --steps 10 --warmup 2 --no-cpu --shard-steps 0 > gpurun_out/bench_${TAG}_4k.json 2> gpurun_out/bench_${TAG}_4k.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --shard-steps 0 > gpurun_out/prof_${TAG}.log 2>&1
