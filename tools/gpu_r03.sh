#!/bin/bash
# r03 GPU pass: parity suite, default bench line (4K RA QP27, end-to-end headline + resident + CPU baseline
# + 8K shard), the 1080p line, rocprofv3 kernel trace of a short resident bench. Each GPU step has its own
# time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --stream ra1080_q32 --no-cpu --shard-steps 0 > gpurun_out/bench_${TAG}_1080.json 2> gpurun_out/bench_${TAG}_1080.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --resident-steps 5 --no-cpu --shard-steps 0 > gpurun_out/prof_$TAG.log 2>&1
