#!/bin/bash
# Round-end evidence on one GPU box: the GPU parity suite, the default bench line (the driver's command),
# a 1080p end-to-end line, a rocprofv3 kernel trace of a one-segment run of the same stream (kernel
# durations without overlap: the bench's roofline is taken the same way), and the PMC traffic passes.
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r03f}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --stream ra1080l_q32 --steps 20 --warmup 2 --resident-steps 10 --no-cpu --shard-steps 0 > gpurun_out/bench_${TAG}_1080l.json 2> gpurun_out/bench_${TAG}_1080l.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --segments 1 --resident-steps 5 --sync-pictures --no-cpu --shard-steps 0 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err &&
bash tools/pmc.sh $TAG
