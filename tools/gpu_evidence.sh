#!/bin/bash
# Round evidence in one GPU call: the full GPU parity suite, the default bench line (1080p headline, CPU
# baseline, end-to-end, 8K shard pass), the 4K QP32 line, a rocprofv3 kernel trace of a short bench, and
# the MC kernels in isolation (tools/mc_bench.py) at 4K / 1080p with their own kernel traces. Each GPU
# step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --stream ra2160_q32 --steps 10 --warmup 2 --no-cpu --shard-steps 0 > gpurun_out/bench_${TAG}_4k.json 2> gpurun_out/bench_${TAG}_4k.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --shard-steps 0 > gpurun_out/prof_$TAG.log 2>&1 &&
timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160_q32 > gpurun_out/mcb_$TAG.json 2>&1 &&
timeout -k 10 120 python -u tools/mc_bench.py --stream ra1080_q32 >> gpurun_out/mcb_$TAG.json 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/mcprof_$TAG -o run -- python3 tools/mc_bench.py --stream ra2160_q32 --reps 20 > /dev/null 2>&1
