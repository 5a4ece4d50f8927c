#!/bin/bash
# One GPU-box pass: parity tests, bench lines (1080p default config, 4K), rocprofv3 kernel-trace summary,
# PMC traffic and SQ instruction-mix passes. Each GPU step has its own time limit; steps are chained so
# that the first failure ends the call.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --stream ra2160_q27 > gpurun_out/bench4k_$TAG.json 2> gpurun_out/bench4k_$TAG.err &&
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --stream ra2160_q32 > gpurun_out/bench4k32_$TAG.json 2> gpurun_out/bench4k32_$TAG.err &&
timeout -k 10 300 python -u bench_rdo.py > gpurun_out/benchrdo_$TAG.json 2> gpurun_out/benchrdo_$TAG.err &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --segments 1 --sync-pictures > gpurun_out/prof_$TAG.log 2>&1 &&
bash tools/pmc.sh $TAG &&
bash tools/pmc_sq.sh $TAG
