#!/bin/bash
# RDO inner loop on the box: parity tests, bench line, rocprofv3 kernel-trace summary
set -o pipefail
TAG=${1:-rdo}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench_rdo.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench_rdo.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
