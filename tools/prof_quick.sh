#!/bin/bash
# Parity tests of the MC/decode paths, then a rocprofv3 kernel-trace of a short bench (first failure ends the call).
set -o pipefail
TAG=${1:-pq}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --segments 1 --sync-pictures > gpurun_out/prof_$TAG.log 2>&1
