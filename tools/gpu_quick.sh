#!/bin/bash
# Quick GPU pass: parity tests then a short bench (each step under its own time limit, first failure ends the call).
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
