#!/bin/bash
# r04: the whole GPU suite, the MC kernels in isolation on the 4K streams, then the default bench line.
set -o pipefail
TAG=${1:-b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
for s in ra2160l_q27 ra2160l_q32; do timeout -k 10 120 python -u tools/mc_bench.py --stream $s --reps 20 > gpurun_out/mcb_${TAG}_$s.json || exit 1; done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
