#!/bin/bash
# closing bench line on the final tree
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04ai.json 2> gpurun_out/bench_r04ai.err
