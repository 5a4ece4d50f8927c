#!/bin/bash
# kernel trace of the pipelined bench (2 segments in flight): overlap analysis (tools/overlap.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace_${1:-seg} -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu --segments 2 > gpurun_out/trace_${1:-seg}.log 2>&1
