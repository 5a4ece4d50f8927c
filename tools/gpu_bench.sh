#!/bin/bash
# The default bench line (what the driver runs at round end), its stderr log beside it.
set -o pipefail
T=${1:-bench}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py $BENCH_ARGS > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -30 gpurun_out/bench_$T.err; exit 1; }
tail -c 3000 gpurun_out/bench_$T.json
