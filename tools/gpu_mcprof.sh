#!/bin/bash
# k_mc / k_mc_affine / k_mc_bidir per-dispatch durations (rocprofv3 kernel trace) of tools/mc_bench.py.
# Usage: bash tools/gpu_mcprof.sh STREAM TAG
S=${1:-ra2160l_q27}; TAG=${2:-a}
export TMPDIR=/tmp
O=gpurun_out/mcprof_$TAG
mkdir -p $O
timeout -k 10 150 rocprofv3 --kernel-trace --stats -f csv -d $O -o run -- python3 -u tools/mc_bench.py --stream $S --reps 3 > $O/mcb.json 2> $O/err.log
