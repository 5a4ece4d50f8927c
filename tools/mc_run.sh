#!/bin/bash
# MC kernels in isolation on the GPU box (tools/mc_bench.py): 4K and 1080p, a rocprofv3 kernel trace of
# the 4K run, and the same runs with an A/B library (vvc_amd/libvvcr_old.so) when it is present.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160_q32 > gpurun_out/mcb_$1.json 2>&1 &&
timeout -k 10 120 python -u tools/mc_bench.py --stream ra1080_q32 >> gpurun_out/mcb_$1.json 2>&1 &&
if [ -f vvc_amd/libvvcr_old.so ]; then
  VVCR_LIB=vvc_amd/libvvcr_old.so timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160_q32 >> gpurun_out/mcb_$1.json 2>&1 &&
  VVCR_LIB=vvc_amd/libvvcr_old.so timeout -k 10 120 python -u tools/mc_bench.py --stream ra1080_q32 >> gpurun_out/mcb_$1.json 2>&1
fi &&
export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mcprof_$1 -o run -- python3 tools/mc_bench.py --stream ra2160_q32 --reps 20 > /dev/null 2>&1  &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mcprof1080_$1 -o run -- python3 tools/mc_bench.py --stream ra1080_q32 --reps 20 > /dev/null 2>&1
