#!/bin/bash
# After the k_mc defaults change: MC / KAT / decode / bitstream / shard / drop-in tests, MC timings, the
# bench line and the one-segment rocprof trace.
set -o pipefail
TAG=r04r
export TMPDIR=/tmp
mkdir -p gpurun_out/r04r
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04r/base_$S.json || exit 1
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04r/fused_$S.json || exit 1
done
VVCR_LIB=vvc_amd/libvvcr_alfnoswz.so timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 --all-stages > gpurun_out/r04r/alfnoswz_ra2160l_q27.json || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --segments 1 --resident-steps 5 --sync-pictures --no-cpu --shard-steps 0 --single-steps 0 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
