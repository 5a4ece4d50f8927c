#!/bin/bash
# Kernel-level A/B: parity tests, then a rocprofv3 kernel trace of a short serial bench with the working
# library and with vvc_amd/libvvcr_old.so (tools/build_ab.sh), then the bench-line A/B (tools/gpu_bench_ab.sh).
set -o pipefail
TAG=${1:-kab}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kab_${TAG}_new -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --segments 1 --sync-pictures --shard-steps 0 --e2e-threads 0 > gpurun_out/kab_${TAG}_new.log 2>&1 &&
VVCR_LIB=vvc_amd/libvvcr_old.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kab_${TAG}_old -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --segments 1 --sync-pictures --shard-steps 0 --e2e-threads 0 > gpurun_out/kab_${TAG}_old.log 2>&1 &&
AB_ENVS="VVCR_LIB=vvc_amd/libvvcr_old.so" bash tools/gpu_bench_ab.sh $TAG
