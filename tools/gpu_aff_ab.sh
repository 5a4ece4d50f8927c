#!/bin/bash
# Affine A/B: MC / decode parity with the working library, then tools/mc_bench.py at 4K and 1080p with
# the libraries in $LIBS (default: the working library and vvc_amd/libvvcr_old.so, the baseline).
set -o pipefail
TAG=${1:-aff}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
for L in ${LIBS:-vvc_amd/libvvcr.so vvc_amd/libvvcr_old.so}; do
  VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160_q32 --reps 20 >> gpurun_out/mcab_$TAG.json 2>&1 || exit 1
  VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream ra1080_q32 --reps 20 >> gpurun_out/mcab_$TAG.json 2>&1 || exit 1
done
