#!/bin/bash
# A/B of a loop-filter change: parity tests, then the bench's kernel table (resident pass, one segment) with
# the new library and vvc_amd/libvvcr_old.so, interleaved twice.
set -o pipefail
TAG=${1:-alf}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lf_gpu.py tests/test_decode_gpu.py tests/test_dropin_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 1
for rep in 1 2; do
  for v in new old; do
    L=; [ $v = old ] && L=vvc_amd/libvvcr_old.so
    VVCR_LIB=$L timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --resident-steps 10 --no-cpu --shard-steps 0 \
      > gpurun_out/kt_${TAG}_${v}_$rep.json 2> gpurun_out/kt_${TAG}_${v}_$rep.err || exit 1
  done
done
