#!/bin/bash
# r03 GPU pass b: the drop-in (DecoderApp linked with libvvcr), the parity suite, and an end-to-end sweep of
# decodes in flight (segments) x parser threads at steady state (steps >> segments) on the 33-picture
# 1080p RA stream. Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r03b}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_dropin_$TAG.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
for seg in 12 6 4; do
  timeout -k 10 240 python -u bench.py --stream ra1080l_q32 --steps 48 --warmup 4 --segments $seg --resident-steps 0 --no-cpu \
    --shard-steps 0 > gpurun_out/e2e_${TAG}_1080l_s$seg.json 2> gpurun_out/e2e_${TAG}_1080l_s$seg.err || exit 1
done
