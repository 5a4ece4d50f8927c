#!/bin/bash
# MC development pass: MC / decode parity tests, then the MC microbenchmark (tools/mc_run.sh).
set -o pipefail
TAG=${1:-m}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py tests/test_recon_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
bash tools/mc_run.sh $TAG
