#!/bin/bash
# r04: parity of the MC / decode / bitstream / shard paths, then the MC kernels in isolation on the 4K streams.
set -o pipefail
TAG=${1:-a}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_mc_gpu.py tests/test_mc_kat.py tests/test_lf_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py tests/test_shard_gpu.py tests/test_shard_mp_gpu.py tests/test_dropin_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
for s in ra2160l_q27 ra2160l_q32; do timeout -k 10 120 python -u tools/mc_bench.py --stream $s --reps 20 > gpurun_out/mcb_${TAG}_$s.json || exit 1; done
