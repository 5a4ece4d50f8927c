#!/bin/bash
# k_mc split by the host into an inside-the-picture kernel and an edge kernel: MC / KAT / decode /
# bitstream / shard tests, then the MC timings (4K QP27 / QP32, plain and fused).
set -o pipefail
mkdir -p gpurun_out/r04n
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_mc_kat.py tests/test_decode_gpu.py tests/test_bitstream.py tests/test_shard_gpu.py -m gpu > gpurun_out/r04n/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04n/base_$S.json || exit 1
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04n/fused_$S.json || exit 1
done
