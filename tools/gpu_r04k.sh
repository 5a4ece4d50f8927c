#!/bin/bash
# MC / loop-filter checks after a kernel change: the MC, KAT, decode, loop-filter and bitstream GPU tests,
# then the MC kernels (plain and fused) and ALF timings on the 4K QP27 / QP32 streams.
set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_mc_kat.py tests/test_decode_gpu.py tests/test_lf_gpu.py tests/test_bitstream.py -m gpu > gpurun_out/r04k/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04k/base_$S.json || exit 1
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04k/fused_$S.json || exit 1
done
