#!/bin/bash
# 16-row luma cells (MC_TALL_LUMA build): MC / decode tests on it, then MC timings against the default.
set -o pipefail
mkdir -p gpurun_out/r04o
VVCR_LIB=vvc_amd/libvvcr_tl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_decode_gpu.py -m gpu > gpurun_out/r04o/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04o/base_$S.json || exit 1
  for v in tl tl_ra3; do
    VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04o/${v}_$S.json || exit 1
  done
done
