#!/bin/bash
# k_mc occupancy variants: list-0 rows in LDS (113 VGPRs), that at 5 waves per SIMD (96 VGPRs, spills),
# 5 waves per SIMD alone; MC tests on the LDS variant first.
set -o pipefail
mkdir -p gpurun_out/r04m
VVCR_LIB=vvc_amd/libvvcr_p0lds_w5.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_decode_gpu.py -m gpu > gpurun_out/r04m/pytest.log 2>&1 || exit 1
S=ra2160l_q27
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04m/base.json || exit 1
for v in p0lds p0lds_w5 w5; do
  VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04m/$v.json || exit 1
done
