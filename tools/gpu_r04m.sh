#!/bin/bash
# MC / DMVR tests on the default build (8-row chroma cells, no persistent path, parallel DMVR minimum),
# then k_mc variants: 4-row chroma cells, list-0 rows in LDS (and at 5 waves per SIMD).
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_mc_kat.py tests/test_decode_gpu.py tests/test_bitstream.py -m gpu > gpurun_out/r04m/pytest.log 2>&1 || exit 1
S=ra2160l_q27
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04m/base.json || exit 1
for v in notall p0lds p0lds_w5; do
  VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04m/$v.json || exit 1
done
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04m/base2.json || exit 1
