#!/bin/bash
# k_mc knobs after the edge-class split: no XCD swizzle, rows of loads in flight 3 / 6, residual prefetch 0.
set -o pipefail
mkdir -p gpurun_out/r04p
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04p/base_$S.json || exit 1
  for v in noswz ra3 ra6; do
    VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04p/${v}_$S.json || exit 1
  done
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04p/basefused_$S.json || exit 1
  VVCR_LIB=vvc_amd/libvvcr_res0.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04p/res0fused_$S.json || exit 1
done
