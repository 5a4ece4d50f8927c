#!/bin/bash
# k_mc variants on the 4K streams (tools/mc_bench.py; --all-stages: the fused reconstruction jobs of the
# product path): workgroup size, rows ahead, residual prefetch distance, persistent grid.
set -o pipefail
mkdir -p gpurun_out/r04e
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/base_$S.json || exit 1
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04e/basefused_$S.json || exit 1
  for v in wg256 ra8; do
    VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/${v}_$S.json || exit 1
  done
  for v in wg256 res0 res4; do
    VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04e/${v}fused_$S.json || exit 1
  done
  VVCR_MC_WGS=4096 timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/wgs4096_$S.json || exit 1
done
timeout -k 10 150 python -u tools/mc_prof.py run ra2160l_q27 > gpurun_out/r04e/mcprof.txt 2>&1
