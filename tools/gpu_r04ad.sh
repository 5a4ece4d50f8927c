#!/bin/bash
# k_mc knobs re-checked under the XCD-run block order (plain and fused, 4K RA QP27 / QP32)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
for V in new tall wg128 ra8 ra2; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > $O/${V}_base_$S.json || exit 1
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/${V}_fused_$S.json || exit 1
  done
done
