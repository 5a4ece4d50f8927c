#!/bin/bash
# k_mc variants on the 4K streams: rows-ahead builds and persistent grid sizes (tools/mc_bench.py).
set -o pipefail
mkdir -p gpurun_out/r04e
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/base_$S.json || exit 1
  for v in ra6 ra8; do
    VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/${v}_$S.json || exit 1
  done
  for g in 1024 2048 3072; do
    VVCR_MC_WGS=$g timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04e/wgs${g}_$S.json || exit 1
  done
done
