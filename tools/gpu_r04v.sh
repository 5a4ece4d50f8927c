#!/bin/bash
# k_alf timing ablations (diagnostics builds: no classification sums / no luma taps / no chroma / none)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
for V in new ablc abll ablch ablall; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 --all-stages > $O/${V}.json || exit 1
done
