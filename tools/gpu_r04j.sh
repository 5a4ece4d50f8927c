#!/bin/bash
# k_mc ablations: job record only / no stores / no loads+filter / no loads+filter+stores (4K QP27 B pictures).
set -o pipefail
mkdir -p gpurun_out/r04j
S=ra2160l_q27
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04j/base.json || exit 1
for v in abl_exit abl_store abl_both abl_all3; do
  VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04j/$v.json || exit 1
done
