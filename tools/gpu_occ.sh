#!/bin/bash
# Occupancy ablation of the MC kernels: extra dynamic LDS per workgroup lowers the workgroups per CU;
# a latency-bound kernel slows in proportion. mc_bench.py at 4K and 1080p per setting.
set -o pipefail
mkdir -p gpurun_out
for X in 0 12000 30000 60000; do
  VVCR_MC_XLDS=$X VVCR_AFF_XLDS=$X timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160_q32 --reps 20 > gpurun_out/occ_4k_$X.json 2>&1 || exit 1
  VVCR_MC_XLDS=$X VVCR_AFF_XLDS=$X timeout -k 10 120 python -u tools/mc_bench.py --stream ra1080_q32 --reps 20 > gpurun_out/occ_1080_$X.json 2>&1 || exit 1
done
