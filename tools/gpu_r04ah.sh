#!/bin/bash
# k_mc_affine occupancy hint: waves_per_eu 8 (50 VGPRs, 63 SGPR spills) vs 6 (57 VGPRs, 26 SGPR spills)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
VVCR_LIB=vvc_amd/libvvcr_aw6.so timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_recon_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_aw6.log 2>&1 || exit 1
for V in new aw6 new aw6; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages >> $O/${V}_$S.jsonl || exit 1
  done
done
