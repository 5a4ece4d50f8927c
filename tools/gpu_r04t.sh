#!/bin/bash
# ALF rework A/B (staging via scalar loads, classification fused into the filter lanes, b64 coefficients):
# parity of the loop-filter / reconstruction tests, k_alf A/B against HEAD (libvvcr_old.so) and the
# uncapped-VGPR variant, phase stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04t}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_recon_gpu.py tests/test_bitstream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  for V in old new alfw1; do
    L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/${V}_$S.json || exit 1
  done
done
timeout -k 10 120 python -u tools/alf_prof.py run ra2160l_q27 > $O/alfprof.txt 2>&1
