#!/bin/bash
# k_alf chroma: two positions of one component per lane (default) vs one position of both components
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_recon_gpu.py tests/test_bitstream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for V in new acp0 new acp0; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages >> $O/${V}_$S.jsonl || exit 1
  done
done
