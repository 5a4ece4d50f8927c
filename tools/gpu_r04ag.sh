#!/bin/bash
# k_alf: 1 / 2 / 4 regions per workgroup (consecutive, no prefetch): parity of the variants, time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ag
mkdir -p $O
for V in apw2 apw4; do
  VVCR_LIB=vvc_amd/libvvcr_$V.so timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_recon_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$V.log 2>&1 || exit 1
done
for V in new apw2 apw4 new apw2 apw4; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 --all-stages >> $O/${V}.jsonl || exit 1
done
