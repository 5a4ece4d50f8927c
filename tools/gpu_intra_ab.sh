#!/bin/bash
# k_intra: decode / bitstream parity (intra-heavy streams), the 4K intra picture in isolation for the
# default library and VARIANTS (vvc_amd/libvvcr_<v>.so), then the per-step profile (tools/intra_prof.py).
set -o pipefail
T=${1:-intraab}
export TMPDIR=/tmp
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_bitstream.py tests/test_recon_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for V in new ${VARIANTS}; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra1080_q32; do
    VVCR_LIB=$L timeout -k 10 180 python -u tools/intra_bench.py --stream $S --reps 20 > $O/${V}_$S.json || exit 1
    echo "$V $S $(tail -c 300 $O/${V}_$S.json)"
  done
done
[ -n "$PROFILE" ] && { INTRA_PROF_PICS=1 timeout -k 10 300 python tools/intra_prof.py run ra2160l_q27 > $O/iprof.log 2>&1 || { tail -20 $O/iprof.log; exit 1; }; }
true
