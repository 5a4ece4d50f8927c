#!/bin/bash
# k_mc block order A/B: dispatch order (default) vs XCD runs of R blocks vs whole-grid XCD runs:
# time (tools/mc_bench.py --all-stages) and HBM read bytes (FETCH_SIZE, one pass per variant).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04x}
mkdir -p $O
for V in ${VARIANTS:-new xr4 xr8 xr16 xsw}; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/${V}_$S.json || exit 1
  done
  VVCR_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_$V -o run -- python3 -u tools/mc_bench.py --stream ra2160l_q27 --reps 1 --all-stages > $O/pmc_$V.log 2>&1 || exit 1
done
