#!/bin/bash
# k_alf block order: whole-grid XCD runs (default) vs XCD runs of R regions; time and HBM read bytes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
for V in new axr60 axr120 axr240; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 --all-stages > $O/${V}.json || exit 1
  VVCR_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_$V -o run -- python3 -u tools/mc_bench.py --stream ra2160l_q27 --reps 1 --all-stages > $O/pmc_$V.log 2>&1 || exit 1
done
