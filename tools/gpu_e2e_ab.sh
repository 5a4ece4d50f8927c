#!/bin/bash
# End-to-end bench A/B on one box: the working tree's libvvcr against vvc_amd/libvvcr_old.so
# (tools/build_ab.sh), interleaved. STREAM (default ra1080l_q32), PASSES (default 2).
set -o pipefail
S=${STREAM:-ra1080l_q32}
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
  for v in new old; do
    if [ $v = old ]; then L="VVCR_LIB=$PWD/vvc_amd/libvvcr_old.so"; else L=""; fi
    env $L timeout -k 10 200 python -u bench.py --stream $S --steps 32 --warmup 2 --no-cpu > gpurun_out/eab_${S}_${v}_$pass.json 2> gpurun_out/eab_${S}_${v}_$pass.err || exit 1
  done
done
