#!/bin/bash
# k_intra A/B on the GPU box: tools/intra_bench.py for libvvcr.so and every vvc_amd/libvvcr_v*.so variant,
# interleaved twice (and the default library under each AB_ENVS setting); one JSON line per run into
# gpurun_out/iab_<tag>.json.
set -o pipefail
TAG=${1:-ab}
STREAM=${2:-ra1080_q32}
mkdir -p gpurun_out
OUT=gpurun_out/iab_$TAG.json
: > $OUT
for pass in 1 2; do
  for lib in vvc_amd/libvvcr.so vvc_amd/libvvcr_v*.so; do
    [ -f "$lib" ] || continue
    VVCR_LIB=$lib timeout -k 10 120 python -u tools/intra_bench.py --stream $STREAM >> $OUT 2>> gpurun_out/iab_$TAG.err || exit 1
  done
  for e in $AB_ENVS; do   # the default library under extra environment settings (VAR=VALUE ...)
    env $e AB_LABEL=$e timeout -k 10 120 python -u tools/intra_bench.py --stream $STREAM >> $OUT 2>> gpurun_out/iab_$TAG.err || exit 1
  done
done
