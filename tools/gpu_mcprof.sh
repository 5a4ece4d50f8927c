#!/bin/bash
# Per-wave timestamps of k_mc (VVCR_MC_PROF build, tools/mc_prof.py build) on the 4K QP32 / QP27 B pictures.
set -o pipefail
TAG=${1:-mcprof}
export TMPDIR=/tmp
mkdir -p gpurun_out
for S in ${STREAMS:-ra2160l_q32 ra2160l_q27}; do
  timeout -k 10 240 python -u tools/mc_prof.py run $S > gpurun_out/${TAG}_$S.txt 2>&1 || exit 1
done
