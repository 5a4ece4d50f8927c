#!/bin/bash
# MC parity + k_mc in isolation with the default SbTMVP jobs, then the default bench line with the
# prepare() phase profile (VVCR_PREP_PROF, printed to the bench's stderr).
set -o pipefail
T=${1:-r05t}
JOINS=${JOINS:-3} PMC_JOINS= bash tools/gpu_sbt_ab.sh ${T}_mc || exit 1
VVCR_PREP_PROF=1 bash tools/gpu_bench.sh $T || exit 1
grep "prepare:" gpurun_out/bench_$T.err || true
