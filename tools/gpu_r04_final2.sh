#!/bin/bash
# Round-4 evidence after the MC block-order / per-component residual / ALF changes: the isolated MC
# stage timings (plain and fused), then tools/gpu_r04_final.sh (GPU suite, bench line, rocprof, PMC).
set -o pipefail
TAG=${1:-r04f2}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/$TAG/base_$S.json || exit 1
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/$TAG/fused_$S.json || exit 1
done
bash tools/gpu_r04_final.sh $TAG
