#!/bin/bash
# Per-component residual flags of the fused reconstruction: full GPU suite, MC timings, PMC traffic.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/fused_$S.json || exit 1
done
bash tools/pmc.sh r04w
