#!/bin/bash
# Full GPU suite, the PMC traffic passes of the bench (tools/pmc.sh), the MC kernels with the fused path.
set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r04h/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 --all-stages > gpurun_out/r04h/mcb_fused.json || exit 1
bash tools/pmc.sh r04h
