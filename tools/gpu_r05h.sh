#!/bin/bash
# Device deblocking planner: parity + kernel table (gpu_dbkp.sh), the stage-by-stage lane test, per-kernel profile.
set -o pipefail
T=${1:-r05h}
bash tools/gpu_dbkp.sh ${T}_dbkp || exit 1
timeout -k 10 120 python -u -m pytest tests/test_decode_gpu.py -k "stage_by_stage" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_dbkp/staged.log 2>&1 || { tail -20 gpurun_out/${T}_dbkp/staged.log; exit 1; }
tail -1 gpurun_out/${T}_dbkp/staged.log
bash tools/gpu_dbkp_prof.sh ${T}_prof
