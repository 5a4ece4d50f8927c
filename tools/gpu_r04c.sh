#!/bin/bash
# r04: GPU suite (drop-in, multi-process shard), HBM traffic per kernel (FETCH / WRITE), MC counters.
set -o pipefail
TAG=${1:-c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_shard_mp_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
bash tools/pmc.sh $TAG && python3 tools/pmc_summary.py gpurun_out/pmc_$TAG ra2160l_q27 > gpurun_out/traffic_$TAG.json
bash tools/pmc_mc4.sh $TAG ra2160l_q27
