#!/bin/bash
# Full GPU test suite, then the default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p/pytest.log 2>&1 || { tail -30 gpurun_out/r05p/pytest.log; exit 1; }
tail -3 gpurun_out/r05p/pytest.log
bash tools/gpu_bench.sh r05p
