#!/bin/bash
# Full GPU test suite, then the default bench line (tag: gpurun_out/bench_<tag>.json, gpurun_out/<tag>/pytest.log).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r05p}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
bash tools/gpu_bench.sh $T
