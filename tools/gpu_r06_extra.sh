#!/bin/bash
# Round-6 extras on the GPU box: the virtual-boundary streams' parity tests, the EncoderApp drop-in with its
# speed record, and the config-5 RDO bench line with its rocprofv3 kernel statistics.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06x}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_bitstream.py tests/test_dbk_plan_gpu.py -m gpu -x -v -k "ravb or rasub" --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_vb.log 2>&1 || { tail -30 gpurun_out/$T/pytest_vb.log; exit 1; }
tail -3 gpurun_out/$T/pytest_vb.log
VVCR_RECORD_DIR=gpurun_out/$T timeout -k 10 400 python -u -m pytest tests/test_enc_dropin_gpu.py -m gpu -x -v -s --timeout 380 --timeout-method thread > gpurun_out/$T/pytest_enc.log 2>&1 || { tail -30 gpurun_out/$T/pytest_enc.log; exit 1; }
tail -3 gpurun_out/$T/pytest_enc.log
timeout -k 10 300 python -u bench_rdo.py > gpurun_out/$T/bench_rdo.json 2> gpurun_out/$T/bench_rdo.err || { tail -20 gpurun_out/$T/bench_rdo.err; exit 1; }
cat gpurun_out/$T/bench_rdo.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$T/rdo_prof -o run -- python3 bench_rdo.py --no-cpu > gpurun_out/$T/rdo_prof.log 2>&1 || { tail -20 gpurun_out/$T/rdo_prof.log; exit 1; }
find gpurun_out/$T/rdo_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {}'
