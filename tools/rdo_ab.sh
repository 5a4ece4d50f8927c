set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rdo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mfma.log 2>&1 &&
timeout -k 10 300 python -u bench_rdo.py --no-cpu > gpurun_out/bench_rdo_mfma.json 2>/dev/null &&
VVCR_FWD_MFMA=0 timeout -k 10 300 python -u bench_rdo.py --no-cpu > gpurun_out/bench_rdo_valu.json 2>/dev/null
