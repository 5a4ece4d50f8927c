set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py tests/test_decode_gpu.py -x -v --timeout 200 --timeout-method thread -k "shard or ratile" > gpurun_out/pytest_sh1.log 2>&1
