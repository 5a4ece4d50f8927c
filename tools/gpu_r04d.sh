#!/bin/bash
# MC checks after a k_mc change: MC / KAT / decode GPU tests, then kernel timings and the per-wave profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_mc_kat.py tests/test_decode_gpu.py tests/test_bitstream.py -m gpu > gpurun_out/r04d_pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q27 --reps 10 > gpurun_out/r04d_mcb27.json &&
timeout -k 10 120 python -u tools/mc_bench.py --stream ra2160l_q32 --reps 10 > gpurun_out/r04d_mcb32.json &&
timeout -k 10 150 python -u tools/mc_prof.py run ra2160l_q27 > gpurun_out/r04d_mcprof.txt 2>&1
