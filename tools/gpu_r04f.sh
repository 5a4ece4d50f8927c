#!/bin/bash
# decode tests (fused MC epilogue), the k_mc variant sweep (tools/gpu_r04e.sh), then the k_intra step
# profile of the 4K I picture and its isolated time.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py tests/test_mc_gpu.py tests/test_lf_gpu.py -m gpu > gpurun_out/r04f_pytest.log 2>&1 &&
bash tools/gpu_r04e.sh &&
INTRA_PROF_PICS=1 timeout -k 10 150 python -u tools/intra_prof.py run ra2160l_q27 > gpurun_out/r04f_iprof.log 2>&1 &&
timeout -k 10 120 python -u tools/intra_bench.py --stream ra2160l_q27 --reps 10 > gpurun_out/r04f_intra_bench.json 2>&1
