set -o pipefail
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
VVCR_LANES=7 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --segments 4 > gpurun_out/ln_7_4.json 2>/dev/null &&
VVCR_LANES=8 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --segments 4 > gpurun_out/ln_8_4.json 2>/dev/null &&
VVCR_LANES=7 timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu --segments 4 --stream ra2160_q32 > gpurun_out/ln_7_4_4k.json 2>/dev/null &&
VVCR_LANES=8 timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu --segments 4 --stream ra2160_q32 > gpurun_out/ln_8_4_4k.json 2>/dev/null &&
VVCR_LANES=7 timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu --segments 4 --stream ra2160_q27 > gpurun_out/ln_7_4_4k27.json 2>/dev/null
