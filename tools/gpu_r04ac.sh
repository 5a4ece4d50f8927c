#!/bin/bash
# bench line with the per-picture-synced kernel-table step, then the k_alf block-order A/B
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04ac.json 2> gpurun_out/bench_r04ac.err &&
bash tools/gpu_r04ab.sh
