#!/bin/bash
# Two ranks on the one-GPU box over gloo (the driver runs N > 1 over RCCL on an 8-GPU node): the default
# bench path at --gpus 2, then the same with a 1-second shard watchdog (the line must still print).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g2
export VVCR_DIST_BACKEND=gloo VVCR_DEVICE=0
timeout -k 10 900 python -u bench.py --gpus 2 --steps 3 --warmup 1 --single-steps 0 --north-star-steps 0 > gpurun_out/r06g2/bench_gpus2.json 2> gpurun_out/r06g2/bench_gpus2.err || { tail -20 gpurun_out/r06g2/bench_gpus2.err; exit 1; }
tail -c 600 gpurun_out/r06g2/bench_gpus2.json
timeout -k 10 600 python -u bench.py --gpus 2 --steps 2 --warmup 1 --single-steps 0 --north-star-steps 0 --resident-steps 0 --shard-timeout 1 > gpurun_out/r06g2/bench_gpus2_dog.json 2> gpurun_out/r06g2/bench_gpus2_dog.err || { tail -20 gpurun_out/r06g2/bench_gpus2_dog.err; exit 1; }
tail -c 300 gpurun_out/r06g2/bench_gpus2_dog.json
