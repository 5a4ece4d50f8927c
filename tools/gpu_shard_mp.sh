#!/bin/bash
# Rehearsal of the multi-process path on a one-GPU box: 2 ranks on GPU 0 with the gloo backend (RCCL
# cannot run two ranks on one device): replica line + the sharded 8K pass through TorchComm.
set -o pipefail
mkdir -p gpurun_out
export VVCR_DIST_BACKEND=gloo VVCR_DEVICE=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e-threads 0 > gpurun_out/bench_mp2.json 2> gpurun_out/bench_mp2.err
