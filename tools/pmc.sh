#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, each under its own kill timer) over a short bench.
# Usage: bash tools/pmc.sh TAG   -> gpurun_out/pmc_TAG/<group>/...csv
TAG=${1:-r01}
export TMPDIR=/tmp
O=gpurun_out/pmc_$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 bench.py --steps 1 --warmup 1 --resident-steps 2 --no-cpu --segments 1 --sync-pictures --shard-steps 0 --single-steps 0 ${PMC_ARGS} > $O/$n.log 2>&1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
