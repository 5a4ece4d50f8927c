#!/bin/bash
# FETCH_SIZE calibration (tools/probe/fetch_cal.hip: 1 GiB read once at 2 / 4 / 8 / 16 B per lane and as
# 8-byte 2-D window gathers), then the PMC traffic passes of the bench on its default stream.
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/cal_$TAG -o run -- ./tools/probe/fetch_cal > gpurun_out/cal_$TAG.log 2>&1 &&
bash tools/pmc.sh $TAG
