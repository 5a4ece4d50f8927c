#!/bin/bash
# A round's kernel evidence in one GPU call: the bench's kernel table of the headline and north-star
# streams with the rocprofv3 kernel traces of the same steps (tools/gpu_kt.sh TAG), then the PMC passes of
# the headline stream alone (tools/pmc.sh TAG: FETCH_SIZE, WRITE_SIZE, SQ issue counters), summarised per
# kernel group (tools/pmc_summary.py, read into bench.py's roofline.traffic from profiles/TAG_traffic_2160l.json).
#   bash tools/gpu_evidence.sh r06
set -o pipefail
TAG=${1:-rNN}
export TMPDIR=/tmp
SYNC=picture bash tools/gpu_kt.sh $TAG || exit 1
PMC_ARGS='--north-star-steps 0 --north-star-stream=' bash tools/pmc.sh $TAG || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG ra2160l_q27 > gpurun_out/${TAG}_traffic_2160l.json || exit 1
