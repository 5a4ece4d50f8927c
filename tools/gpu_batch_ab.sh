#!/bin/bash
# Frame-batched plain MC A/B (round 6): the GPU tests of the batched path, then the bench's kernel table
# (median of 7 synced one-segment steps, 4K QP27 + the north-star QP32 stream) with the decode loop's
# groups of up to 4 (default), 2 and 1 picture (VVCP_MC_BATCH=k), alternated twice.
set -o pipefail
T=${1:-r06a}
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_batch.py tests/test_decode_gpu.py tests/test_bitstream.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
  tail -2 gpurun_out/$T/pytest.log
fi
for k in 1 2; do
  for B in ${BATCHES:-4 2 1}; do
    VVCP_MC_BATCH=$B timeout -k 10 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 > gpurun_out/$T/kt_b${B}_$k.json 2> gpurun_out/$T/kt_b${B}_$k.err || exit 1
    python - gpurun_out/$T/kt_b${B}_$k.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for tag, m in (("q27", d["mc_roofline"]), ("q32", d["north_star_mc"])):
    x = m["mc"]
    print(sys.argv[1], tag, "k_mc us/launch %.2f us/picture %.2f launches %d pictures %d  %.0f GB/s frac %.3f  stage %.0f GB/s  exact %s" % (
        x["us_per_launch"], x["us_per_picture"], x["launches_per_step"], x["pictures_per_step"], x["achieved"], x["frac"],
        m["mc_stage"]["achieved"], d["bitexact_vs_reference"] if tag == "q27" else m["bitexact_vs_reference"]))
PY
  done
done
