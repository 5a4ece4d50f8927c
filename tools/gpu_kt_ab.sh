#!/bin/bash
# Kernel-table A/B of library variants (tools/mc_variants.py): the bench's kernel table (median of 7 synced
# one-segment steps of the 4K QP27 stream and the north-star QP32 stream, frame-batched launch groups) with
# the default library and each VARIANTS library, alternated ROUNDS times; then each result's k_mc summary.
set -o pipefail
T=${1:-ktab}
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
  tail -2 gpurun_out/$T/pytest.log
fi
for k in $(seq ${ROUNDS:-2}); do
  for V in new $VARIANTS; do
    L=$PWD/vvc_amd/libvvcr_$V.so; [ $V = new ] && L=$PWD/vvc_amd/libvvcr.so
    VVCR_LIB=$L timeout -k 10 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 > gpurun_out/$T/kt_${V}_$k.json 2> gpurun_out/$T/kt_${V}_$k.err || exit 1
    python - gpurun_out/$T/kt_${V}_$k.json <<'PY'
import json, os, sys
d = json.load(open(sys.argv[1]))
for tag, m in (("q27", d["mc_roofline"]), ("q32", d["north_star_mc"])):
    x = m["mc"]
    print("%-22s %s k_mc us/pic %6.2f (%5.2f/launch, %2d launches) %5.0f GB/s %.3f | bidir %6.2f affine %6.2f us | stage %5.0f GB/s exact %s" % (
        os.path.basename(sys.argv[1]), tag, x["us_per_picture"], x["us_per_launch"], x["launches_per_step"], x["achieved"], x["frac"],
        m["mc_bidir"]["us_per_launch"], m["mc_affine"]["us_per_launch"], m["mc_stage"]["achieved"],
        d["bitexact_vs_reference"] if tag == "q27" else m["bitexact_vs_reference"]))
PY
  done
done
