#!/bin/bash
# SbTMVP sub-block joining (VVCR_SBT_JOIN 0 none / 1 any run / 2 power-of-two runs / 3 whole PU lines):
# MC parity with the default, k_mc in isolation (tools/mc_bench.py) per mode on the 4K QP27 / QP32
# streams, then FETCH_SIZE / WRITE_SIZE per k_mc launch (QP27) for the modes in PMC_JOINS.
set -o pipefail
TAG=${1:-sbtab}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for J in ${JOINS:-0 1 2}; do
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_SBT_JOIN=$J timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/j${J}_$S.json || exit 1
  done
done
O=$O python - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ["O"] + "/j*_ra2160l_q*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), {k: (v["us_per_launch"], v["alg_GBps"]) for k, v in d["kernels"].items() if k.startswith("mc")})
PY
for J in ${PMC_JOINS}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    VVCR_SBT_JOIN=$J timeout -s KILL 90 rocprofv3 --pmc $C -f csv -d $O/pmc_j$J/$C -o run -- python3 tools/mc_bench.py --stream ra2160l_q27 --reps 3 --all-stages > $O/pmc_j${J}_$C.log 2>&1 || exit 1
  done
  python tools/pmc_table.py $O/pmc_j$J k_mc
done
