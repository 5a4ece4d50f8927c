#!/bin/bash
# Device deblocking planner: parity against the host planner (every picture of 10 streams), the decode /
# bitstream tests on the device-planned path, then the bench's kernel table (deblock_plan / deblock rows).
set -o pipefail
TAG=${1:-dbkp}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dbk_plan_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --kernel-table-only --kernel-table-reps 5 --kernel-table-sync step > $O/kt.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
python - "$O/kt.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["stream"], d["sync"], "bitexact", d["bitexact_vs_reference"])
for n, r in d["kernels"].items():
    print(f"{n:14s} {r['us_per_launch']:10.2f} us x {r['launches_per_step']:3d}  {r['ms_per_step']:8.3f} ms/step")
PY
