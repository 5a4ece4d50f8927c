#!/bin/bash
# MC / decode parity + MC in isolation (gpu_mc_ab.sh), then the kernel table with its rocprof check
# (gpu_kt.sh, a sync after every picture).
set -o pipefail
T=${1:-r05s}
bash tools/gpu_mc_ab.sh ${T}_mc || exit 1
SYNC=picture bash tools/gpu_kt.sh ${T} || exit 1
python - $T <<'PY'
import json, sys
t = sys.argv[1]
for s in ("ra2160l_q27", "ra2160l_q32"):
    d = json.load(open("gpurun_out/prof_kt_%s_%s.summary.json" % (t, s)))
    k = d["kernels"]
    print(s, {n: (v["count"], v["avg_us"], v["median_us"], v.get("bench_event_median_us")) for n, v in k.items() if n.startswith("k_mc") or n.startswith("k_dbkp") or n == "k_alf"})
PY
