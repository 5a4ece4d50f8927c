#!/bin/bash
# Round-end evidence: the GPU suite and the default bench line (gpu_suite.sh), then the picture-synced
# kernel table of the headline and north-star streams with its rocprofv3 pass (gpu_kt.sh).
set -o pipefail
T=${1:-final}
bash tools/gpu_suite.sh $T || exit 1
SYNC=picture bash tools/gpu_kt.sh $T || exit 1
python - $T <<'PY'
import json, sys
t = sys.argv[1]
for s in ("ra2160l_q27", "ra2160l_q32"):
    d = json.load(open("gpurun_out/prof_kt_%s_%s.summary.json" % (t, s)))
    k = d["kernels"]
    print(s, {n: (v["count"], v["avg_us"], v["median_us"], v.get("bench_event_median_us")) for n, v in k.items()
              if n.startswith("k_mc") or n.startswith("k_dbkp") or n in ("k_alf", "k_intra")})
PY
