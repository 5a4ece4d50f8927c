#!/bin/bash
# The default bench under a few environments (A/B of host-side settings): ENVS="name:VAR=v,VAR2=v name2:..."
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in $ENVS; do
  name=${spec%%:*}; vars=${spec#*:}
  env $(echo $vars | tr ',' ' ') timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/benchab_$name.json 2> gpurun_out/benchab_$name.err || { tail -20 gpurun_out/benchab_$name.err; exit 1; }
  python - gpurun_out/benchab_$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["host_ms_per_picture"], d.get("single_stream", {}).get("value"))
PY
done
