#!/bin/bash
# Per-kernel times of the device deblocking planner (k_dbkp_maps / k_dbkp_pos and its memsets) under
# rocprofv3 --kernel-trace --stats, one kernel-table step of the headline stream.
set -o pipefail
TAG=${1:-dbkp_prof}
export TMPDIR=/tmp
P=gpurun_out/$TAG
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $P -o run -- python3 -u bench.py --kernel-table-only --kernel-table-reps 2 --kernel-table-sync step --north-star-stream "" > $P/kt.json 2> $P/kt.err || { tail -20 $P/kt.err; exit 1; }
python - $P <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("dbk", "Memset", "fill", "k_mc", "k_alf", "k_sao", "intra")):
        print(f"{n[:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:9.2f} us")
PY
