#!/bin/bash
# Kernel ablations (first written for the device deblocking planner): per-kernel averages (rocprofv3 kernel trace, picture-synced kernel
# table of the headline stream) of the product library and of diagnostics builds in tmp_abl/lib_*.so
# (VVCR_LIB; results of those are wrong by construction).
set -o pipefail
TAG=${1:-dbkp_abl}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for L in vvc_amd/libvvcr.so ${ABL_DIR:-tmp_abl}/lib_*.so; do
  N=$(basename $L .so)
  P=gpurun_out/$TAG/$N
  VVCR_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $P -o run -- python3 -u bench.py --kernel-table-only --kernel-table-reps 3 --kernel-table-sync picture --stream ${STREAM:-ra2160l_q27} --north-star-stream "" > $P.json 2> $P.err || { tail -5 $P.err; exit 1; }
  echo "== $N"
  python - $P ${FILTER:-dbk,fill} <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in sys.argv[2].split(",")):
        print(f"  {n[:50]:50s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:9.2f} us")
PY
done
