#!/bin/bash
# r05 GPU session: device deblocking planner parity, MC / decode parity, MC A/B (affine one-wave form vs
# r04, bidir ablations), kernel tables (picture / step sync) and their rocprof traces, k_mc wave profile.
# A failing test does not stop the later measurements; a fault, abort or time limit does.
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
run() {   # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stop after $n"; exit $rc; fi
  return 0
}
run pytest_dbkplan 400 python -u -m pytest tests/test_dbk_plan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
run pytest_mc 500 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py tests/test_mc_kat.py tests/test_enc_dropin_gpu.py -m gpu -q --timeout 200 --timeout-method thread
for V in new affv1 abl1 abl2 abl4 abl7; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L run mcb_${V}_$S 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages
  done
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r05c/mcb_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(os.path.basename(f), {k: (v["us_per_launch"], v["alg_GBps"]) for k, v in d["kernels"].items() if k.startswith("mc")})
    except Exception as e:
        print(f, "unreadable", e)
PY
run kt_pic 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 --kernel-table-sync picture
VVCR_LANES=2 VVCR_INTRA_LANES=1 run kt_step2 300 python -u bench.py --kernel-table-only --kernel-table-reps 7 --kernel-table-sync step
SYNC=step run kt_rocprof 700 bash tools/gpu_kt.sh r05c
run mcprof 300 bash tools/gpu_mcprof.sh r05c_mcprof
