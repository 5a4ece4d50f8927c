#!/bin/bash
# MC kernels: GPU parity (MC / decode / bitstream tests), then an A/B in isolation (tools/mc_bench.py, fused
# path) of the default library against VARIANTS (vvc_amd/libvvcr_<v>.so) on the 4K QP27 / QP32 streams.
set -o pipefail
TAG=${1:-mcab}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py tests/test_mc_kat.py tests/test_enc_dropin_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for V in new ${VARIANTS}; do
  L=vvc_amd/libvvcr_$V.so; [ $V = new ] && L=vvc_amd/libvvcr.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/${V}_$S.json || exit 1
  done
done
O=$O python - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ.get("O", "gpurun_out/x") + "/*_ra2160l_q*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), {k: (v["us_per_launch"], v["alg_GBps"]) for k, v in d["kernels"].items() if k.startswith("mc")})
PY
