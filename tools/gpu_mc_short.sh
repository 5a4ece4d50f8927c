set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05sl; mkdir -p $O
VVCR_LIB=vvc_amd/libvvcr_sl.so timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py tests/test_decode_gpu.py tests/test_bitstream.py tests/test_mc_kat.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_sl.log 2>&1 || { tail -20 $O/pytest_sl.log; exit 1; }
tail -1 $O/pytest_sl.log
for V in base sl base sl; do
  L=vvc_amd/libvvcr.so; [ $V = sl ] && L=vvc_amd/libvvcr_sl.so
  for S in ra2160l_q27 ra2160l_q32; do
    VVCR_LIB=$L timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/${V}_$S.json || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/${V}_$S.json')); print('$V $S', {k: (v['us_per_launch'], v['alg_GBps']) for k, v in d['kernels'].items() if k.startswith('mc')})"
  done
done
