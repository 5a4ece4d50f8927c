set -o pipefail
mkdir -p gpurun_out
for v in s01 s24 nw5; do
VVCR_LIB=$PWD/alt/libvvcr_$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_base.json 2>/dev/null
