#!/bin/bash
# ALF: 32-row regions (ALF_ROWS=32 build) A/B against the 16-row default, bit-exactness of the variant,
# and the SQ instruction-mix / stall counters of the default k_alf (tools/mc_bench.py --all-stages).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
VVCR_LIB=vvc_amd/libvvcr_alf32.so timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_recon_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_alf32.log 2>&1 || exit 1
for S in ra2160l_q27 ra2160l_q32; do
  timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/base_$S.json || exit 1
  VVCR_LIB=vvc_amd/libvvcr_alf32.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > $O/alf32_$S.json || exit 1
done
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $O/sq/$n -o run -- python3 -u tools/mc_bench.py --stream ra2160l_q27 --reps 1 --all-stages > $O/sq_$n.log 2>&1
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run b SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
