#!/bin/bash
# Full GPU suite, then k_mc ablations (no reference loads / no filter arithmetic / neither), the fused MC
# kernels' timings, SQ + instruction-cache counters of the MC kernels alone (tools/pmc_mcb.sh), 4K QP27.
set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r04g/pytest.log 2>&1 || exit 1
S=ra2160l_q27
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04g/base.json || exit 1
timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 --all-stages > gpurun_out/r04g/basefused.json || exit 1
for v in abl_loads abl_filter abl_both wg256; do
  VVCR_LIB=vvc_amd/libvvcr_$v.so timeout -k 10 120 python -u tools/mc_bench.py --stream $S --reps 10 > gpurun_out/r04g/$v.json || exit 1
done
bash tools/pmc_mcb.sh $S g
