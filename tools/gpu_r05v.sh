#!/bin/bash
set -o pipefail
VVCR_PREP_PROF=1 bash tools/gpu_r05p.sh r05v || exit 1
grep "prepare:" gpurun_out/bench_r05v.err || true
INTRA_PROF_PICS=1 timeout -k 10 300 python tools/intra_prof.py run ra2160l_q27 > gpurun_out/iprof_fill.log 2>&1 || { tail -20 gpurun_out/iprof_fill.log; exit 1; }
