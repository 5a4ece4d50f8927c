#!/bin/bash
# ALF phase stamps, then the k_mc knob comparison (tools/gpu_r04p.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/alf_prof.py run ra2160l_q27 > gpurun_out/r04q_alfprof.txt 2>&1 &&
bash tools/gpu_r04p.sh
