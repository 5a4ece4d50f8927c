#!/bin/bash
# SIGPROF PC samples of one phase of the host path on the box's CPU (hostab/host_prof_new, -gdwarf-4):
# gpurun_out/hostpcs_<tag>.txt, symbolised here with addr2line on the same binary.
mkdir -p gpurun_out
HOST_PROF_PCS=gpurun_out/hostpcs_$1.txt timeout 600 ./hostab/host_prof_new tests/golden/streams/ra2160l_q27.bin ${2:-20} | tail -1
