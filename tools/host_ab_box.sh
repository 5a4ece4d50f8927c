#!/bin/bash
# Host-side A/B on the GPU box's CPU (no GPU use): two host_prof builds (tools/host_prof_main.cpp linked
# against two library builds) alternated, picture 0's CABAC pass (HOST_PROF_PARSE0), picture 0's plan
# (HOST_PROF_PLAN0, one planner thread) and the whole 17-picture decode's parse / derive / plan (min of runs).
#   bash tools/host_ab_box.sh DIR  (DIR holds host_prof_old and host_prof)
D=${1:-tmp_hostab}
S=tests/golden/streams/ra2160l_q27.bin
for k in 1 2 3; do
  for b in host_prof_old host_prof; do
    echo "$b $(HOST_PROF_PARSE0=1 timeout 120 $D/$b $S 5)"
    echo "$b $(VVCR_PLAN_THREADS=1 HOST_PROF_PLAN0=1 timeout 120 $D/$b $S 5)"
    echo "$b $(VVCR_PLAN_THREADS=1 timeout 120 $D/$b $S 2)"
  done
done
