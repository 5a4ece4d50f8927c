#!/bin/bash
# Host-side A/B of two host_prof builds on the GPU box's CPU (no GPU use): parse of the intra picture
# (min / median of 15), then the per-phase totals of a whole decode (parse / derive / plan, 3 repeats).
S=tests/golden/streams/ra2160l_q27.bin
for i in 1 2 3; do
  for b in base new; do
    echo "$b $(HOST_PROF_PARSE0=1 timeout 120 ./hostab/host_prof_$b $S 15)"
  done
done
for i in 1 2; do
  for b in base new; do
    echo "$b $(timeout 300 ./hostab/host_prof_$b $S 3 2>/dev/null | tail -1)"
    VVCR_PLAN_PROF=1 timeout 300 ./hostab/host_prof_$b $S 1 2>&1 | grep "plan intra\|intra plan jobs\|vvcp plan" | head -3 | sed "s/^/   $b /"
  done
done
