#!/bin/bash
# Host-only A/B of the whole decode's phases (parse / derive / plan totals per repeat), alternated.
S=tests/golden/streams/ra2160l_q27.bin
for i in 1 2 3 4; do
  for b in base new; do echo "$b $(timeout 300 ./hostab/host_prof_$b $S 3 2>/dev/null | tail -1)"; done
done
