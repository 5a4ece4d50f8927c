#!/bin/bash
# MC known-answer vectors from the reference's own interpolation filters (oracle/capture/mc_kat.cpp, built
# by oracle/ref.mk from /root/reference). Test infrastructure; runs in the build container.
set -e
cd "$(dirname "$0")/.."
make -f oracle/ref.mk -j8 mc_kat
mkdir -p tests/golden/mc_kat
for s in 1 2 3 4 5 6; do oracle/_ref/mc_kat $s tests/golden/mc_kat/kat_$s.bin; done
