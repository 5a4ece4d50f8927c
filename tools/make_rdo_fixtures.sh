#!/bin/bash
# RDO known-answer vectors from the reference's own functions (oracle/capture/rdo_kat.cpp, built by
# oracle/ref.mk from /root/reference): tests/golden/rdo/{dist,tr}.bin. Test infrastructure only.
set -e
cd "$(dirname "$0")/.."
make -f oracle/ref.mk -j8 rdo_kat
mkdir -p tests/golden/rdo
oracle/_ref/rdo_kat 1234 tests/golden/rdo/dist.bin tests/golden/rdo/tr.bin
