"""Host logic of the replay driver (no GPU): DPB slot allocation per segment copy (vvc_amd/stream.py
SlotAllocator) — disjoint slot ranges, no slot reused while a later picture still references it, and the
minimum slot counts bench.py relies on (4 segment copies in 32 slots)."""
import os

import pytest

from vvc_amd import stream as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _refs(p):
    h = p["hdr"]
    return {int(p["ref_poc"][l][r]) for l in range(2) for r in range(h["num_ref_l%d" % l])}


@pytest.mark.parametrize("name", ["ra416_q32", "ra1080_q32", "ra2160_q32"])
def test_slot_allocator_keeps_references_resident(name):
    pics = S.load_sequence(os.path.join(GOLD, name))
    per = 32 // 4
    for c in range(4):
        a = S.SlotAllocator(pics, per, base=per * c)
        for i, p in enumerate(pics):
            poc = p["hdr"]["poc"]
            refs = _refs(p)
            slot = a.assign(i, poc)
            assert per * c <= slot < per * (c + 1)
            # every reference of this picture is still resident, in its own slot, and not this picture's slot
            for r in refs:
                assert r in a.slot_of and a.slot_of[r] != slot, (name, poc, r)


def test_slot_allocator_reports_exhaustion():
    pics = S.load_sequence(os.path.join(GOLD, "ra1080_q32"))
    with pytest.raises(RuntimeError):
        a = S.SlotAllocator(pics, 2)
        for i, p in enumerate(pics):
            a.assign(i, p["hdr"]["poc"])
