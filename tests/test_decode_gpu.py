"""End-to-end parity: every picture of each stream reconstructed by libvvcr from its descriptors alone
(references are libvvcr's own output in its device DPB) matches the reference decoder's output
picture MD5s (= the stream's decoded-picture-hash SEI) and the MD5 of DecoderApp's YUV file."""
import os

import pytest

from vvc_amd import decode as D
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32", "ra1080_q32", "ailm416_q37", "ralm416_q32", "rawp416_q32", "ra2160_q27", "ra2160_q32"])
def test_decode_matches_reference_md5(golden_dir, name):
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    md5, yuv = D.decode_and_hash(pics)
    for poc, exp in meta["poc_plane_md5"].items():
        assert md5[int(poc)] == exp, "POC %s: plane MD5 %s != reference %s" % (poc, md5[int(poc)], exp)
    assert yuv == meta["yuv_md5"]


@pytest.mark.parametrize("lanes", ["4", "7"])
@pytest.mark.parametrize("name", ["ra416_q32", "ra1080_q32"])
def test_concurrent_segments_match_reference_md5(golden_dir, name, lanes, monkeypatch):
    """Two copies of the stream on disjoint DPB slots, every picture launched back to back with no host
    synchronisation in between: the execution lanes run pictures concurrently, ordered only by their
    slot dependencies (vvcr_api.cpp launch), and every picture of both copies must still be bit-exact."""
    from vvc_amd import native as N
    monkeypatch.setenv("VVCR_LANES", lanes)   # read by vvcr_create
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    n = len(pics)
    per = min(n, 16)                                   # 2 copies within the 32 DPB slots
    dec = D.Decoder(pics, dpb_slots=2 * per)
    ctx = dec.ctx
    try:
        copies = []
        for c in range(2):
            alloc = S.SlotAllocator(pics, per, base=per * c)
            hs = []
            for i, p in enumerate(pics):
                slot = alloc.assign(i, p["hdr"]["poc"])
                ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
                S.submit(ctx, p)
                S.set_loop_filter_params(ctx, p)
                hs.append((ctx.prepare(N.STAGE_ALL), p["hdr"]["poc"], slot))
            copies.append(hs)
        for rnd in range(2):
            for i in range(n):                      # interleaved: copy 0 picture i, copy 1 picture i
                for hs in copies:
                    ctx.launch(hs[i][0])
            ctx.sync()
            for hs in copies:
                owner = {slot: poc for _, poc, slot in hs}   # the last picture written to each slot
                for slot, poc in owner.items():
                    exp = meta["poc_plane_md5"][str(poc)]
                    assert D.plane_md5s(dec.read(slot)) == exp, "round %d POC %d differs" % (rnd, poc)
        for hs in copies:
            for h, _, _ in hs:
                ctx.release(h)
    finally:
        dec.close()
