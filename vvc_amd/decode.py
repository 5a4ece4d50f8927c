"""Whole-sequence reconstruction through libvvcr: the host side of the drop-in path.

Replays one parsed picture after the other in decoding order (what DecApp::decode / DecLib do per
picture: DecApp.cpp:118-200, DecLib::executeLoopFilters DecLib.cpp:560), keeping every reference
picture in the library's device DPB. The only host work per picture is handing over the descriptors
(vvcr_submit) and the loop-filter parameters; all sample processing runs on the GPU.
"""
import hashlib

import numpy as np

from . import native as N
from . import stream as S


class Decoder:
    def __init__(self, pics, dpb_slots=12, device=0, ctx=None):
        h0 = pics[0]["hdr"]
        self.pics = pics
        self.W, self.H = h0["width"], h0["height"]
        self.ctx = ctx or N.Context(self.W, self.H, bit_depth=h0["bitdepth_y"], ctu_log2=h0["ctu_log2"],
                                    dpb_slots=dpb_slots, device=device)
        self.alloc = S.SlotAllocator(pics, dpb_slots)

    def decode_picture(self, i, stages=N.STAGE_ALL):
        p = self.pics[i]
        poc = p["hdr"]["poc"]
        slot = self.alloc.assign(i, poc)
        self.ctx.begin_picture(S.pic_params(p, slot, self.alloc.slot_of))
        S.submit(self.ctx, p)
        S.set_loop_filter_params(self.ctx, p)
        self.ctx.end_picture(stages)
        return poc, slot

    def read(self, slot):
        return [self.ctx.read_plane(N.BUF_RECO, slot, c) for c in range(3)]

    def close(self):
        self.ctx.close()


def plane_md5s(planes):
    return [hashlib.md5(np.ascontiguousarray(pl).astype("<u2").tobytes()).hexdigest() for pl in planes]


def decode_and_hash(pics, **kw):
    """Decode all pictures; returns {poc: [md5 y, u, v]} and the MD5 of the output YUV in POC order
    (DecoderApp -o writes 16-bit little-endian samples for a 10-bit stream)."""
    dec = Decoder(pics, **kw)
    md5, out = {}, {}
    try:
        for i in range(len(pics)):
            poc, slot = dec.decode_picture(i)
            planes = dec.read(slot)
            md5[poc] = plane_md5s(planes)
            out[poc] = planes
    finally:
        dec.close()
    h = hashlib.md5()
    for poc in sorted(out):
        for pl in out[poc]:
            h.update(np.ascontiguousarray(pl).astype("<u2").tobytes())
    return md5, h.hexdigest()
