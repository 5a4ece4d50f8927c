"""The device deblocking planner (vvcr_dbk_plan.hip: edges, boundary strengths, filter lengths and QPs of
every 4-sample edge segment, one thread per CU and direction) against the host planner
(vvcr_dbk_host.cpp, VVCR_DBK_GPU=0), which restates LoopFilter::xDeblockCU (LoopFilter.cpp:261-408) and is
pinned by the decode tests to DecoderApp's deblocked planes: the four segment lists must hold the same
segments with the same words, picture by picture (the device lists' order differs; it does not change the
filtered samples). Streams: dual-tree intra pictures (ai*), ISP / MIP / BDPCM (aibdpcm), affine, SbTMVP,
GEO / CIIP (rageo), LMCS, weighted prediction, tiles, DQ0, tiles and slices not deblocked across (ratilenf)."""
import ctypes as C
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _lists(L, pic):
    sizes = (C.c_int32 * 4)()
    assert L.vvcr_debug_dbk_list_sizes(pic.h, sizes) == 4
    n = L.vvcr_debug_dbk_segments(pic.h, None, 0)
    a = np.zeros((n, 2), np.uint32)
    if n:
        L.vvcr_debug_dbk_segments(pic.h, a.ctypes.data, n)
    out, o = [], 0
    for k in range(4):
        seg = a[o:o + sizes[k]]
        o += sizes[k]
        key = (seg[:, 0] >> 16) * 65536 + (seg[:, 0] & 0xffff)   # (y4, x4) of the packed x4 | y4 << 16
        out.append(seg[np.argsort(key, kind="stable")])
    return out, list(sizes)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ai416_q37", "aibdpcm416_q32", "ailm416_q37", "ra416_q32", "rageo480_q32", "ralmgeo416_q32",
                                  "rawp416_q32", "ratile416_q32", "radq0416_q32", "ra1080_q32", "ratilenf416_q32",
                                  "rasub480_q32", "ravb416_q32", "ravb416b_q37", "raladf416_q32", "rarsc416_q32"])
def test_device_deblocking_plan_equals_host_plan(name, monkeypatch):
    L = N.lib()
    L.vvcr_debug_dbk_segments.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    L.vvcr_debug_dbk_list_sizes.argtypes = [C.c_void_p, C.c_void_p]
    L.vvcr_debug_dbk_gpu_segments.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
    pics = S.load_sequence(os.path.join(GOLD, name))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], ctu_log2=h0["ctu_log2"], dpb_slots=16)
    alloc = S.SlotAllocator(pics, 16)
    try:
        for i, p in enumerate(pics):
            slot = alloc.assign(i, p["hdr"]["poc"])
            monkeypatch.setenv("VVCR_DBK_GPU", "0")
            host = S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16)
            ref, sizes = _lists(L, host)
            host.close()
            monkeypatch.delenv("VVCR_DBK_GPU")
            dev = S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16)
            n = L.vvcr_debug_dbk_gpu_segments(ctx.h, dev.h, None, 0)
            assert n >= 0, L.vvcr_last_error(ctx.h)
            got = np.zeros((max(n, 1), 2), np.uint32)
            assert L.vvcr_debug_dbk_gpu_segments(ctx.h, dev.h, got.ctypes.data, n) == n
            dev.close()
            assert n == sum(sizes), "POC %d: %d device segments, %d host (%s)" % (p["hdr"]["poc"], n, sum(sizes), sizes)
            o = 0
            for k in range(4):
                g = got[o:o + sizes[k]]
                o += sizes[k]
                bad = np.nonzero((g != ref[k]).any(axis=1))[0]
                assert len(bad) == 0, "POC %d list %d: %d of %d segments differ, first host %s device %s" % (
                    p["hdr"]["poc"], k, len(bad), sizes[k], ref[k][bad[0]], g[bad[0]])
    finally:
        ctx.close()
