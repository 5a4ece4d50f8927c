"""Error behaviour of the C-ABI's host-only picture builder (include/vvcr.h, vvcr_picture_*), no GPU:
every entry point returns a negative VVCR_E_* code and no exception crosses the boundary, as the
reference's CHECK/THROW (TypeDef.h:1152-1166) would stop DecoderApp on the same inputs.
  VVCR_E_ARG -1: null handle / pointer, descriptors outside the picture; VVCR_E_STATE -3: calls out of
  order; VVCR_E_UNSUPPORTED -4: sequence parameters the path does not handle."""
import ctypes as C
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
E_ARG, E_STATE, E_UNSUPPORTED = -1, -3, -4


def _pic0():
    pics = S.load_sequence(os.path.join(GOLD, "ra416_q32"), max_pics=1)
    p = pics[0]
    alloc = S.SlotAllocator(pics, 16)
    slot = alloc.assign(0, p["hdr"]["poc"])
    return p, S.pic_params(p, slot, dict(alloc.slot_of))


def _seq(h, **kw):
    v = dict(width=h["width"], height=h["height"], chroma=1, bd=h["bitdepth_y"], ctu=h["ctu_log2"], slots=16, dev=0)
    v.update(kw)
    return N.SeqParams(v["width"], v["height"], v["chroma"], v["bd"], v["ctu"], v["slots"], v["dev"])


def _create(sp, pp):
    L = N.lib()
    h = C.c_void_p()
    r = L.vvcr_picture_create(C.byref(sp), C.byref(pp), C.byref(h))
    return r, h


def test_create_rejects_unsupported_sequences():
    p, pp = _pic0()
    h = p["hdr"]
    for kw in ({"chroma": 2}, {"width": h["width"] + 4}, {"ctu": 8}, {"slots": 0}, {"slots": 257}, {"height": 0},
               {"bd": 7}, {"bd": 12}):
        r, hd = _create(_seq(h, **kw), pp)
        assert r == E_UNSUPPORTED, kw
        assert not hd.value
    L = N.lib()
    assert L.vvcr_picture_create(None, C.byref(pp), C.byref(C.c_void_p())) == E_ARG


def test_create_errors_from_several_threads():
    """The error text of a failed create is per thread (vvcr_picture_last_error(NULL)): threads failing
    and succeeding at once each read their own outcome."""
    import threading
    p, pp = _pic0()
    h = p["hdr"]
    L = N.lib()
    bad = []

    def run(k):
        for _ in range(50):
            r, hd = _create(_seq(h, bd=12) if k % 2 else _seq(h), pp)
            if k % 2:
                msg = L.vvcr_picture_last_error(None).decode()
                if r != E_UNSUPPORTED or hd.value or "8..10 bit" not in msg:
                    bad.append((k, r, msg))
            else:
                if r != 0 or not hd.value:
                    bad.append((k, r))
                else:
                    L.vvcr_picture_destroy(hd)
    ts = [threading.Thread(target=run, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not bad, bad[:3]


def test_calls_out_of_order_and_null_handles():
    L = N.lib()
    p, pp = _pic0()
    r, h = _create(_seq(p["hdr"]), pp)
    assert r == 0 and h.value
    try:
        assert L.vvcr_picture_plan(h, N.STAGE_ALL) == E_STATE            # planned before submit
        assert "submitted" in L.vvcr_picture_last_error(h).decode()
        c = (C.c_int64 * 10)()
        assert L.vvcr_picture_work_counts(h, c, 10) == E_STATE            # counts before planning
    finally:
        assert L.vvcr_picture_destroy(h) == 0
    assert L.vvcr_picture_plan(None, N.STAGE_ALL) == E_ARG
    assert L.vvcr_picture_destroy(None) == E_ARG
    assert L.vvcr_picture_set_loop_filter_params(None, None, None) == E_ARG


def test_submit_rejects_out_of_range_references_and_coefficients():
    p, pp = _pic0()
    h = p["hdr"]

    def plan(mut):
        cu, pu, tu, coef = (np.array(p[k], np.int32, copy=True) for k in ("cu", "pu", "tu", "coef"))
        motion = np.array(p["motion"], np.int32, copy=True).reshape(-1, 10)
        mut(cu, pu, tu, coef)
        pic = N.Picture(h["width"], h["height"], pp, bit_depth=h["bitdepth_y"], ctu_log2=h["ctu_log2"], dpb_slots=16)
        try:
            geo = p["geo"] if p["geo"].size else np.zeros((0, 13), np.int32)
            pic.submit(cu, pu, tu, coef, motion, geo)
            S.set_loop_filter_params(pic, p)
            pic.plan()
        finally:
            pic.close()

    plan(lambda cu, pu, tu, coef: None)   # the unmodified picture plans

    # SAO enabled in the picture parameters but no SAO parameters set: a state error at planning
    pic = N.Picture(h["width"], h["height"], pp, bit_depth=h["bitdepth_y"], ctu_log2=h["ctu_log2"], dpb_slots=16)
    try:
        S.submit(pic, p)
        with pytest.raises(N.VvcrError) as e:
            pic.plan()
        assert "(-3)" in str(e.value)
    finally:
        pic.close()

    def coef_past_pool(cu, pu, tu, coef):
        t = tu.reshape(len(tu), -1)
        k = int(np.argmax(t[:, 6 + 6] >= 0))     # a luma TB with coefficients: coef_off past the pool
        t[k, 6 + 6] = coef.size
    with pytest.raises(N.VvcrError) as e:
        plan(coef_past_pool)
    assert "(-1)" in str(e.value)

    def cu_past_width(cu, pu, tu, coef):
        c = cu.reshape(len(cu), -1)
        c[0, 0] = h["width"]                     # CU x at the picture's right edge
    with pytest.raises(N.VvcrError) as e:
        plan(cu_past_width)
    assert "(-1)" in str(e.value)


# ---- the device context (vvcr_*): the same conventions on a GPU

@pytest.mark.gpu
def test_context_calls_out_of_order_and_bad_arguments():
    p, pp = _pic0()
    h = p["hdr"]
    ctx = N.Context(h["width"], h["height"], dpb_slots=4)
    try:
        with pytest.raises(N.VvcrError) as e:
            ctx.end_picture()                                  # no picture begun
        assert "(-3)" in str(e.value)
        with pytest.raises(N.VvcrError) as e:
            ctx.read_plane(N.BUF_RECO, 4, 0)                   # slot past the DPB
        assert "(-1)" in str(e.value)
        with pytest.raises(N.VvcrError) as e:
            ctx.launch(12345)                                  # no such prepared picture
        assert "(-1)" in str(e.value) or "(-3)" in str(e.value)
        bad = S.pic_params(p, 0, {})
        bad.slot = 7                                           # current picture's slot past the DPB
        with pytest.raises(N.VvcrError) as e:
            ctx.begin_picture(bad)
        assert "(-1)" in str(e.value)
        # the context stays usable: the picture reconstructs after the failed calls
        ctx.begin_picture(pp)
        S.submit(ctx, p)
        S.set_loop_filter_params(ctx, p)
        ctx.end_picture()
        ctx.sync()
    finally:
        ctx.close()


def test_inter_jobs_address_every_dpb_slot():
    """DPB slots up to VVCR_MAX_SLOTS (256) survive into the inter work lists: a picture whose references
    sit in slots 128..255 plans jobs that read exactly those slots (a job's slot field once held 7 bits)."""
    L = N.lib()
    L.vvcr_debug_mc_slots.restype = C.c_int
    L.vvcr_debug_mc_slots.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32]
    pics = S.load_sequence(os.path.join(GOLD, "ra416_q32"), max_pics=4)
    for p in pics[1:]:
        h = p["hdr"]
        refs = sorted({int(p["ref_poc"][l][r]) for l in range(2) for r in range(h["num_ref_l%d" % l])})
        slot_of = {poc: 255 - 3 * k for k, poc in enumerate(refs)}
        pic = S.plan_picture(p, 130, slot_of, dpb_slots=256)
        try:
            n = L.vvcr_debug_mc_slots(pic.h, None, 0)
            assert n > 0
            out = (C.c_int32 * n)()
            assert L.vvcr_debug_mc_slots(pic.h, out, n) == n
            assert set(out) <= set(slot_of.values()) and max(out) == 255
        finally:
            pic.close()
