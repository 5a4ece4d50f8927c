"""Encoder RDO inner loop on the GPU through the C-ABI (vvcr_rd_dist / vvcr_fwd_transform): SAD and
Hadamard SATD per block and forward transforms, bit-exact against the reference's own outputs
(tests/golden/rdo, from RdCost::setDistParam + distFunc and fastFwdTrans via oracle/capture/rdo_kat.cpp)
and against the C oracle on a larger random batch."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
import rdo_golden
from vvc_amd import native as N

pytestmark = pytest.mark.gpu


def _ctx():
    return N.Context(64, 64, dpb_slots=1)


def _pools(items):
    """pack 2-D blocks into one int16 pool; returns (pool, offsets)"""
    offs, tot = [], 0
    for a in items:
        offs.append(tot)
        tot += a.size
    pool = np.zeros(tot, np.int16)
    for a, o in zip(items, offs):
        pool[o:o + a.size] = a.ravel()
    return pool, offs


def test_rd_dist_matches_reference():
    blocks = rdo_golden.dist_blocks()
    org, oo = _pools([b[2] for b in blocks])
    cur, co = _pools([b[3] for b in blocks])
    bl = np.zeros(len(blocks), N.RD_BLOCK)
    for i, (w, h, *_r) in enumerate(blocks):
        bl[i] = (oo[i], co[i], w, w, w, h)
    ctx = _ctx()
    try:
        sad, satd = ctx.rd_dist(bl, org, cur)
    finally:
        ctx.close()
    assert np.array_equal(sad, [b[4] for b in blocks])
    assert np.array_equal(satd, [b[5] for b in blocks])


def test_rd_dist_random_batch_matches_oracle():
    """a 1080p-like batch: blocks at picture positions with the picture stride, every even shape"""
    rng = np.random.default_rng(7)
    W, H = 640, 384
    org = rng.integers(0, 1024, (H, W)).astype(np.int16)
    cur = np.clip(org + rng.integers(-40, 41, (H, W)), 0, 1023).astype(np.int16)
    shapes = [(w, h) for w in (2, 4, 8, 16, 32, 64, 128) for h in (2, 4, 8, 16, 32, 64, 128)] + [(6, 10), (12, 4), (24, 16)]
    bl = np.zeros(600, N.RD_BLOCK)
    for i in range(len(bl)):
        w, h = shapes[i % len(shapes)]
        x, y = int(rng.integers(0, W - w + 1)), int(rng.integers(0, H - h + 1))
        bl[i] = (y * W + x, y * W + x, W, W, w, h)
    ctx = _ctx()
    try:
        sad, satd = ctx.rd_dist(bl, org, cur)
    finally:
        ctx.close()
    L = oracle_lib.lib()
    L.or_sad.restype = C.c_uint32
    L.or_satd.restype = C.c_uint32
    for i, b in enumerate(bl):
        o = org.ravel()[b["org_off"]:]
        c = cur.ravel()[b["cur_off"]:]
        po, pc = C.c_void_p(o.ctypes.data), C.c_void_p(c.ctypes.data)
        assert sad[i] == L.or_sad(po, W, pc, W, int(b["width"]), int(b["height"])), i
        assert satd[i] == L.or_satd(po, W, pc, W, int(b["width"]), int(b["height"])), i


def test_rd_dist_staging_reuse():
    """consecutive calls on one context: the staging span is reused, grown for a larger pool and reused
    again; every call's results equal the C oracle's"""
    rng = np.random.default_rng(11)
    L = oracle_lib.lib()
    L.or_sad.restype = C.c_uint32
    L.or_satd.restype = C.c_uint32
    ctx = _ctx()
    try:
        for W, H, n in ((16, 16, 1), (1280, 720, 200), (32, 8, 3), (1920, 1088, 50), (8, 8, 1)):
            org = rng.integers(0, 1024, (H, W)).astype(np.int16)
            cur = np.clip(org + rng.integers(-60, 61, (H, W)), 0, 1023).astype(np.int16)
            bl = np.zeros(n, N.RD_BLOCK)
            for i in range(n):
                w, h = [(8, 8), (16, 4), (4, 16), (2, 2), (32, 8)][i % 5]
                w, h = min(w, W), min(h, H)
                x, y = int(rng.integers(0, W - w + 1)), int(rng.integers(0, H - h + 1))
                bl[i] = (y * W + x, y * W + x, W, W, w, h)
            sad, satd = ctx.rd_dist(bl, org, cur)
            for i, b in enumerate(bl):
                o, c = org.ravel()[b["org_off"]:], cur.ravel()[b["cur_off"]:]
                po, pc = C.c_void_p(o.ctypes.data), C.c_void_p(c.ctypes.data)
                assert sad[i] == L.or_sad(po, W, pc, W, int(b["width"]), int(b["height"])), (W, i)
                assert satd[i] == L.or_satd(po, W, pc, W, int(b["width"]), int(b["height"])), (W, i)
    finally:
        ctx.close()


def test_fwd_transform_matches_reference():
    blocks = rdo_golden.tr_blocks()
    resi, ro = _pools([b[5] for b in blocks])
    bl = np.zeros(len(blocks), N.FWD_BLOCK)
    co = 0
    for i, (w, h, th, tv, lf, _r, _c) in enumerate(blocks):
        bl[i] = (ro[i], co, w, w, h, th, tv, lf)
        co += w * h
    ctx = _ctx()
    try:
        coef = ctx.fwd_transform(bl, resi, co)
    finally:
        ctx.close()
    for i, (w, h, *_r, exp) in enumerate(blocks):
        got = coef[bl[i]["dst_off"]:bl[i]["dst_off"] + w * h].reshape(h, w)
        assert np.array_equal(got, exp), (w, h, blocks[i][2:5])


def test_rdo_rejects_bad_sizes():
    ctx = _ctx()
    try:
        bl = np.zeros(1, N.RD_BLOCK)
        bl[0] = (0, 0, 8, 8, 3, 4)
        with pytest.raises(N.VvcrError):
            ctx.rd_dist(bl, np.zeros(64, np.int16), np.zeros(64, np.int16))
        fb = np.zeros(1, N.FWD_BLOCK)
        fb[0] = (0, 0, 64, 64, 64, 1, 1, 0)   # DST7 is at most 32 points
        with pytest.raises(N.VvcrError):
            ctx.fwd_transform(fb, np.zeros(4096, np.int16), 4096)
    finally:
        ctx.close()
