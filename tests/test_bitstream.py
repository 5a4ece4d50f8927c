"""The bitstream decode path (vvc_amd/bitstream.py): host parser -> motion derivation with the GPU's
DMVR feedback -> native planning (vvcp_plan_picture) -> libvvcr, from the .bin alone.

CPU: the native plan of every parsed picture (rows, parameters and ALF from the parser; the capture's
DMVR deltas stand in for the GPU's) has the same work lists as the plan built from the reference
decoder's own descriptors (vvc_amd/stream.py plan_picture), and the decode plan's DPB / output order.
GPU: every picture's plane MD5s and the output YUV file's MD5 equal DecoderApp's (md5.json), with the
DMVR deltas of collocated pictures coming from the GPU (vvcr_picture_dmvr_deltas)."""
import ctypes as C
import glob
import hashlib
import os

import numpy as np
import pytest

from vvc_amd import bitstream as B
from vvc_amd import capfile, parser
from vvc_amd import native as N
from vvc_amd import stream as S

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bin(name):
    return open(os.path.join(ROOT, "streams", name + ".bin"), "rb").read()


@pytest.mark.parametrize("name", ["ra416_q32", "rageo480_q32", "ailm416_q37", "ratile416_q32"])
def test_native_plan_matches_capture_plan(name):
    s = parser.Stream(_bin(name))
    L = B._bind(N.lib())
    plan = B.Plan(s, 16)
    inf = plan.info[0]
    sp = N.SeqParams(inf["width"], inf["height"], 1, inf["bit_depth"], inf["ctu_log2"], 16, 0)
    for i, f in enumerate(sorted(glob.glob(os.path.join(ROOT, name, "pic_*.xz")))):
        cap = capfile.unpack(open(f, "rb").read())
        s.parse(i)
        s.derive(i)
        s.refine(i, cap["dmvr_delta"])
        rs = plan.ref_slots(i)
        h = C.c_void_p()
        assert L.vvcp_plan_picture(s.h, i, C.byref(sp), plan.slot[i], rs.ctypes.data, N.STAGE_ALL, C.byref(h)) == 0, \
            L.vvcp_last_error().decode()
        ours = N.Picture.wrap(h)
        slot_of = {int(cap["ref_poc"][l][r]): int(rs[l, r]) for l in range(2) for r in range(cap["hdr"]["num_ref_l%d" % l])}
        ref = S.plan_picture(cap, plan.slot[i], slot_of, dpb_slots=16)
        assert ours.work_counts() == ref.work_counts(), "picture %d" % i
        ours.close()
        ref.close()


def test_decode_plan_order_and_slots():
    s = parser.Stream(_bin("ra1080l_q32"))
    plan = B.Plan(s, 8)
    pocs = [inf["poc"] for inf in plan.info]
    assert [pocs[i] for i in plan.out_order] == sorted(pocs)
    n = len(pocs)
    for j in range(n):   # no slot is overwritten while a later picture still reads it or it awaits output
        for i in range(j):
            if plan.slot[i] == plan.slot[j]:
                assert plan.last_use[i] < j
        for l in range(2):
            for poc in plan.refs[j][l]:
                assert plan.slot[plan._find(j, poc)] in plan.ref_slots(j)[l]
    with pytest.raises(RuntimeError):
        B.Plan(s, 2)     # an RA GOP needs more than two pictures in the DPB


@pytest.mark.parametrize("name", ["ra1080l_q32", "ra416_q32", "ai416_q37", "ratile416_q32"])
def test_native_decode_plan_matches(name):
    """vvcp_decode_plan (the plan the native loop follows) equals the Python restatement above."""
    s = parser.Stream(_bin(name))
    L = B._bind(N.lib())
    n = len(s)
    for base, nslots in ((0, 16), (5, 9)):
        slots, order = (C.c_int32 * n)(), (C.c_int32 * n)()
        m = L.vvcp_decode_plan(s.h, base, nslots, slots, order)
        plan = B.Plan(s, nslots, base)
        assert list(slots) == plan.slot
        assert list(order)[:m] == plan.out_order
    if name.startswith("ra"):   # a random-access GOP needs more than one picture in the DPB
        assert L.vvcp_decode_plan(s.h, 0, 1, None, None) < 0


def test_decode_releases_handles_of_pictures_never_collocated():
    """vvcp_decode's handle release: a referenced picture with DMVR sub-blocks that no later
    picture uses as its collocated picture must not pin every later handle. On the 33-picture stream, with
    every picture assumed to have DMVR sub-blocks and no handles kept beyond the policy, the live handles
    stay within the DPB's reference span instead of growing with the stream."""
    s = parser.Stream(_bin("ra1080l_q32"))
    L = B._bind(N.lib())
    n = len(s)
    assert n > 24
    for keep in (0, 4, 24):
        peak = L.vvcp_decode_live_bound(s.h, 0, 16, keep)
        assert 0 < peak <= keep + 1 + 16, (keep, peak)
    assert L.vvcp_decode_live_bound(s.h, 0, 16, 0) < n // 2
    assert L.vvcp_decode_live_bound(s.h, 0, 16, -1) < 0


STREAMS = ["ai416_q37", "ailm416_q37", "ra416_q32", "ralm416_q32", "rawp416_q32", "ratile416_q32", "ra412c_q32",
           "ra1080_q32", "ratile1080_q32", "rawp1080_q32", "ra1080l_q32", "aibdpcm416_q32", "radq0416_q32", "rageo480_q32",
           "ra2160_q27", "ra2160_q32", "ra2160n_q27", "ra2160l_q32", "ra2160l_q27", "ralmgeo416_q32",
           # WPP (entropy coding sync) and tiles / slices without loop filtering across them (round 6)
           "rawpp416_q32", "ratilenf416_q32", "rawpp1080_q32", "ratilenf1080_q32", "rasub480_q32",
           "ravb416_q32", "ravb416b_q37", "raladf416_q32",
           "rarsc416_q32"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", STREAMS)
def test_bitstream_decode_matches_decoderapp(name):
    meta = S.load_meta(os.path.join(ROOT, name))
    data = _bin(name)
    s = parser.Stream(data)
    inf = s.info(0)
    s.close()
    op = N.OutputParams(0, inf["conf_left"], inf["conf_right"], inf["conf_top"], inf["conf_bottom"], 0)
    planes, yuv = {}, hashlib.md5()
    ctx = [None]

    def on_output(poc, slot):
        c = ctx[0]
        planes[poc] = [hashlib.md5(np.ascontiguousarray(c.read_plane(N.BUF_RECO, slot, k)).astype("<u2").tobytes()).hexdigest()
                       for k in range(3)]
        yuv.update(c.write_output(slot, op).tobytes())

    c = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=16)
    ctx[0] = c
    try:
        order, _ = B.decode_bitstream(data, ctx=c, on_output=on_output)
    finally:
        c.close()
    assert len(order) == meta["pictures"]
    for poc, exp in meta["poc_plane_md5"].items():
        assert planes[int(poc)] == exp, "POC %s differs" % poc
    assert yuv.hexdigest() == meta["yuv_md5"]
