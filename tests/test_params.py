"""Picture parameters and ALF filters built by the host parser (vvcp_picture_params / vvcp_alf_filters)
against the values the capture fixtures record from the reference decoder's state
(oracle/capture/vtm_capture.cpp dumpDescriptors / dumpAlf: slice and picture header fields, reference
POCs, weighted-prediction tables after Slice::initWpScaling, chroma QP mapping tables, tiles, the LMCS
model of Reshape::constructReshaper, AdaptiveLoopFilter::reconstructCoeffAPSs). Compared where the
reference's value is defined: the capture keeps stale LMCS tables when LMCS is off, stale chroma ALF
alternatives beyond the APS's count, and WeightPrediction's per-call scratch fields. Bit-exact.
"""
import glob
import os

import numpy as np
import pytest

from vvc_amd import capfile, parser, stream

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STREAMS = ["ai416_q37", "ailm416_q37", "ra416_q32", "ralm416_q32", "rawp416_q32", "ratile416_q32", "ra412c_q32",
           "ra1080_q32", "ratile1080_q32", "rawp1080_q32", "aibdpcm416_q32", "radq0416_q32", "rageo480_q32"]


def _fields(pp):
    out = {}
    for n, _ in pp._fields_:
        v = getattr(pp, n)
        out[n] = np.ctypeslib.as_array(v).copy() if hasattr(v, "_length_") else v
    return out


def compare_params(ours, cap):
    ref = _fields(stream.pic_params(cap, 0, {int(q): 0 for q in cap["ref_poc"].ravel()}))
    ours = _fields(ours)
    bad = []
    nref = ref["num_ref"]
    for k in ref:
        a, b = ours[k], ref[k]
        if k in ("slot", "ref_slot"):
            continue
        if k.startswith("lmcs_") and k != "lmcs_enabled" and not ref["lmcs_enabled"]:
            continue
        if k in ("ref_poc", "ref_lt", "wp"):
            a = np.concatenate([a[l][:nref[l]].ravel() if k != "wp" else a[l][:nref[l], :, :4].ravel() for l in range(2)])
            b = np.concatenate([b[l][:nref[l]].ravel() if k != "wp" else b[l][:nref[l], :, :4].ravel() for l in range(2)])
        if k == "chroma_qp_map":   # defined for qp >= -QpBdOffsetC
            off = 6 * (cap["hdr"]["bitdepth_c"] - 8)
            a, b = a[:, 64 - off:], b[:, 64 - off:]
        if k in ("num_tile_cols", "num_tile_rows"):   # 0 (captures without a tile layout) = one tile
            a, b = max(a, 1), max(b, 1)
        if k in ("tile_col_bd", "tile_row_bd"):
            if "tile_col_bd" not in cap:
                continue
            n = ref["num_tile_cols" if "col" in k else "num_tile_rows"] + 1
            a, b = a[:n], b[:n]
        if not np.array_equal(np.asarray(a), np.asarray(b)):
            bad.append(k)
    return bad


def compare_alf(A, cap):
    h = cap["hdr"]
    bad = []
    if not (h["alf_enabled"] and any(h["alf_slice_en%d" % c] for c in range(3))):
        return bad
    if h["alf_slice_en0"]:
        n = len(cap["alf_aps_ids"])
        if len(A["luma_coef"]) != 16 + n:
            bad.append("luma set count")
        elif not (np.array_equal(A["luma_coef"][16:], cap["alf_coef_aps"][:n]) and
                  np.array_equal(A["luma_clip"][16:], cap["alf_clip_aps"][:n]) and
                  np.array_equal(A["luma_coef"][:16], cap["alf_fixed"]) and
                  (A["luma_clip"][:16] == cap["alf_clip_default"]).all()):
            bad.append("luma")
    if h["alf_slice_en1"] or h["alf_slice_en2"]:
        nalt = int((A["chroma_coef"] != 0).any(axis=1).sum())
        if not (np.array_equal(A["chroma_coef"][:nalt], cap["alf_chroma_coef"][:nalt]) and
                np.array_equal(A["chroma_clip"][:nalt], cap["alf_chroma_clip"][:nalt])):
            bad.append("chroma")
    for c, key in enumerate(("ccalf_en_cb", "ccalf_en_cr")):
        if h[key]:
            cnt = cap["ccalf_info"][c][0]
            if not np.array_equal(A["cc_coef"][c][:cnt], cap["ccalf_coef"][c][:cnt]):
                bad.append("cc%d" % c)
    return bad


@pytest.mark.parametrize("name", STREAMS)
def test_params_match_capture(name):
    s = parser.Stream(open(os.path.join(ROOT, "streams", name + ".bin"), "rb").read())
    for i, path in enumerate(sorted(glob.glob(os.path.join(ROOT, name, "pic_*.xz")))):
        cap = capfile.unpack(open(path, "rb").read())
        bad = compare_params(s.pic_params(i), cap) + compare_alf(s.alf_filters(i), cap)
        assert not bad, "%s picture %d: %s" % (name, i, bad)
