"""Host bitstream parser (include/vvcp.h) against the capture fixtures of the reference decoder.

Every picture of the golden streams is parsed from the .bin and its rows are compared field by field
with tests/golden/<stream>/pic_NNN.xz (the reference's CodingStructure after DecLib decoded the
picture, oracle/capture/vtm_capture.cpp): CU / PU / TU rows, coefficient levels, SAO parameters
(merges resolved) and ALF / CC-ALF CTB syntax. Fields that depend on motion derivation (DecCu::
xDeriveCUMV) are excluded until the derivation runs in the parser; the LMCS chroma scale of a TU
(computed by DecCu) likewise. Bit-exact: integer syntax, no tolerance.
"""
import glob
import os

import numpy as np
import pytest

from vvc_amd import capfile, parser

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CU_F = ("x y w h cx cy cw ch chtype predmode qp treetype modetype skip mmvdskip affine affinetype geo bdpcm bdpcmc imv "
        "rootcbf sbtinfo mtsflag lfnst bcw mip isp smvd act cqpadj depth qtdepth firstpu npu firsttu ntu slice yvalid cvalid").split()
PU_F = ("cu x y w h cx cy cw ch chtype idir_l idir_c fidir_l fidir_c mipt mrl merge regmerge mergeidx geodir geoi0 geoi1 mmvd "
        "interdir mv0x mv0y mv1x mv1y ref0 ref1 mrgtype mvrefine ciip").split() + ["aff%d" % i for i in range(12)] + [
        "dmvr_off", "bdof", "dmvr"]
TU_F = "cu chtype depth noresi jccr cadj".split() + ["%s%d" % (f, c) for c in range(3) for f in "x y w h cbf mts coff qp qpts".split()]
CU_MV = {"imv", "bcw", "affinetype"}
PU_MV = {"interdir", "mv0x", "mv0y", "mv1x", "mv1y", "ref0", "ref1", "mrgtype", "mvrefine", "mergeidx", "dmvr_off", "bdof",
         "dmvr"} | {"aff%d" % k for k in range(12)}


def _cols(fields, mask):
    return [i for i, f in enumerate(fields) if f not in mask]


def compare_picture(rows, cap, intra):
    """Returns a list of mismatch descriptions (empty = identical)."""
    out = []
    for name, fields, mask in (("cu", CU_F, set() if intra else CU_MV), ("pu", PU_F, set() if intra else PU_MV),
                               ("tu", TU_F, {"cadj"})):
        a, b = rows[name], cap[name]
        if a.shape != b.shape:
            out.append("%s shape %s vs %s" % (name, a.shape, b.shape))
            continue
        c = _cols(fields, mask)
        d = np.argwhere(a[:, c] != b[:, c])
        if len(d):
            r, k = d[0]
            out.append("%s row %d %s: %d vs %d" % (name, r, fields[c[k]], a[r, c[k]], b[r, c[k]]))
    if not np.array_equal(rows["coef"], cap["coef"]):
        out.append("coef")
    on = cap["sao"][:, :, 0] != 0   # offsets of SAO-off components are not defined
    if not (np.array_equal(rows["sao"][:, :, 0], cap["sao"][:, :, 0]) and np.array_equal(rows["sao"][on], cap["sao"][on])):
        out.append("sao")
    for k in ("alf_ctb_en", "alf_ctb_alt", "alf_ctb_fidx"):
        if not np.array_equal(rows[k], cap[k]):
            out.append(k)
    for c, key in enumerate(("ccalf_en_cb", "ccalf_en_cr")):   # the capture's array is stale when CC-ALF is off
        if cap["hdr"].get(key) and not np.array_equal(rows["ccalf_ctl"][c], cap["ccalf_ctl"][c]):
            out.append("ccalf_ctl[%d]" % c)
    return out


STREAMS = ["ai416_q37", "ailm416_q37", "ra416_q32", "ralm416_q32", "rawp416_q32", "ratile416_q32", "ra412c_q32",
           "ra1080_q32", "ratile1080_q32", "aibdpcm416_q32", "radq0416_q32", "rageo480_q32"]


@pytest.mark.parametrize("stream", STREAMS)
def test_parser_matches_capture(stream):
    data = open(os.path.join(ROOT, "streams", stream + ".bin"), "rb").read()
    caps = sorted(glob.glob(os.path.join(ROOT, stream, "pic_*.xz")))
    s = parser.Stream(data)
    assert len(s) == len(caps)
    for i, path in enumerate(caps):
        cap = capfile.unpack(open(path, "rb").read())
        info = s.info(i)
        assert info["poc"] == cap["hdr"]["poc"]
        assert info["slice_type"] == cap["hdr"]["slice_type"]
        s.parse(i)
        bad = compare_picture(s.rows(i), cap, info["slice_type"] == 2)
        assert not bad, "%s picture %d (POC %d): %s" % (stream, i, info["poc"], "; ".join(bad))


def test_parser_rejects_garbage():
    with pytest.raises(parser.ParseError):
        s = parser.Stream(b"\x00\x00\x01\x00\x79" + bytes(range(40)))
        for i in range(len(s)):
            s.parse(i)
