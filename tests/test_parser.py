"""Host bitstream parser (include/vvcp.h) against the capture fixtures of the reference decoder.

Every picture of the golden streams is parsed from the .bin and its rows are compared field by field
with tests/golden/<stream>/pic_NNN.xz (the reference's CodingStructure after DecLib decoded the
picture, oracle/capture/vtm_capture.cpp): CU / PU / TU rows, coefficient levels, SAO parameters
(merges resolved) and ALF / CC-ALF CTB syntax. Motion is derived in decoding order (vvcp_derive_motion:
merge / AMVP / affine / SbTMVP / GEO / MMVD / history candidates, TMVP from the refined field of the
collocated picture) and compared too: the MV fields of the rows, the 4x4 motion field and the GEO
candidate rows. The DMVR refinements that feed later pictures' temporal candidates are the capture's
own (dmvr_delta) here; tests/test_decode_gpu.py closes that loop with the GPU's. The LMCS chroma
scale of a TU (computed by DecCu) is not a parser output. Bit-exact: integer syntax, no tolerance.
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


def _cols(fields, mask):
    return [i for i, f in enumerate(fields) if f not in mask]


def compare_picture(rows, cap):
    """Returns a list of mismatch descriptions (empty = identical)."""
    out = []
    for name, fields, mask in (("cu", CU_F, set()), ("pu", PU_F, set()), ("tu", TU_F, {"cadj"})):
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
    if "motion" in rows:
        if rows["motion"].shape != cap["motion"].shape:
            out.append("motion shape")
        else:
            d = np.argwhere(rows["motion"] != cap["motion"])
            if len(d):
                out.append("motion at 4x4 (%d,%d) field %d (%d diffs)" % (d[0][1], d[0][0], d[0][2], len(d)))
        g = cap["geo"]   # captured in reconstruction order; the parser emits CU order
        g = g[np.argsort(g[:, 0], kind="stable")] if len(g) else g
        if not np.array_equal(rows["geo"], g):
            out.append("geo")
    return out


STREAMS = ["ai416_q37", "ailm416_q37", "ra416_q32", "ralm416_q32", "rawp416_q32", "ratile416_q32", "ra412c_q32",
           "ra1080_q32", "ratile1080_q32", "rawp1080_q32", "aibdpcm416_q32", "radq0416_q32", "rageo480_q32",
           "ra2160n_q27", "ra2160l_q32", "ra2160l_q27", "ra2160_q27", "ra2160_q32", "ra1080l_q32", "ra4320t_q32", "ralmgeo416_q32",
           "rawpp416_q32", "ratilenf416_q32", "rawpp1080_q32", "ratilenf1080_q32", "rasub480_q32",
           "ravb416_q32", "ravb416b_q37", "raladf416_q32",
           "rarsc416_q32"]


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
        s.derive(i)
        s.refine(i, cap["dmvr_delta"])
        bad = compare_picture(s.rows(i), cap)
        assert not bad, "%s picture %d (POC %d): %s" % (stream, i, info["poc"], "; ".join(bad))


def test_motion_needs_order():
    """The collocated picture must be refined before a picture that reads it is derived."""
    data = open(os.path.join(ROOT, "streams", "ra416_q32.bin"), "rb").read()
    s = parser.Stream(data)
    s.parse(0)
    s.parse(1)
    with pytest.raises(parser.ParseError):
        s.derive(1)             # POC 16 reads POC 0's motion, which is not refined yet
    with pytest.raises(parser.ParseError):
        s.refine(0)             # not derived
    s.derive(0)
    s.refine(0)
    s.derive(1)


def test_parser_rejects_garbage():
    with pytest.raises(parser.ParseError):
        s = parser.Stream(b"\x00\x00\x01\x00\x79" + bytes(range(40)))
        for i in range(len(s)):
            s.parse(i)


_FUZZ = r'''
import random, sys
sys.path.insert(0, sys.argv[1])
from vvc_amd import parser
data = open(sys.argv[2], "rb").read()
starts = [i + 3 for i in range(len(data) - 3) if data[i:i + 3] == b"\x00\x00\x01"]
rng = random.Random(int(sys.argv[3]))
ok = err = 0
for trial in range(int(sys.argv[4])):
    b = bytearray(data)
    for _ in range(rng.randint(1, 3)):   # flip bits in the NAL header / parameter set / picture and slice headers
        p = rng.choice(starts) + rng.randint(0, 24)
        if p < len(b):
            b[p] ^= 1 << rng.randint(0, 7)
    try:
        s = parser.Stream(bytes(b))
        for i in range(len(s)):
            s.parse(i)
            s.derive(i)
            s.refine(i)
        ok += 1
    except parser.ParseError:
        err += 1
print(ok, err)
'''


@pytest.mark.parametrize("stream,seed", [("ra416_q32", 1), ("rawp416_q32", 2), ("ratile416_q32", 3), ("rawpp416_q32", 4),
                                         ("ratilenf416_q32", 5)])
def test_parser_survives_corrupted_headers(stream, seed, tmp_path):
    """Malformed parameter sets and picture / slice headers (bit flips near every NAL start) must end in a
    ParseError or a decode, never in an out-of-bounds access: the parser runs in-process under every
    decode. A child process, so a crash fails the test instead of the runner."""
    import subprocess
    import sys
    script = tmp_path / "fuzz.py"
    script.write_text(_FUZZ)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, str(script), repo, os.path.join(ROOT, "streams", stream + ".bin"), str(seed), "150"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    ok, err = map(int, r.stdout.split())
    assert err > 0   # the mutations reach checked syntax
