"""Motion compensation against the reference's own interpolation filters: known-answer vectors made by
oracle/capture/mc_kat.cpp (tools/make_mc_kat.sh) from InterpolationFilter::filterHor / filterVer
(InterpolationFilter.cpp:743,828) driven as InterPrediction::xPredInterBlk does (InterPrediction.cpp:
698-804), with AreaBuf::addAvg for bi-prediction. Each vector: two random 10-bit reference pictures and
a 128x128 picture tiled with 4x4..32x32 blocks, random motion (every luma / chroma fraction, up to 56
samples past the picture edges, uni from either list, bi, IMV_HPEL alternative half-sample filter).

CPU: the vectors' layout and coverage. GPU: the blocks go through the C-ABI as CUs / PUs of one B
picture (vvcr_submit, vvcr_end_picture_stages(VVCR_STAGE_INTER)) whose references are the vectors'
pictures; the prediction planes (VVCR_BUF_PRED) equal the reference's, sample for sample."""
import glob
import os

import numpy as np
import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mc_kat")
FILES = sorted(glob.glob(os.path.join(ROOT, "kat_*.bin")))

# row layouts of include/vvcr.h (every field int32)
CU_FIELDS = ("x y w h cx cy cw ch chtype predmode qp treetype modetype skip mmvdskip affine affinetype geo bdpcm bdpcmc "
             "imv rootcbf sbtinfo mtsflag lfnst bcw mip isp smvd act cqpadj depth qtdepth firstpu npu firsttu ntu slice "
             "yvalid cvalid").split()
PU_FIELDS = ("cu x y w h cx cy cw ch chtype idir_l idir_c fidir_l fidir_c mipt mrl merge regmerge mergeidx geodir geoi0 "
             "geoi1 mmvd interdir mv0x mv0y mv1x mv1y ref0 ref1 mrgtype mvrefine ciip").split() + \
            ["aff%d" % k for k in range(12)] + ["dmvr_off", "bdof", "dmvr"]
TU_FIELDS = 6 + 27
IMV_HPEL, BCW_DEFAULT = 3, 2


def load(path):
    raw = open(path, "rb").read()
    hdr = np.frombuffer(raw[:20], "<i4")
    assert hdr[0] == 0x544B434D
    W, H, bd, n = (int(v) for v in hdr[1:])
    o = 20
    sizes = [W * H, W * H // 4, W * H // 4]

    def planes(o):
        out = []
        for c, s in enumerate(sizes):
            sh = (H, W) if c == 0 else (H // 2, W // 2)
            out.append(np.frombuffer(raw[o:o + 2 * s], "<i2").reshape(sh).copy())
            o += 2 * s
        return out, o
    ref0, o = planes(o)
    ref1, o = planes(o)
    blocks = np.frombuffer(raw[o:o + 40 * n], "<i4").reshape(n, 10).copy()
    o += 40 * n
    exp, o = planes(o)
    assert o == len(raw)
    return dict(W=W, H=H, bd=bd, refs=(ref0, ref1), blocks=blocks, expected=exp)


def test_vectors_cover_the_filter_cases():
    assert len(FILES) >= 6
    fx, fy, cf, dirs, sizes, alt, outside = set(), set(), set(), set(), set(), 0, 0
    for f in FILES:
        k = load(f)
        W, H = k["W"], k["H"]
        covered = np.zeros((H // 4, W // 4), np.int32)
        for x, y, w, h, d, m0x, m0y, m1x, m1y, a in k["blocks"]:
            covered[y // 4:(y + h) // 4, x // 4:(x + w) // 4] += 1
            dirs.add(int(d))
            sizes.add((int(w), int(h)))
            alt += int(a)
            for l, (mx, my) in enumerate(((m0x, m0y), (m1x, m1y))):
                if not (int(d) >> l) & 1:
                    continue
                fx.add(mx & 15); fy.add(my & 15); cf.add(mx & 31)
                if x + (mx >> 4) + w <= 0 or x + (mx >> 4) >= W or y + (my >> 4) + h <= 0 or y + (my >> 4) >= H:
                    outside += 1
        assert (covered == 1).all()      # the blocks tile the picture once
        for p in k["expected"]:
            assert 0 <= p.min() and p.max() <= (1 << k["bd"]) - 1
    assert fx == set(range(16)) and fy == set(range(16)) and cf == set(range(32))
    assert dirs == {1, 2, 3} and (4, 4) in sizes and (32, 32) in sizes and alt > 50 and outside > 20


def _descriptors(k):
    n = len(k["blocks"])
    cu = np.zeros((n, len(CU_FIELDS)), np.int32)
    pu = np.zeros((n, len(PU_FIELDS)), np.int32)
    tu = np.zeros((n, TU_FIELDS), np.int32)
    C = {f: i for i, f in enumerate(CU_FIELDS)}
    P = {f: i for i, f in enumerate(PU_FIELDS)}
    for i, (x, y, w, h, d, m0x, m0y, m1x, m1y, a) in enumerate(k["blocks"]):
        for f, v in dict(x=x, y=y, w=w, h=h, cx=x // 2, cy=y // 2, cw=w // 2, ch=h // 2, predmode=0, qp=32,
                         imv=IMV_HPEL if a else 0, bcw=BCW_DEFAULT, firstpu=i, npu=1, firsttu=i, ntu=1,
                         yvalid=1, cvalid=1).items():
            cu[i, C[f]] = v
        for f, v in dict(cu=i, x=x, y=y, w=w, h=h, cx=x // 2, cy=y // 2, cw=w // 2, ch=h // 2, interdir=d,
                         mv0x=m0x if d & 1 else 0, mv0y=m0y if d & 1 else 0, mv1x=m1x if d & 2 else 0,
                         mv1y=m1y if d & 2 else 0, ref0=0 if d & 1 else -1, ref1=0 if d & 2 else -1).items():
            pu[i, P[f]] = v
        tu[i, 0] = i
        for c, (bx, by, bw, bh) in enumerate(((x, y, w, h), (x // 2, y // 2, w // 2, h // 2), (x // 2, y // 2, w // 2, h // 2))):
            tu[i, 6 + 9 * c:6 + 9 * c + 9] = (bx, by, bw, bh, 0, 0, -1, 32, 32)
    motion = np.zeros(((k["H"] // 4) * (k["W"] // 4), 10), np.int32)
    return cu, pu, tu, motion


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_mc_matches_reference_filters(path):
    from vvc_amd import native as N
    k = load(path)
    ctx = N.Context(k["W"], k["H"], bit_depth=k["bd"], ctu_log2=7, dpb_slots=3)
    try:
        for s, planes in ((1, k["refs"][0]), (2, k["refs"][1])):
            for c, pl in enumerate(planes):
                ctx.write_plane(N.BUF_RECO, s, c, pl)
        pp = N.PicParams()
        pp.poc, pp.slot, pp.slice_type, pp.slice_qp = 8, 0, 0, 32
        pp.num_ref[0] = pp.num_ref[1] = 1
        pp.ref_slot[0][0], pp.ref_slot[1][0] = 1, 2
        pp.ref_poc[0][0], pp.ref_poc[1][0] = 0, 16
        pp.dbk_disable, pp.max_tb_log2 = 1, 6
        cu, pu, tu, motion = _descriptors(k)
        ctx.begin_picture(pp)
        ctx.submit(cu, pu, tu, np.zeros(1, np.int32), motion, np.zeros((0, 13), np.int32))
        ctx.end_picture(N.STAGE_INTER)
        for c in range(3):
            got = np.asarray(ctx.read_plane(N.BUF_PRED, 0, c))
            exp = k["expected"][c]
            bad = np.argwhere(got != exp)
            assert bad.size == 0, "component %d: %d samples differ, first at %s (got %d, reference %d)" % (
                c, len(bad), tuple(bad[0]), got[tuple(bad[0])], exp[tuple(bad[0])])
    finally:
        ctx.close()
