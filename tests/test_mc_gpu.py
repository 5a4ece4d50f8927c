"""Motion compensation parity: libvvcr prediction planes vs the reference decoder's MC output
(InterPrediction::motionCompensation, captured per CU by oracle/capture) on VTM-7.3 streams.
Reference pictures are the reference decoder's own decoded pictures, so every picture is an
independent check. Bit-exact."""
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S
from helpers import cu_mask, is_inter

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ra416_q32", "rawp416_q32"])
def test_mc_matches_reference(golden_dir, name):
    """Every inter CU (uni/bi/BCW, SbTMVP, GEO, affine+PROF, DMVR, BDOF; explicit weighted prediction in
    rawp416_q32) and the DMVR deltas."""
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    by_poc = {p["hdr"]["poc"]: p for p in pics}
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=20)
    checked = 0
    for p in pics:
        if p["hdr"]["slice_type"] == 2:
            continue
        # put the reference decoder's pictures into DPB slots 0..n
        slot_of = {}
        for l in range(2):
            for r in range(p["hdr"]["num_ref_l%d" % l]):
                poc = int(p["ref_poc"][l][r])
                if poc not in slot_of:
                    slot_of[poc] = len(slot_of) + 1
                    for c, pl in enumerate("yuv"):
                        ctx.write_plane(N.BUF_RECO, slot_of[poc], c, by_poc[poc]["alf_" + pl])
        ctx.begin_picture(S.pic_params(p, 0, slot_of))
        S.submit(ctx, p)
        ctx.end_picture(N.STAGE_INTER)
        exp_d = p["dmvr_delta"].reshape(-1, 2)
        got_d = ctx.dmvr_deltas()
        assert got_d.shape == exp_d.shape and (got_d == exp_d).all(), "POC %d DMVR deltas differ" % p["hdr"]["poc"]
        for c, pl in enumerate("yuv"):
            got = ctx.read_plane(N.BUF_PRED, 0, c)
            m = cu_mask(p, is_inter, c)
            exp = p["pmc_" + pl]
            bad = (got != exp) & m
            assert not bad.any(), "POC %d comp %s: %d/%d samples differ, first at %s" % (
                p["hdr"]["poc"], pl, bad.sum(), m.sum(), np.argwhere(bad)[0])
            checked += int(m.sum())
    ctx.close()
    assert checked > 0
