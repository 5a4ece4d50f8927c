"""Reconstruction parity on the GPU: residual + motion compensation + intra / CIIP dependency waves
reproduce the reference decoder's reconstructed picture before the in-loop filters (captured at
DecLib::executeLoopFilters). Reference pictures are the reference decoder's own output. Bit-exact."""
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32", "ailm416_q37", "ralm416_q32", "rawp416_q32"])
def test_reconstruction_matches_reference(golden_dir, name):
    pics = S.load_sequence(os.path.join(golden_dir, name))
    by_poc = {p["hdr"]["poc"]: p for p in pics}
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=20)
    for p in pics:
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
        ctx.end_picture(N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA)
        for c, pl in enumerate("yuv"):
            got = ctx.read_plane(N.BUF_RECO, 0, c)
            exp = p["prelf_" + pl]
            bad = got != exp
            assert not bad.any(), "POC %d %s: %d differ, first %s" % (p["hdr"]["poc"], pl, bad.sum(), np.argwhere(bad)[0])
    ctx.close()
