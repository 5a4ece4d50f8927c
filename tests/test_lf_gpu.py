"""In-loop filter parity on the GPU: SAO and ALF/CC-ALF kernels applied to the reference decoder's
deblocked picture reproduce its SAO and ALF pictures (and the C oracle). Bit-exact."""
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_sao_alf_match_reference(golden_dir, name):
    pics = S.load_sequence(os.path.join(golden_dir, name))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=2)
    for p in pics:
        for stages, src, dst in ((N.STAGE_SAO, "dbk", "sao"), (N.STAGE_SAO | N.STAGE_ALF, "dbk", "alf"),
                                 (N.STAGE_ALF, "sao", "alf")):
            for c, pl in enumerate("yuv"):
                ctx.write_plane(N.BUF_RECO, 0, c, p[src + "_" + pl])
            ctx.begin_picture(S.pic_params(p, 0, {}, missing_ref_slot=0))
            S.submit(ctx, p)
            S.set_loop_filter_params(ctx, p)
            ctx.end_picture(stages)
            for c, pl in enumerate("yuv"):
                got = ctx.read_plane(N.BUF_RECO, 0, c)
                bad = got != p[dst + "_" + pl]
                assert not bad.any(), "POC %d %s %s->%s: %d differ, first %s" % (
                    p["hdr"]["poc"], pl, src, dst, bad.sum(), np.argwhere(bad)[0])
    ctx.close()


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_deblocking_matches_reference(golden_dir, name):
    """DBK alone (dbkin -> dbk) and the whole loop-filter chain (dbkin -> DBK -> SAO -> ALF -> alf)."""
    pics = S.load_sequence(os.path.join(golden_dir, name))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=2)
    for p in pics:
        for stages, dst in ((N.STAGE_DBK, "dbk"), (N.STAGE_DBK | N.STAGE_SAO | N.STAGE_ALF, "alf")):
            for c, pl in enumerate("yuv"):
                ctx.write_plane(N.BUF_RECO, 0, c, p["dbkin_" + pl])
            ctx.begin_picture(S.pic_params(p, 0, {}, missing_ref_slot=0))
            S.submit(ctx, p)
            S.set_loop_filter_params(ctx, p)
            ctx.end_picture(stages)
            for c, pl in enumerate("yuv"):
                got = ctx.read_plane(N.BUF_RECO, 0, c)
                bad = got != p[dst + "_" + pl]
                assert not bad.any(), "POC %d %s dbkin->%s: %d differ, first %s" % (
                    p["hdr"]["poc"], pl, dst, bad.sum(), np.argwhere(bad)[0])
    ctx.close()
