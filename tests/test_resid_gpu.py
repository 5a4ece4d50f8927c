"""Residual parity: libvvcr's dequant + LFNST + inverse transform kernel vs the reference decoder's
residual (TrQuant::invTransformNxN / invTransformICT output) for every TU, and vs the C oracle on the
same descriptors. Bit-exact."""
import os

import numpy as np
import pytest

from vvc_amd import native as N
from vvc_amd import stream as S
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_residual_matches_reference_and_oracle(golden_dir, name):
    pics = S.load_sequence(os.path.join(golden_dir, name))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=2)
    for p in pics:
        ctx.begin_picture(S.pic_params(p, 0, {}, missing_ref_slot=0))
        S.submit(ctx, p)
        ctx.end_picture(N.STAGE_RESID)
        orc = O.residual_picture(p)
        for c, pl in enumerate("yuv"):
            got = ctx.read_plane(N.BUF_RESI, 0, c)
            assert np.array_equal(got, orc[c]), "POC %d %s: GPU != oracle at %d samples" % (
                p["hdr"]["poc"], pl, int((got != orc[c]).sum()))
            if c and p["hdr"]["lmcs_enabled"] and p["hdr"]["lmcs_chroma_scale"]:
                continue
            exp = p["resi_" + pl]
            assert np.array_equal(got, exp), "POC %d %s: %d samples differ from the reference" % (
                p["hdr"]["poc"], pl, int((got != exp).sum()))
    ctx.close()
