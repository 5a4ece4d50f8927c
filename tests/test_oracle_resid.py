"""Oracle pinning: the C restatement of dequant + LFNST + inverse MTS + JCCR reproduces the reference
decoder's residual (captured at TrQuant::invTransformNxN / invTransformICT) for every TU of the
committed VTM-7.3 streams. CPU only."""
import os

import numpy as np
import pytest

from vvc_amd import stream as S
import oracle_lib as O


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_oracle_residual_matches_reference(golden_dir, name):
    pics = S.load_sequence(os.path.join(golden_dir, name))
    for p in pics:
        got = O.residual_picture(p)
        for c, pl in enumerate("yuv"):
            exp = p["resi_" + pl]
            if c and p["hdr"]["lmcs_enabled"] and p["hdr"]["lmcs_chroma_scale"]:
                continue   # chroma residual scaling is checked with the reconstruction stage
            bad = got[c] != exp
            assert not bad.any(), "POC %d %s: %d samples differ, first %s" % (p["hdr"]["poc"], pl, bad.sum(), np.argwhere(bad)[0])
