"""Oracle pinning for the in-loop filters: the C restatements of SAO and ALF/CC-ALF reproduce the
reference decoder's per-stage pictures (captured around SAOProcess / ALFProcess). CPU only."""
import os

import numpy as np
import pytest

from vvc_amd import stream as S
import oracle_lib as O


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_oracle_sao_alf_match_reference(golden_dir, name):
    for p in S.load_sequence(os.path.join(golden_dir, name)):
        poc = p["hdr"]["poc"]
        sao = O.sao_picture(p, [p["dbk_" + c] for c in "yuv"])
        for c, pl in enumerate("yuv"):
            bad = sao[c] != p["sao_" + pl]
            assert not bad.any(), "SAO POC %d %s: %d differ, first %s" % (poc, pl, bad.sum(), np.argwhere(bad)[0])
        if not p["hdr"]["alf_enabled"]:
            continue
        alf = O.alf_picture(p, [p["sao_" + c] for c in "yuv"])
        for c, pl in enumerate("yuv"):
            bad = alf[c] != p["alf_" + pl]
            assert not bad.any(), "ALF POC %d %s: %d differ, first %s" % (poc, pl, bad.sum(), np.argwhere(bad)[0])


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32"])
def test_oracle_deblocking_matches_reference(golden_dir, name):
    for p in S.load_sequence(os.path.join(golden_dir, name)):
        poc = p["hdr"]["poc"]
        out = O.deblock_picture(p, [p["dbkin_" + c] for c in "yuv"])
        for c, pl in enumerate("yuv"):
            bad = out[c] != p["dbk_" + pl]
            assert not bad.any(), "DBK POC %d %s: %d differ, first %s" % (poc, pl, bad.sum(), np.argwhere(bad)[0])
