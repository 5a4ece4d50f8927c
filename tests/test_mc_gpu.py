"""Motion compensation parity: libvvcr prediction planes vs the reference decoder's MC output
(InterPrediction::motionCompensation, captured per CU by oracle/capture) on VTM-7.3 streams.
Reference pictures are the reference decoder's own decoded pictures, so every picture is an
independent check. Bit-exact."""
import os
import subprocess
import sys

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
    check_mc(golden_dir, name)


@pytest.mark.parametrize("name", ["ra416_q32", "rawp416_q32"])
def test_affine_global_fallback_matches_reference(golden_dir, name):
    """k_mc_affine's path for sub-block windows whose union does not fit its LDS buffers (strongly
    diverging affine MVs: windows read straight from the reference picture), forced on every affine tile
    with VVCR_AFF_FALLBACK=1 (read once per process, hence the child process)."""
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_mc_gpu as T; T.check_mc(%r, %r); print('ok')"
            % (here, os.path.dirname(here), golden_dir, name))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, VVCR_AFF_FALLBACK="1"),
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def check_mc(golden_dir, name):
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
