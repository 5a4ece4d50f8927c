"""The drop-in: the reference's own DecoderApp — DecApp / DecLib / DecCu of VTM 7.3
compiled unchanged from /root/reference by oracle/ref.mk — linked against libvvcr.so (oracle/_ref/vtm_vvcr),
with the reference's reconstruction and loop filters REPLACED: DecCu parses and derives motion, its calls
into the reference's prediction / transforms / LMCS mapping return without running, and
DecLib::executeLoopFilters (DecLib.cpp:560) hands each picture's descriptors to libvvcr
(vvcr_begin_picture / vvcr_submit / vvcr_set_loop_filter_params / vvcr_end_picture), whose final picture
(vvcr_read_picture) is the only content of the reference's picture buffer, and whose DMVR refinements
(vvcr_get_dmvr_deltas) feed CS::setRefinedMotionField. The tool counts the calls into the reference's
reconstruction that ran (InterpolationFilter::filterHor, motionCompensation, predIntra*,
TrQuant::invTransformNxN, LoopFilter::loopFilterPic, SAOProcess): zero. DecLib's own decoded-picture-hash
check must pass on every picture and the -o file must be byte-identical to DecoderApp's (md5.json).

The binary is built in this container (it needs /root/reference); the GPU box runs the prebuilt one."""
import hashlib
import os
import subprocess

import pytest

from vvc_amd import stream as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "oracle", "_ref", "vtm_vvcr")
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ra416_q32", "ailm416_q37", "rageo480_q32", "rawp416_q32", "ralmgeo416_q32", "ra1080_q32",
                                  "rawpp416_q32", "ratilenf416_q32", "rasub480_q32", "ravb416_q32", "raladf416_q32",
                                  "rarsc416_q32"])
def test_decoderapp_linked_with_libvvcr(name, tmp_path):
    if not os.access(APP, os.X_OK):
        pytest.fail("oracle/_ref/vtm_vvcr is not built (make -f oracle/ref.mk dropin, in the build container)")
    meta = S.load_meta(os.path.join(GOLD, name))
    out = tmp_path / "out.yuv"
    r = subprocess.run([APP, "-b", os.path.join(GOLD, "streams", name + ".bin"), "-o", str(out)], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "%d pictures decoded through libvvcr, 0 calls into the reference's reconstruction" % meta["pictures"] in r.stderr, \
        r.stderr[-2000:]
    assert r.stdout.count("(OK)") == meta["pictures"] and "ERROR" not in r.stdout, r.stdout[-2000:]   # DecLib's SEI MD5 check
    assert hashlib.md5(out.read_bytes()).hexdigest() == meta["yuv_md5"]
