"""The drop-in: the reference's own DecoderApp — DecApp / DecLib of VTM 7.3 compiled
unchanged from /root/reference by oracle/ref.mk — linked against libvvcr.so (oracle/_ref/vtm_vvcr). At
DecLib::executeLoopFilters (DecLib.cpp:560) each picture's descriptors go through vvcr_begin_picture /
vvcr_submit / vvcr_set_loop_filter_params / vvcr_end_picture; libvvcr's final picture (vvcr_read_picture)
overwrites the reference's reconstruction before DecApp writes it and before later pictures predict
from it, and libvvcr's DMVR refinements (vvcr_get_dmvr_deltas) replace the reference's before
CS::setRefinedMotionField. The -o file must be byte-identical to DecoderApp's (md5.json yuv_md5), and the
tool reports how many pictures libvvcr reconstructed differently from the reference's own DecCu (0).

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
@pytest.mark.parametrize("name", ["ra416_q32", "ailm416_q37", "rageo480_q32", "rawp416_q32"])
def test_decoderapp_linked_with_libvvcr(name, tmp_path):
    if not os.access(APP, os.X_OK):
        pytest.fail("oracle/_ref/vtm_vvcr is not built (make -f oracle/ref.mk dropin, in the build container)")
    meta = S.load_meta(os.path.join(GOLD, name))
    out = tmp_path / "out.yuv"
    r = subprocess.run([APP, "-b", os.path.join(GOLD, "streams", name + ".bin"), "-o", str(out)], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "%d pictures decoded through libvvcr, 0 differ" % meta["pictures"] in r.stderr, r.stderr[-2000:]
    assert hashlib.md5(out.read_bytes()).hexdigest() == meta["yuv_md5"]
