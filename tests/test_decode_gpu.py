"""End-to-end parity: every picture of each stream reconstructed by libvvcr from its descriptors alone
(references are libvvcr's own output in its device DPB) matches the reference decoder's output
picture MD5s (= the stream's decoded-picture-hash SEI) and the MD5 of DecoderApp's YUV file."""
import os

import pytest

from vvc_amd import decode as D
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32", "ra1080_q32", "ailm416_q37", "ralm416_q32", "rawp416_q32", "ra2160_q27"])
def test_decode_matches_reference_md5(golden_dir, name):
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    md5, yuv = D.decode_and_hash(pics)
    for poc, exp in meta["poc_plane_md5"].items():
        assert md5[int(poc)] == exp, "POC %s: plane MD5 %s != reference %s" % (poc, md5[int(poc)], exp)
    assert yuv == meta["yuv_md5"]
