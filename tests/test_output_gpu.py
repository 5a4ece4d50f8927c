"""vvcr_write_output (DecoderApp's -o file written by the GPU, include/vvcr.h) against the reference
decoder's own output files (MD5 of the whole file at several output bit depths, tests/golden/<stream>/
output_md5.json) and, per picture, against the C oracle (oracle/oracle_output.c) for parameters the
fixtures do not cover (odd bit depths, other conformance windows). Also the plane MD5s (= the stream's SEI)
of the conformance-window stream ra412c_q32.

Parity unpinned: the reference's own output files cover 8/10/12-bit output with the right/bottom crop
of ra412c_q32 (0, 4, 0, 4) only. 9- and 16-bit output and crops with left/top offsets (`extra` below) are
checked against the C oracle alone, a restatement of TVideoIOYuv::write (VideoIOYuv.cpp) that no
reference-produced file confirms."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch  # noqa: F401  (the HIP runtime before libvvcr creates contexts)

from vvc_amd import decode as D, native as N, stream as S
import oracle_lib as O
from test_output import CASES, CONF

pytestmark = pytest.mark.gpu


def params(fbd=0, conf=(0, 0, 0, 0), clip=0):
    return N.OutputParams(fbd, *conf, clip)


@pytest.mark.parametrize("name", ["ra416_q32", "ra412c_q32"])
def test_write_output_matches_decoderapp_files(golden_dir, name):
    with open(os.path.join(golden_dir, name, "output_md5.json")) as f:
        ref = json.load(f)
    with open(os.path.join(golden_dir, name, "md5.json")) as f:
        meta = json.load(f)
    pics = S.load_sequence(os.path.join(golden_dir, name))
    dec = D.Decoder(pics)
    conf = CONF.get(name, (0, 0, 0, 0))
    hs = {case: {} for case in CASES}
    extra = [params(9, (2, 6, 4, 2)), params(16, (0, 2, 2, 0)), params(8, (4, 0, 0, 4), 1)]
    try:
        for i in range(len(pics)):
            poc, slot = dec.decode_picture(i)
            planes = dec.read(slot)
            assert D.plane_md5s(planes) == meta["poc_plane_md5"][str(poc)], "POC %d planes" % poc
            for case, (fbd, clip) in CASES.items():
                hs[case][poc] = dec.ctx.write_output(slot, params(fbd, conf, clip)).tobytes()
            for op in extra:
                got = dec.ctx.write_output(slot, op)
                want = O.write_output(planes, 10, op.file_bit_depth, (op.conf_left, op.conf_right, op.conf_top, op.conf_bottom),
                                      op.clip_rec709)
                assert np.array_equal(got, want), "POC %d output d%d" % (poc, op.file_bit_depth)
    finally:
        dec.close()
    for case in CASES:
        h = hashlib.md5()
        for poc in sorted(hs[case]):
            h.update(hs[case][poc])
        assert h.hexdigest() == ref[case], case


def test_write_output_to_device_memory(golden_dir):
    pics = S.load_sequence(os.path.join(golden_dir, "ai416_q37"), max_pics=1)
    dec = D.Decoder(pics)
    try:
        _, slot = dec.decode_picture(0)
        op = params(8)
        buf = torch.zeros(dec.ctx.output_bytes(op), dtype=torch.uint8, device="cuda")
        dec.ctx.write_output(slot, op, buf.data_ptr())
        assert np.array_equal(buf.cpu().numpy(), dec.ctx.write_output(slot, op))
    finally:
        dec.close()
