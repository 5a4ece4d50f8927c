"""vvcdec, the DecoderApp-compatible command-line decoder (vvc_amd/app/vvcdec.cpp): bitstream in, YUV
file out, every picture checked against the stream's decoded-picture-hash SEI, exit status = number of
mismatching pictures (DecoderApp's, decmain.cpp:91). The -o file must be byte-identical to DecoderApp's
(md5.json yuv_md5 is the MD5 of DecoderApp's -o file)."""
import hashlib
import os
import subprocess

import pytest

from vvc_amd import stream as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "vvc_amd", "vvcdec")
GOLD = os.path.join(ROOT, "tests", "golden")


def test_vvcdec_built_and_rejects_bad_usage():
    assert os.access(APP, os.X_OK), "vvcdec is not built (__graft_entry__.build())"
    r = subprocess.run([APP], capture_output=True, text=True, timeout=30)
    assert r.returncode == 255 and "usage" in r.stderr
    r = subprocess.run([APP, "-b", os.path.join(GOLD, "streams", "ra416_q32.bin"), "--no-such-option"], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 255 and "unknown option" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ra416_q32", "ailm416_q37", "rageo480_q32", "ra1080l_q32"])
def test_vvcdec_output_equals_decoderapp(name, tmp_path):
    meta = S.load_meta(os.path.join(GOLD, name))
    out = tmp_path / "out.yuv"
    r = subprocess.run([APP, "-b", os.path.join(GOLD, "streams", name + ".bin"), "-o", str(out)], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count(",(OK)]") == meta["pictures"], r.stdout[-2000:]
    assert "%d of %d picture hashes match (OK)" % (meta["pictures"], meta["pictures"]) in r.stdout
    assert hashlib.md5(out.read_bytes()).hexdigest() == meta["yuv_md5"]
