"""EncoderApp drop-in (SURVEY.md §8 north_star: "DecoderApp and EncoderApp link unchanged"; INTEGRATION.md
§2b). oracle/_ref/vtm_enc_vvcr is the reference's EncoderApp / EncoderLib / CommonLib, unchanged, linked
against libvvcr.so (oracle/capture/enc_vvcr.cpp, oracle/ref.mk `encdropin`): the Hadamard SATD of the
merge-candidate pass (EncCu::xCheckRDCostMerge2Nx2N, EncCu.cpp:2421-2451) runs through vvcr_rd_dist on the
GPU. The bitstream must be byte-identical to plain EncoderApp's on the same input and configuration, with
SATD calls actually routed. Input: synthetic 416x240 content (tools/gen_synth.py, seed 1234), 3 pictures,
the low-delay configuration tests/golden/enc/lowdelay_small.cfg."""
import os
import re
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
CFG = os.path.join(ROOT, "tests", "golden", "enc", "lowdelay_small.cfg")


@pytest.mark.gpu
def test_encoderapp_with_gpu_merge_satd_is_byte_identical(tmp_path):
    enc, enc_gpu = os.path.join(REF, "EncoderApp"), os.path.join(REF, "vtm_enc_vvcr")
    if not (os.path.exists(enc) and os.path.exists(enc_gpu)):
        pytest.skip("reference EncoderApp / vtm_enc_vvcr not built (oracle/ref.mk)")
    yuv = str(tmp_path / "s416.yuv")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_synth.py"), "416", "240", "3", yuv], check=True)
    args = ["-c", CFG, "-i", yuv, "-wdt", "416", "-hgt", "240", "-f", "3", "-q", "32", "-o", "/dev/null"]
    out, secs = {}, {}
    for name, exe in (("cpu", enc), ("gpu", enc_gpu)):
        b = str(tmp_path / (name + ".bin"))
        t0 = time.perf_counter()
        r = subprocess.run([exe] + args + ["-b", b], capture_output=True, text=True, timeout=300)
        secs[name] = time.perf_counter() - t0
        assert r.returncode == 0, "%s: rc %d\n%s" % (name, r.returncode, (r.stdout + r.stderr)[-2000:])
        out[name] = (open(b, "rb").read(), r.stderr)
    m = re.search(r"vvcr-enc: routed (\d+) merge-pass SATD calls to the GPU, (\d+) fell back", out["gpu"][1])
    assert m, out["gpu"][1][-1000:]
    routed = int(m.group(1))
    print("EncoderApp %.1f s, with GPU merge SATD %.1f s: %d calls routed, %s fell back, %d bytes" % (
        secs["cpu"], secs["gpu"], routed, m.group(2), len(out["gpu"][0])))
    assert routed > 0
    assert out["gpu"][0] == out["cpu"][0], "bitstreams differ"
