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
    # speed record (VVCR_RECORD_DIR): the link-time binding makes one synchronous GPU round trip per SATD (one
    # staged upload, the launches, one read-back),
    # because the reference's merge loop consumes each candidate's cost before it forms the next
    # (EncCu.cpp:2421-2451); DESIGN.md §9 and bench_rdo.py give the batched entry's rate
    rec = os.environ.get("VVCR_RECORD_DIR")
    if rec:
        import json
        os.makedirs(rec, exist_ok=True)
        with open(os.path.join(rec, "enc_dropin_speed.json"), "w") as f:
            json.dump({"input": "416x240 synthetic, 3 pictures, lowdelay_small.cfg, QP 32", "encoderapp_s": round(secs["cpu"], 3),
                       "encoderapp_gpu_merge_satd_s": round(secs["gpu"], 3), "routed_calls": routed,
                       "fallback_calls": int(m.group(2)), "bytes": len(out["gpu"][0]),
                       "us_added_per_routed_call": round((secs["gpu"] - secs["cpu"]) / max(routed, 1) * 1e6, 2),
                       "bitstreams_identical": out["gpu"][0] == out["cpu"][0]}, f, indent=1)
    assert routed > 0
    assert out["gpu"][0] == out["cpu"][0], "bitstreams differ"
