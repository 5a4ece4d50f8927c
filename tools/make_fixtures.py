"""Generates the committed golden fixtures from a test bitstream with the REFERENCE decoder
(oracle/_ref/vtm_capture, built by oracle/ref.mk from /root/reference). Runs only in the build
container. Output: tests/golden/<name>/pic_NNN.xz (+ md5.json with per-POC plane MD5s of the
reference decoder's output, which equal the stream's decoded-picture-hash SEI).

  python tools/make_fixtures.py ra416_q32 [--descriptors-only] [--max-pics N]
"""
import argparse
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import capfile  # noqa: E402

GOLDEN_PLANES = ("pmc", "pfin", "resi", "prelf", "dbkin", "dbk", "sao")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--descriptors-only", action="store_true", help="keep only the final (ALF) planes of I pictures")
    ap.add_argument("--max-pics", type=int, default=0)
    ap.add_argument("--no-planes", action="store_true", help="descriptors and MD5s only (large streams: end-to-end tests)")
    a = ap.parse_args()
    bs = os.path.join(ROOT, "tests", "golden", "streams", a.name + ".bin")
    out = os.path.join(ROOT, "tests", "golden", a.name)
    tmp = tempfile.mkdtemp(prefix="cap_")
    yuv = os.path.join(tmp, "dec.yuv")
    env = dict(os.environ, VVCR_CAPTURE_DIR=tmp)
    r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "vtm_capture"), "-b", bs, "-o", yuv],
                       env=env, capture_output=True, text=True)
    if a.no_planes:
        a.descriptors_only = True
    if r.returncode != 0 or "(OK)" not in r.stdout:
        raise SystemExit("reference decode failed:\n" + r.stdout[-2000:] + r.stderr[-2000:])
    os.makedirs(out, exist_ok=True)
    for f in glob.glob(os.path.join(out, "pic_*.xz")):
        os.remove(f)
    caps = sorted(glob.glob(os.path.join(tmp, "pic_*.cap")))
    md5 = {}
    pics = []
    for i, f in enumerate(caps):
        p = capfile.load(f)
        pics.append(p)
        h = p["hdr"]
        md5[str(h["poc"])] = [hashlib.md5(p["alf_" + c].astype("<u2").tobytes()).hexdigest() for c in "yuv"]
        if a.max_pics and i >= a.max_pics:
            continue
        if a.descriptors_only:
            for k in list(p):
                parts = k.split("_")
                if len(parts) == 2 and parts[0] in GOLDEN_PLANES and parts[1] in ("y", "u", "v"):
                    del p[k]
            if h["slice_type"] != 2 or a.no_planes:   # reference pictures are re-created by the decoder itself
                for c in "yuv":
                    del p["alf_" + c]
        with open(os.path.join(out, "pic_%03d.xz" % i), "wb") as fo:
            fo.write(capfile.pack(p))
    W, H = pics[0]["hdr"]["width"], pics[0]["hdr"]["height"]
    with open(yuv, "rb") as fi:
        ymd5 = hashlib.md5(fi.read()).hexdigest()
    meta = {"stream": a.name, "width": W, "height": H, "pictures": len(caps), "poc_plane_md5": md5,
            "yuv_md5": ymd5, "descriptors_only": a.descriptors_only,
            "generator": "oracle/_ref/vtm_capture (VTM 7.3 DecoderApp, /root/reference) via tools/make_fixtures.py"}
    with open(os.path.join(out, "md5.json"), "w") as fo:
        json.dump(meta, fo, indent=1)
    shutil.rmtree(tmp)
    sz = sum(os.path.getsize(f) for f in glob.glob(os.path.join(out, "*")))
    print("%s: %d pictures, %.2f MB" % (a.name, len(caps), sz / 1e6))


if __name__ == "__main__":
    main()
