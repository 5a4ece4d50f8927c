"""Golden MD5s of DecoderApp's output file (-o) at several output bit depths, for the output-writer tests
(tests/test_output.py, tests/test_output_gpu.py): runs the reference DecoderApp built by oracle/ref.mk
(oracle/_ref/DecoderApp, this container only) on tests/golden/streams/<stream>.bin and writes
tests/golden/<stream>/output_md5.json = {"d<bits>[_709]": md5 of the whole file}.

  python tools/make_output_fixtures.py ra416_q32 ai416_q37 ...
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEC = os.path.join(ROOT, "oracle", "_ref", "DecoderApp")
CASES = [("d10", []), ("d8", ["-d", "8"]), ("d12", ["-d", "12"]), ("d8_709", ["-d", "8", "--ClipOutputVideoToRec709Range=1"])]


def main(streams):
    for s in streams:
        bs = os.path.join(ROOT, "tests", "golden", "streams", s + ".bin")
        out = {}
        with tempfile.TemporaryDirectory() as td:
            for name, args in CASES:
                yuv = os.path.join(td, name + ".yuv")
                subprocess.run([DEC, "-b", bs, "-o", yuv] + args, check=True, capture_output=True)
                with open(yuv, "rb") as f:
                    out[name] = hashlib.md5(f.read()).hexdigest()
        with open(os.path.join(ROOT, "tests", "golden", s, "output_md5.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(s, out)


if __name__ == "__main__":
    main(sys.argv[1:])
