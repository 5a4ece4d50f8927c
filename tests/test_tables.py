"""The kernels' generated constant tables equal the reference's own tables (dumped from the running
reference decoder into tests/golden/tables.cap)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_tables as G  # noqa: E402
import oracle_lib as O  # noqa: E402


def test_transform_matrices_match_reference():
    t = O.tables()
    for N in (2, 4, 8, 16, 32, 64):
        assert (G.dct2(N) == t["dct2_%d" % N]).all()
    for N in (4, 8, 16, 32):
        assert (G.dst7(N) == t["dst7_%d" % N]).all()
        assert (G.dct8(N) == t["dct8_%d" % N]).all()


def test_generated_header_is_current():
    hdr = open(os.path.join(ROOT, "vvc_amd", "csrc", "vvcr_gen_tables.h")).read()
    t = O.tables()
    for name in ("lfnst8x8", "lfnst4x4", "lfnst_lut", "mip16x16", "dbk_tc"):
        body = hdr.split(" %s[" % name, 1)[1].split("{", 1)[1].split("}", 1)[0]
        vals = np.array([int(v) for v in body.split(",")])
        assert (vals == t[name].reshape(-1)).all(), name
