"""The C oracle of the RDO inner loop (oracle/oracle_rdo.c SAD / Hadamard SATD, or_fwd_transform in
oracle_resid.c) reproduces the reference's own outputs (tests/golden/rdo, from oracle/capture/rdo_kat.cpp)."""
import ctypes as C

import numpy as np

import oracle_lib
import rdo_golden


def _p(a):
    return C.c_void_p(a.ctypes.data)


def test_oracle_sad_satd_match_reference():
    L = oracle_lib.lib()
    L.or_sad.restype = C.c_uint32
    L.or_satd.restype = C.c_uint32
    blocks = rdo_golden.dist_blocks()
    assert len(blocks) > 100
    for w, h, org, cur, sad, satd in blocks:
        o, c = np.ascontiguousarray(org), np.ascontiguousarray(cur)
        assert L.or_sad(_p(o), w, _p(c), w, w, h) == sad, (w, h)
        assert L.or_satd(_p(o), w, _p(c), w, w, h) == satd, (w, h)


def test_oracle_forward_transform_matches_reference():
    L = oracle_lib.lib()
    blocks = rdo_golden.tr_blocks()
    assert len(blocks) > 100
    for w, h, th, tv, lf, resi, coef in blocks:
        out = np.zeros((h, w), np.int32)
        r = np.ascontiguousarray(resi)
        assert L.or_fwd_transform(_p(r), w, h, th, tv, lf, 10, _p(out)) == 0
        assert np.array_equal(out, coef), (w, h, th, tv, lf)
