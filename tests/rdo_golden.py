"""Readers of the RDO known-answer vectors (tests/golden/rdo, written by the reference's own RdCost /
forward-transform functions through oracle/capture/rdo_kat.cpp; tools/make_rdo_fixtures.sh)."""
import os

import numpy as np

D = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rdo")


def dist_blocks():
    """[(w, h, org[h][w] int16, cur[h][w] int16, sad, satd)]"""
    b = open(os.path.join(D, "dist.bin"), "rb").read()
    n = int(np.frombuffer(b, np.int32, 1, 0)[0])
    off, out = 4, []
    for _ in range(n):
        w, h = (int(v) for v in np.frombuffer(b, np.int32, 2, off))
        off += 8
        org = np.frombuffer(b, np.int16, w * h, off).reshape(h, w)
        off += 2 * w * h
        cur = np.frombuffer(b, np.int16, w * h, off).reshape(h, w)
        off += 2 * w * h
        sad, satd = (int(v) for v in np.frombuffer(b, np.uint32, 2, off))
        off += 8
        out.append((w, h, org, cur, sad, satd))
    return out


def tr_blocks():
    """[(w, h, trh, trv, lfnst, resi[h][w] int16, coef[h][w] int32)]; tr types 0 DCT2, 1 DST7, 2 DCT8"""
    b = open(os.path.join(D, "tr.bin"), "rb").read()
    n = int(np.frombuffer(b, np.int32, 1, 0)[0])
    off, out = 4, []
    for _ in range(n):
        w, h, th, tv, lf = (int(v) for v in np.frombuffer(b, np.int32, 5, off))
        off += 20
        resi = np.frombuffer(b, np.int16, w * h, off).reshape(h, w)
        off += 2 * w * h
        coef = np.frombuffer(b, np.int32, w * h, off).reshape(h, w)
        off += 4 * w * h
        out.append((w, h, th, tv, lf, resi, coef))
    return out
