"""Test helpers: region masks per coding tool, so each kernel is checked exactly on the samples it owns."""
import numpy as np

from vvc_amd import capfile as cf

CU, PU = cf.CU, cf.PU


def cu_mask(pic, pred, comp=0):
    """Boolean plane mask of the CUs for which pred(cu, pus) is True."""
    h = pic["hdr"]
    W, H = (h["width"], h["height"]) if comp == 0 else (h["width"] // 2, h["height"] // 2)
    m = np.zeros((H, W), bool)
    cus, pus = pic["cu"], pic["pu"]
    for c in cus:
        if not c[CU["yvalid"]]:
            continue
        p = pus[c[CU["firstpu"]]: c[CU["firstpu"]] + c[CU["npu"]]]
        if pred(c, p):
            s = 0 if comp == 0 else 1
            x, y, w, hh = c[CU["x"]] >> s, c[CU["y"]] >> s, c[CU["w"]] >> s, c[CU["h"]] >> s
            m[y:y + hh, x:x + w] = True
    return m


def is_basic_mc(c, pus):
    """CUs reconstructed by the basic MC kernel (see vvcr_host.cpp build_work_lists)."""
    if c[CU["predmode"]] != 0 or c[CU["geo"]] or c[CU["affine"]]:
        return False
    for p in pus:
        if p[PU["mrgtype"]] == 1:
            continue
        if p[PU["dmvr"]] or p[PU["bdof"]]:
            return False
    return True


def is_inter(c, pus):
    return c[CU["predmode"]] == 0
