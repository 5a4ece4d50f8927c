"""Host-only: the plain-MC job mix of a stream's planned pictures (vvcr_debug_mc_jobs), from its captures.
  python tools/mc_mix.py [--stream ra2160l_q27]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import native as N, stream as S  # noqa: E402

MCJOB = np.dtype([("x", "<i2"), ("y", "<i2"), ("w", "u1"), ("h", "u1"), ("flags", "<u2"), ("mv", "<i2", (2, 2)),
                  ("slot", "u1", (2,)), ("bcw", "i1"), ("ridx", "u1"), ("aux", "<i4"), ("pu_x", "<i2"), ("pu_y", "<i2"),
                  ("pad", "<i4")])


def jobs(pic, which):
    L = N.lib()
    L.vvcr_debug_mc_jobs.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]
    n = L.vvcr_debug_mc_jobs(pic.h, which, None, 0)
    a = np.zeros(n, MCJOB)
    if n:
        L.vvcr_debug_mc_jobs(pic.h, which, a.ctypes.data, n)
    return a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="ra2160l_q27")
    a = ap.parse_args()
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", a.stream))
    alloc = S.SlotAllocator(pics, 16)
    tot = {}
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        if p["hdr"]["slice_type"] == 2:
            continue
        pic = S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16, stages=N.STAGE_INTER)
        row = []
        for which, name in ((0, "tile"), (1, "basic"), (2, "bidir")):
            j = jobs(pic, which)
            bi = ((j["flags"] & 3) == 3).sum()
            px = (j["w"].astype(int) * j["h"]).sum()
            sizes = {}
            for w, h in zip(j["w"], j["h"]):
                sizes[(int(w), int(h))] = sizes.get((int(w), int(h)), 0) + 1
            top = sorted(sizes.items(), key=lambda kv: -kv[1])[:4]
            row.append("%s %d (bi %d, %.1f Mpx) %s" % (name, len(j), bi, px / 1e6, top))
            t = tot.setdefault(name, [0, 0, 0])
            t[0] += len(j); t[1] += bi; t[2] += px
        wc = pic.work_counts()
        print("POC %2d aff %5d | %s" % (p["hdr"]["poc"], wc["affine"], " | ".join(row)))
        pic.close()
    print(tot)


if __name__ == "__main__":
    main()
