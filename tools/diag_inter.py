"""Diagnostics (GPU box): one inter picture reconstructed from its capture with the reference's own
reference pictures in the DPB; the prediction, residual and pre-loop-filter planes are compared with the
reference's, and the CUs holding mismatching samples are listed with their coding tools.
Usage: python tools/diag_inter.py STREAM PICTURE_INDEX"""
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import capfile  # noqa: E402
from vvc_amd import native as N  # noqa: E402
from vvc_amd import stream as S  # noqa: E402

CU, PU = capfile.CU, capfile.PU


def main():
    name, idx = sys.argv[1], int(sys.argv[2])
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", name), max_pics=idx + 1)
    by_poc = {p["hdr"]["poc"]: p for p in pics}
    p = pics[idx]
    h = p["hdr"]
    ctx = N.Context(h["width"], h["height"], dpb_slots=20)
    slot_of = {}
    for l in range(2):
        for r in range(h["num_ref_l%d" % l]):
            poc = int(p["ref_poc"][l][r])
            if poc not in slot_of:
                slot_of[poc] = len(slot_of) + 1
                for c, pl in enumerate("yuv"):
                    ctx.write_plane(N.BUF_RECO, slot_of[poc], c, by_poc[poc]["alf_" + pl])
    ctx.begin_picture(S.pic_params(p, 0, slot_of))
    S.submit(ctx, p)
    ctx.end_picture(N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA)
    cu, pu = p["cu"], p["pu"]
    for c, pl in enumerate("yuv"):
        got = ctx.read_plane(N.BUF_RECO, 0, c)
        exp = p["prelf_" + pl]
        res = ctx.read_plane(N.BUF_RESI, 0, c)
        bad = got != exp
        print("%s: recon differs at %d samples; residual differs at %d" % (pl, int(bad.sum()), int((res != p["resi_" + pl]).sum())))
        if not bad.any():
            continue
        sx = 0 if c == 0 else 1
        cus = Counter()
        for y, x in np.argwhere(bad):
            X, Y = x << sx, y << sx
            k = np.where((cu[:, CU["x"]] <= X) & (X < cu[:, CU["x"]] + cu[:, CU["w"]]) & (cu[:, CU["y"]] <= Y) &
                         (Y < cu[:, CU["y"]] + cu[:, CU["h"]]) & (cu[:, CU["chtype"]] == 0))[0]
            cus[int(k[0]) if len(k) else -1] += 1
        for k, n in cus.most_common(8):
            if k < 0:
                print("   (no CU)", n)
                continue
            r = cu[k]
            u = pu[r[CU["firstpu"]]]
            print("   cu %d at (%d,%d) %dx%d: %d samples; predmode %d skip %d geo %d affine %d ciip %d mmvd %d interdir %d "
                  "bdof %d dmvr %d imv %d bcw %d mts %d lfnst %d sbt %d" % (
                      k, r[CU["x"]], r[CU["y"]], r[CU["w"]], r[CU["h"]], n, r[CU["predmode"]], r[CU["skip"]], r[CU["geo"]],
                      r[CU["affine"]], u[PU["ciip"]], u[PU["mmvd"]], u[PU["interdir"]], u[PU["bdof"]], u[PU["dmvr"]],
                      r[CU["imv"]], r[CU["bcw"]], r[CU["mtsflag"]], r[CU["lfnst"]], r[CU["sbtinfo"]]))
            if r[CU["geo"]]:
                print("      geodir %d idx %d %d" % (u[PU["geodir"]], u[PU["geoi0"]], u[PU["geoi1"]]))
        y, x = np.argwhere(bad)[0]
        print("   first (%d,%d): got %s exp %s" % (x, y, got[y, x:x + 8].tolist(), exp[y, x:x + 8].tolist()))
    ctx.close()


if __name__ == "__main__":
    main()
