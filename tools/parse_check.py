"""Compares the host parser's rows with the capture fixtures of a golden stream (development aid;
tests/test_parser.py is the test). Usage: python tools/parse_check.py STREAM [--lib PATH] [--pics N]"""
import argparse
import ctypes as C
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vvc_amd import capfile, parser  # noqa: E402

CU_F = "x y w h cx cy cw ch chtype predmode qp treetype modetype skip mmvdskip affine affinetype geo bdpcm bdpcmc imv rootcbf sbtinfo mtsflag lfnst bcw mip isp smvd act cqpadj depth qtdepth firstpu npu firsttu ntu slice yvalid cvalid".split()
PU_F = ("cu x y w h cx cy cw ch chtype idir_l idir_c fidir_l fidir_c mipt mrl merge regmerge mergeidx geodir geoi0 geoi1 mmvd interdir "
        "mv0x mv0y mv1x mv1y ref0 ref1 mrgtype mvrefine ciip").split() + ["aff%d" % i for i in range(12)] + ["dmvr_off", "bdof", "dmvr"]
TU_F = "cu chtype depth noresi jccr cadj".split() + ["%s%d" % (f, c) for c in range(3) for f in "x y w h cbf mts coff qp qpts".split()]


def first_diff(name, a, b, fields, mask=()):
    if a.shape != b.shape:
        return "%s: shape %s vs capture %s" % (name, a.shape, b.shape)
    cols = [i for i, f in enumerate(fields) if f not in mask]
    d = np.argwhere(a[:, cols] != b[:, cols])
    if len(d) == 0:
        return None
    r, c = d[0]
    return "%s row %d field %s: %d vs capture %d (%d diffs)\n  ours %s\n  cap  %s" % (
        name, r, fields[cols[c]], a[r, cols[c]], b[r, cols[c]], len(d), a[r].tolist(), b[r].tolist())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stream")
    ap.add_argument("--lib")
    ap.add_argument("--pics", type=int, default=0)
    ap.add_argument("--no-mv", action="store_true", help="skip motion derivation (syntax fields only)")
    args = ap.parse_args()
    lib = C.CDLL(args.lib) if args.lib else None
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
    data = open(os.path.join(root, "streams", args.stream + ".bin"), "rb").read()
    s = parser.Stream(data, lib=lib)
    caps = sorted(glob.glob(os.path.join(root, args.stream, "pic_*.xz")))
    print("pictures", len(s), "captures", len(caps))
    n = len(caps) if not args.pics else min(args.pics, len(caps))
    ok = True
    for i in range(n):
        cap = capfile.unpack(open(caps[i], "rb").read())
        info = s.info(i)
        err = None
        try:
            s.parse(i)
        except parser.ParseError as e:
            err = str(e)
        r = s.rows(i)
        if err:
            nc = min(len(r["cu"]), len(cap["cu"]))
            bad = [k for k in range(nc) if not np.array_equal(r["cu"][k][:31], cap["cu"][k][:31])]
            print("pic %d: %s; parsed %d CUs (capture %d); first differing CU %s" % (i, err, len(r["cu"]), len(cap["cu"]), bad[:1]))
            k = bad[0] if bad else nc
            for j in range(max(0, k - 2), min(nc, k + 1)):
                print("   cu", j, "ours", r["cu"][j].tolist())
                print("   cu", j, "cap ", cap["cu"][j].tolist())
                pj, pc = r["pu"][j], cap["pu"][j]
                print("   pu", j, "ours", pj.tolist())
                print("   pu", j, "cap ", pc.tolist())
            ok = False
            break
        msgs = []
        mvmask = set()
        pumask = set()
        if args.no_mv and info["slice_type"] != 2:
            mvmask = {"imv", "bcw", "affinetype"}
            pumask = {"interdir", "mv0x", "mv0y", "mv1x", "mv1y", "ref0", "ref1", "mrgtype", "mvrefine", "mergeidx", "dmvr_off", "bdof", "dmvr"} | {"aff%d" % k for k in range(12)}
        else:
            try:
                s.derive(i)
                s.refine(i, cap["dmvr_delta"])
            except parser.ParseError as e:
                msgs.append(str(e))
            r = s.rows(i)
            if "motion" in r:
                mo, mc = r["motion"], cap["motion"]
                if mo.shape != mc.shape:
                    msgs.append("motion shape %s vs %s" % (mo.shape, mc.shape))
                else:
                    d = np.argwhere(mo != mc)
                    if len(d):
                        y, x, f = d[0]
                        msgs.append("motion (%d,%d) field %d: ours %s cap %s (%d diffs)" % (x * 4, y * 4, f, mo[y, x].tolist(), mc[y, x].tolist(), len(d)))
                cg = cap["geo"][np.argsort(cap["geo"][:, 0], kind="stable")] if len(cap["geo"]) else cap["geo"]
                if not np.array_equal(r["geo"], cg):
                    g = r["geo"]
                    msgs.append("geo differs: %d vs %d rows; first ours %s cap %s" % (len(g), len(cg), g[:1].tolist(), cg[:1].tolist()))
        m = first_diff("cu", r["cu"], cap["cu"], CU_F, mvmask)
        if m: msgs.append(m)
        m = first_diff("pu", r["pu"], cap["pu"], PU_F, pumask)
        if m: msgs.append(m)
        m = first_diff("tu", r["tu"], cap["tu"], TU_F, {"cadj"})
        if m: msgs.append(m)
        if r["coef"].shape != cap["coef"].shape or not np.array_equal(r["coef"], cap["coef"]):
            msgs.append("coef: %s vs %s" % (r["coef"].shape, cap["coef"].shape))
        sa, sb = r["sao"], cap["sao"]
        on = sb[:, :, 0] != 0
        if not (np.array_equal(sa[:, :, 0], sb[:, :, 0]) and np.array_equal(sa[on], sb[on])):
            msgs.append("sao differs")
        for k in ("alf_ctb_en", "alf_ctb_alt", "alf_ctb_fidx"):
            if k in cap and not np.array_equal(r[k], cap[k]):
                msgs.append("%s differs" % k)
        for c, key in enumerate(("ccalf_en_cb", "ccalf_en_cr")):   # the capture's array is stale when CC-ALF is off
            if cap["hdr"].get(key) and not np.array_equal(r["ccalf_ctl"][c], cap["ccalf_ctl"][c]):
                msgs.append("ccalf_ctl[%d] differs" % c)
        print("pic %d poc %d type %d: cu %d pu %d tu %d coef %d %s" % (i, info["poc"], info["slice_type"], len(r["cu"]), len(r["pu"]),
              len(r["tu"]), len(r["coef"]), "OK" if not msgs else "MISMATCH"))
        for m in msgs:
            print("   ", m)
        ok &= not msgs
    print("ALL OK" if ok else "FAILED")


if __name__ == "__main__":
    main()
