"""Critical path of k_intra on one picture: the profile of tools/intra_prof.py (gpurun_out/iprof_<stream>.npz,
per step take / ready / done stamps) joined with the step dependencies of the host plan
(vvcr_debug_plan_intra, run here on the CPU). Walks back from the last step to finish, each time to the
dependency that finished last, and splits the path into step bodies (ready -> done) and hand-offs
(dependency done -> ready).   python tools/iprof_path.py [stream]"""
import ctypes as C
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import native as N, stream as S  # noqa: E402


def plan(p):
    L = N.lib()
    h = p["hdr"]
    sp = N.SeqParams(h["width"], h["height"], 1, 10, 7, 4, 0)
    pp = S.pic_params(p, 0, {}, missing_ref_slot=0)
    arrs = [np.ascontiguousarray(p[k], np.int32) for k in ("cu", "pu", "tu")]
    cap, dcap = 1 << 18, 1 << 21
    out = np.zeros(8 * cap, np.int32)
    ds = np.zeros(cap + 1, np.int32)
    dd = np.zeros(dcap, np.int32)
    cnt = np.zeros(2, np.int32)
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    f = L.vvcr_debug_plan_intra
    f.restype = C.c_int
    n = f(C.byref(sp), C.byref(pp), P(arrs[0]), len(arrs[0]), P(arrs[1]), len(arrs[1]), P(arrs[2]), len(arrs[2]),
          P(out), cap, P(ds), P(dd), dcap, P(cnt))
    assert n > 0, n
    return out[:8 * n].reshape(n, 8), ds[:n + 1], dd[:cnt[1]]


def main(stream="ra1080_q32"):
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", stream), max_pics=1)
    steps, ds, dd = plan(pics[0])
    n = len(steps)
    # CTU of each step (luma 128, chroma 64 sample CTUs) and the CTU's first step (local deps are relative)
    cx = np.where(steps[:, 2] == 0, steps[:, 0] >> 7, steps[:, 0] >> 6)
    cy = np.where(steps[:, 2] == 0, steps[:, 1] >> 7, steps[:, 1] >> 6)
    ctu = cy * 10000 + cx
    first = np.zeros(n, np.int64)
    for i in range(1, n):
        first[i] = first[i - 1] if ctu[i] == ctu[i - 1] else i
    a = np.load(os.path.join(ROOT, "gpurun_out", "iprof_%s.npz" % stream))["prof"]
    a = a[(a[:, 9] == a[:, 9].max()) & (a[:, 8] == 0)]
    gj = (a[:, 6] & np.uint64(0xffffffff)).astype(np.int64)
    t0 = np.full(n, -1, np.int64); t1 = t0.copy(); t2 = t0.copy()
    t0[gj], t1[gj], t2[gj] = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64), a[:, 2].astype(np.int64)
    assert (t2 >= 0).all(), "profile does not cover every step"
    info = a[:, 5]
    flags = np.zeros(n, np.int64); flags[gj] = ((info >> np.uint64(24)) & np.uint64(0xff)).astype(np.int64)
    mode = np.zeros(n, np.int64); mode[gj] = ((info >> np.uint64(32)) & np.uint64(0xff)).astype(np.int64)
    s = int(np.argmax(t2))
    path = []
    while True:
        deps = []
        for k in range(ds[s], ds[s + 1]):
            v = int(dd[k])
            deps.append(first[s] + v if v >= 0 else ~v)
        if not deps:
            path.append((s, None)); break
        d = max(deps, key=lambda q: t2[q])
        path.append((s, d))
        s = d
    path.reverse()
    us = 0.01
    body = sum((t2[s] - t1[s]) for s, _ in path) * us
    hand = sum((t1[s] - t2[d]) for s, d in path if d is not None) * us
    late = sum(max(0, t0[s] - t2[d]) for s, d in path if d is not None) * us
    span = (t2.max() - t0.min()) * us
    print("steps %d, span %.0f us; critical path %d steps: bodies %.0f us, hand-offs %.0f us (of which taken after the "
          "dependency finished: %.0f us)" % (n, span, len(path), body, hand, late))
    kinds = Counter()
    tk = Counter()
    for s, d in path:
        f = flags[s]
        k = "ISP" if f & 0x30 else "MIP" if f & 1 else "BDPCM" if f & 4 else "CIIP" if f & 8 else \
            ("chroma" if steps[s, 2] else "luma")
        kinds[k] += 1
        tk[k] += (t2[s] - t1[s]) * us
    for k in kinds:
        print("  %-7s %4d steps  body %.0f us  (%.2f us/step)" % (k, kinds[k], tk[k], tk[k] / kinds[k]))
    cross = sum(1 for s, d in path if d is not None and first[s] != first[d])
    hx = [(t1[s] - t2[d]) * us for s, d in path if d is not None and first[s] != first[d]]
    hl = [(t1[s] - t2[d]) * us for s, d in path if d is not None and first[s] == first[d]]
    print("  hand-offs: %d within a CTU (median %.2f us), %d across CTUs (median %.2f us)" %
          (len(hl), np.median(hl) if hl else 0, cross, np.median(hx) if hx else 0))


if __name__ == "__main__":
    main(*sys.argv[1:2])


def late_takes(stream="ra1080_q32", show=8):
    """For the critical steps taken after their critical dependency finished: what the CTU's waves were
    doing in between (the steps taken just before, their wait and whether they wait on another CTU)."""
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", stream), max_pics=1)
    steps, ds, dd = plan(pics[0])
    return steps, ds, dd
