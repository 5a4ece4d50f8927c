"""Diagnostics (GPU box): pre-loop-filter reconstruction of one picture vs the reference plane, with
the mismatching 4x4 units listed (position, component) — for bisecting a kernel change."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import native as N  # noqa: E402
from vvc_amd import stream as S  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "ai416_q37"
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 0
pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", name))
by_poc = {p["hdr"]["poc"]: p for p in pics}
p = pics[idx]
h0 = p["hdr"]
ctx = N.Context(h0["width"], h0["height"], dpb_slots=20)
slot_of = {}
for l in range(2):
    for r in range(p["hdr"]["num_ref_l%d" % l]):
        poc = int(p["ref_poc"][l][r])
        if poc not in slot_of:
            slot_of[poc] = len(slot_of) + 1
            for c, pl in enumerate("yuv"):
                ctx.write_plane(N.BUF_RECO, slot_of[poc], c, by_poc[poc]["alf_" + pl])
ctx.begin_picture(S.pic_params(p, 0, slot_of))
S.submit(ctx, p)
ctx.end_picture(N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA)
for c, pl in enumerate("yuv"):
    got = ctx.read_plane(N.BUF_RECO, 0, c)
    exp = p["prelf_" + pl]
    bad = got != exp
    u = 4 if c == 0 else 2
    units = sorted({(y // u * u, x // u * u) for y, x in np.argwhere(bad)})
    print(pl, "differ", int(bad.sum()), "units", len(units), "first", units[:12])
    if units:
        y, x = units[0]
        print(" got", got[y:y + u, x:x + u].tolist(), "exp", exp[y:y + u, x:x + u].tolist())
ctx.close()
if len(sys.argv) > 3:
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=20)
    ctx.begin_picture(S.pic_params(p, 0, slot_of))
    S.submit(ctx, p)
    ctx.end_picture(N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA)
    got = ctx.read_plane(N.BUF_RECO, 0, 0)
    res = ctx.read_plane(N.BUF_RESI, 0, 0)
    exp = p["prelf_y"]
    print("resi ok", bool((res == p["resi_y"]).all()))
    bad = (got != exp)[:64, :64]
    print("block0 bad", int(bad.sum()))
    for r in range(16):
        print("".join("X" if b else "." for b in bad[r, :64]))
    print("got-512", (got[:4, :8].astype(int) - 512).tolist())
    print("res", res[:4, :8].tolist())
    print("exp-512", (exp[:4, :8].astype(int) - 512).tolist())
if os.environ.get("VVCR_DIAG_DUMP"):
    import ctypes as C
    L = N.lib()
    buf = np.zeros(1024, np.int32)
    L.vvcr_diag_dump(buf.ctypes.data_as(C.c_void_p))
    print("top", buf[:16].tolist()); print("left", buf[16:32].tolist()); print("topF", buf[32:48].tolist())
    print("av/mode/refFilter/predMode/pdpc/flags/lens", buf[48:58].tolist()); print("pred", buf[64:128].tolist())
    print("refU0", buf[256:416].tolist()); print("refF0", buf[512:672].tolist()); print("refF1", buf[768:928].tolist())
