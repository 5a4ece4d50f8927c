"""Host-side cost of the decode path on the CPU, no GPU: per picture of a committed stream, the CABAC
pass (vvcp_parse_picture), motion derivation (vvcp_derive_motion, refined with the captured DMVR
deltas when the golden directory holds them) and native planning (vvcp_plan_picture), single thread.

  python tools/host_prof.py ra2160_q27 [repeats]
"""
import ctypes as C
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import bitstream as B  # noqa: E402
from vvc_amd import capfile  # noqa: E402
from vvc_amd import native as N  # noqa: E402
from vvc_amd import parser  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ra2160_q27"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    data = open(os.path.join(ROOT, "tests", "golden", "streams", name + ".bin"), "rb").read()
    caps = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", name, "pic_*.xz")))
    deltas = [capfile.unpack(open(f, "rb").read())["dmvr_delta"] for f in caps]
    L = B._bind(N.lib())
    tot = {}
    for _ in range(reps):
        s = parser.Stream(data)
        plan = B.Plan(s, 16)
        inf = plan.info[0]
        sp = N.SeqParams(inf["width"], inf["height"], 1, inf["bit_depth"], inf["ctu_log2"], 16, 0)
        for i in range(len(s)):
            t0 = time.perf_counter()
            s.parse(i)
            t1 = time.perf_counter()
            s.derive(i)
            s.refine(i, deltas[i] if i < len(deltas) else None)
            t2 = time.perf_counter()
            h = C.c_void_p()
            rc = L.vvcp_plan_picture(s.h, i, C.byref(sp), plan.slot[i], plan.ref_slots(i).ctypes.data, N.STAGE_ALL, C.byref(h))
            assert rc == 0, L.vvcp_last_error().decode()
            t3 = time.perf_counter()
            N.Picture.wrap(h).close()
            kind = "I" if plan.info[i]["slice_type"] == 2 else "B"
            r = tot.setdefault(kind, [0, 0.0, 0.0, 0.0])
            r[0] += 1
            r[1] += t1 - t0
            r[2] += t2 - t1
            r[3] += t3 - t2
        s.close()
    for k, (n, a, b, c) in sorted(tot.items()):
        print("%s x%d  parse %.2f ms  derive %.2f ms  plan %.2f ms  (per picture)" % (k, n, a / n * 1e3, b / n * 1e3, c / n * 1e3))


if __name__ == "__main__":
    main()
