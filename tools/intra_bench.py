"""k_intra in isolation on the GPU box: the stream's intra picture reconstructed --reps times (residual +
intra + loop filters, one picture at a time), the HIP-event time of the intra kernel averaged.
VVCR_LIB selects a library variant (tools/intra_variants.sh). Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (HIP runtime before libvvcr creates contexts)
from vvc_amd import native as N, stream as S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="ra1080_q32")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", a.stream))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=4)
    alloc = S.SlotAllocator(pics[:1], 4)
    p = pics[0]
    slot = alloc.assign(0, p["hdr"]["poc"])
    ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
    S.submit(ctx, p)
    S.set_loop_filter_params(ctx, p)
    h = ctx.prepare(N.STAGE_ALL)
    ctx.set_timing(True)
    ms = []
    for r in range(a.reps + 2):
        ctx.launch(h)
        ctx.sync()
        for name, n, t, alg, _ in ctx.kernel_stats(h):
            if name == "intra" and r >= 2:
                ms.append(t)
    ms.sort()
    out = {"lib": os.path.basename(os.environ.get("VVCR_LIB", "libvvcr.so")) + (" " + os.environ["AB_LABEL"] if os.environ.get("AB_LABEL") else ""),
           "stream": a.stream,
           "intra_ms_median": round(ms[len(ms) // 2], 4), "intra_ms_min": round(ms[0], 4), "reps": len(ms)}
    ctx.release(h)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
