"""MC kernels in isolation: the inter stage (VVCR_STAGE_INTER: k_mc, k_mc_bidir, k_mc_affine) of
every B picture of a stream, prepared once and launched --reps times back to back; per-kernel HIP-event
times and algorithmic bytes (vvcr_kernel_stats) of the last repetition, and the wall time per picture.
Reference content is irrelevant for timing (the DPB holds whatever the slots contain).
  python tools/mc_bench.py [--stream ra2160_q32] [--reps 50]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import native as N, stream as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="ra2160_q32")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--all-stages", action="store_true", help="prepare and launch every stage (the fused reconstruction path of k_mc)")
    a = ap.parse_args()
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", a.stream))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=16)
    alloc = S.SlotAllocator(pics, 16)
    hs = []
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        if p["hdr"]["slice_type"] == 2:
            continue
        ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
        S.submit(ctx, p)
        if a.all_stages:
            S.set_loop_filter_params(ctx, p)
        hs.append(ctx.prepare(N.STAGE_ALL if a.all_stages else N.STAGE_INTER))
    ctx.set_timing(False)
    for h in hs:
        ctx.launch(h)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        for h in hs:
            ctx.launch(h)
            ctx.sync()
    t1 = time.perf_counter()
    ctx.set_timing(True)
    out = {"stream": a.stream, "pictures": len(hs), "ms_per_picture_wall": round((t1 - t0) / a.reps / len(hs) * 1e3, 4)}
    agg = {}
    per_pic = []
    for h in hs:
        ctx.launch(h)
        ctx.sync()
        row = {}
        for name, n, ms, alg, _ in ctx.kernel_stats(h):
            if n:
                g = agg.setdefault(name, [0, 0.0, 0.0])
                g[0] += n; g[1] += ms; g[2] += alg
                row[name] = [round(ms * 1e3, 1), round(alg / 1e6, 1), round(alg / (ms / 1e3) / 1e9) if ms else 0]
        per_pic.append(row)
    out["per_picture_us_MB_GBps"] = per_pic
    out["kernels"] = {k: {"launches": v[0], "us_per_launch": round(v[1] / v[0] * 1e3, 2), "alg_MB_per_launch": round(v[2] / v[0] / 1e6, 3),
                          "alg_GBps": round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] else 0} for k, v in agg.items()}
    for h in hs:
        ctx.release(h)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
