"""Diagnostics: per-workgroup start / end timestamps of k_mc (VVCR_MC_PROF build) on a stream's B pictures.

  python tools/mc_prof.py build               # here: builds vvc_amd/libvvcr_mcprof.so
  python tools/mc_prof.py run [stream]        # GPU box: one k_mc launch per B picture, prints the duration
                                              # distribution and the slowest workgroups' first jobs
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.path.join(ROOT, "vvc_amd", "libvvcr_mcprof.so")   # vvc_amd/ travels to the GPU box, build/ does not


def build():
    sys.path.insert(0, ROOT)
    from vvc_amd import build as B
    B.build_lib(extra=["-DVVCR_MC_PROF"], obj_dir=os.path.join(ROOT, "build", "mcprof", "obj"), lib=PROF_LIB)


def run(stream):
    os.environ["VVCR_LIB"] = PROF_LIB
    sys.path.insert(0, ROOT)
    import ctypes as C
    import numpy as np
    from vvc_amd import native as N, stream as S
    L = N.lib()
    L.vvcr_mc_prof_read.argtypes = [C.c_void_p, C.c_int]
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", stream))
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=16)
    alloc = S.SlotAllocator(pics, 16)
    prev_end = 0
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        if p["hdr"]["slice_type"] == 2:
            continue
        ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
        S.submit(ctx, p)
        h = ctx.prepare(N.STAGE_INTER)
        buf = np.zeros((1 << 16, 4), np.uint64)
        for rep in range(3):
            ctx.launch(h)
            ctx.sync()
            if rep < 2:   # only the last launch's stamps count: start after the previous ones
                L.vvcr_mc_prof_read(buf.ctypes.data, buf.shape[0])
                m = buf[:, 1].max()
                prev_end = max(prev_end, int(m))
        L.vvcr_mc_prof_read(buf.ctypes.data, buf.shape[0])
        valid = buf[:, 1] > prev_end   # entries of this picture's last launch (older ones are stale)
        b = buf[valid]
        if len(b) == 0:
            print("POC %d: no plain-MC launch" % p["hdr"]["poc"])
            ctx.release(h)
            continue
        prev_end = int(b[:, 1].max())
        t0 = b[:, 0].astype(np.int64)
        t1 = b[:, 1].astype(np.int64)
        base = t0.min()
        dur = (t1 - t0) / 100.0   # us (100 MHz)
        start = (t0 - base) / 100.0
        end = (t1 - base) / 100.0
        hw = (b[:, 2] & 0xffffffff).astype(np.int64)
        xcc = ((b[:, 2] >> 32) & 0xf).astype(np.int64)
        cu = ((hw >> 8) & 15) | (((hw >> 13) & 7) << 4) | (((hw >> 12) & 1) << 7)
        cu_g = xcc * 256 + cu
        span = end.max()
        ncu = len(np.unique(cu_g))
        conc = dur.sum() / (span * ncu)
        per_cu = np.bincount(np.unique(cu_g, return_inverse=True)[1])
        print("POC %d: %d waves on %d CUs (%.1f per CU, max %d), span %.1f us, start spread %.1f us, wave duration median %.2f p10 %.2f p90 %.2f max %.2f us, mean live waves per CU %.1f" % (
            p["hdr"]["poc"], len(b), ncu, per_cu.mean(), per_cu.max(), span, start.max(), np.median(dur), np.percentile(dur, 10),
            np.percentile(dur, 90), dur.max(), conc))
        tag = b[:, 3].astype(np.uint64)
        lum = (tag >> np.uint64(63)).astype(np.int64)
        cw = ((tag >> np.uint64(8)) & np.uint64(255)).astype(np.int64)
        chh = (tag & np.uint64(255)).astype(np.int64)
        nbi = ((tag >> np.uint64(16)) & np.uint64(255)).astype(np.int64)
        nrec = ((tag >> np.uint64(24)) & np.uint64(255)).astype(np.int64)
        nwp = ((tag >> np.uint64(32)) & np.uint64(255)).astype(np.int64)
        nact = ((tag >> np.uint64(40)) & np.uint64(255)).astype(np.int64)
        for k in np.argsort(-dur)[:6]:
            print("   slow wave: start %.1f dur %.1f  %s %dx%d active %d bi %d recon %d wp/geo %d  cu %d" % (
                start[k], dur[k], "luma" if lum[k] else "chroma", cw[k], chh[k], nact[k], nbi[k], nrec[k], nwp[k], cu_g[k]))
        for isl in (1, 0):
            m = lum == isl
            if m.any():
                print("   %s waves %d: duration median %.2f p90 %.2f; bi-full waves median %.2f, uni-full %.2f" % (
                    "luma" if isl else "chroma", m.sum(), np.median(dur[m]), np.percentile(dur[m], 90),
                    np.median(dur[m & (nbi == 64)]) if (m & (nbi == 64)).any() else -1,
                    np.median(dur[m & (nbi == 0) & (nact == 64)]) if (m & (nbi == 0) & (nact == 64)).any() else -1))
        cls = {}
        for k in range(len(b)):
            key = ("L" if lum[k] else "C") + "%dx%d" % (cw[k], chh[k])
            c = cls.setdefault(key, [0, 0.0, 0])
            c[0] += 1
            c[1] += dur[k]
            c[2] += nact[k]
        tot = dur.sum()
        print("   wave-time by class (waves, share of wave-us, median us, active lanes/wave):",
              ", ".join("%s %d %.0f%% %.1f %.0f" % (key, c[0], 100 * c[1] / tot, c[1] / c[0], c[2] / c[0])
                        for key, c in sorted(cls.items(), key=lambda kv: -kv[1][1])))
        hist = np.histogram(start, bins=8, range=(0, span))[0]
        print("   wave starts per eighth of the span:", list(hist))
        ctx.release(h)
    ctx.close()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "ra2160_q32")
