"""Diagnostics: phase timestamps of every k_intra step (VVCR_INTRA_PROF build).

  python tools/intra_prof.py build [-Dxx]     # here: builds build/prof/libvvcr_prof.so (extra defines)
  python tools/intra_prof.py run [stream]    # GPU box: decodes the stream, writes gpurun_out/iprof_<stream>.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.environ.get("VVCR_PROF_LIB") or os.path.join(ROOT, "vvc_amd", "libvvcr_iprof.so")   # vvc_amd/ travels to the GPU box


def build(extra=()):
    sys.path.insert(0, ROOT)
    from vvc_amd import build as B
    B.build_lib(extra=["-DVVCR_INTRA_PROF"] + list(extra), obj_dir=os.path.join(ROOT, "build", "prof", "obj"), lib=PROF_LIB)


def run(stream):
    os.environ["VVCR_LIB"] = PROF_LIB
    sys.path.insert(0, ROOT)
    import ctypes as C
    import numpy as np
    from vvc_amd import native as N, stream as S, decode as D
    L = N.lib()
    L.vvcr_intra_prof_read.argtypes = [C.c_void_p, C.c_int]
    d = os.path.join(ROOT, "tests", "golden", stream)
    pics = S.load_sequence(d)
    npics = int(os.environ.get("INTRA_PROF_PICS", "0"))
    if npics:
        pics = pics[:npics]
    dec = D.Decoder(pics, dpb_slots=12, device=0)
    ctx = dec.ctx
    hs = []
    for i, p in enumerate(pics):
        slot = dec.alloc.assign(i, p["hdr"]["poc"])
        ctx.begin_picture(S.pic_params(p, slot, dec.alloc.slot_of))
        S.submit(ctx, p)
        S.set_loop_filter_params(ctx, p)
        hs.append(ctx.prepare(N.STAGE_ALL))
    buf = np.zeros((1 << 17, 8), np.uint64)
    out = []
    for rep in range(3):
        for i, h in enumerate(hs):
            ctx.launch(h)
            ctx.sync()
            n = L.vvcr_intra_prof_read(buf.ctypes.data, buf.shape[0])
            a = np.concatenate([buf[:n], np.full((n, 1), i, np.uint64), np.full((n, 1), rep, np.uint64)], axis=1)
            out.append(a)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "iprof_%s.npz" % stream), prof=np.concatenate(out))
    print("steps", sum(len(a) for a in out))


def summary(path, pic=0):
    """Critical-path view of one picture's k_intra launch from the npz that run() wrote: span, per-CTU
    durations, per-kind step latencies, and the CTU chain that ends last."""
    import numpy as np
    a = np.load(path)["prof"]
    rep = a[:, 9].max()
    a = a[(a[:, 8] == pic) & (a[:, 9] == rep)]
    t0 = a[:, 0].astype(np.int64); tr = a[:, 1].astype(np.int64); t1 = a[:, 2].astype(np.int64)
    base = t0.min()
    us = lambda v: (v - base) / 100.0
    info = a[:, 5]
    comp = (info & 255).astype(int); w = ((info >> 8) & 255).astype(int); h = ((info >> 16) & 255).astype(int)
    flags = ((info >> 24) & 255).astype(int)
    ctu = (a[:, 7] >> 32).astype(int)
    x = (a[:, 7] & 0xffff).astype(int); y = ((a[:, 7] >> 16) & 0xffff).astype(int)
    wg = (a[:, 6] >> 32).astype(int)
    run = (t1 - tr) / 100.0; wait = (tr - t0) / 100.0
    print("steps %d, span %.1f us, workgroups %d, CTUs %d" % (len(a), us(t1).max(), len(np.unique(wg)), len(np.unique(ctu))))
    print("run us: mean %.2f median %.2f p90 %.2f; wait us: mean %.2f median %.2f" % (run.mean(), np.median(run), np.percentile(run, 90), wait.mean(), np.median(wait)))
    cs = {}
    for c in np.unique(ctu):
        m = ctu == c
        cs[c] = (us(t0[m]).min(), us(t1[m]).max(), m.sum(), run[m].sum())
    d = np.array([v[1] - v[0] for v in cs.values()]); r = np.array([v[3] for v in cs.values()]); n = np.array([v[2] for v in cs.values()])
    print("per CTU: duration mean %.1f median %.1f max %.1f us; steps mean %.1f max %d; sum of run mean %.1f us" % (d.mean(), np.median(d), d.max(), n.mean(), n.max(), r.mean()))
    order = sorted(cs.items(), key=lambda kv: kv[1][0])
    print("CTU start times (first 10 / last 5):", [(int(k), round(v[0], 1), round(v[1] - v[0], 1)) for k, v in order[:10]], [(int(k), round(v[0], 1), round(v[1] - v[0], 1)) for k, v in order[-5:]])
    for nm, m in (("luma", comp == 0), ("chroma", comp > 0)):
        for s_ in (4, 8, 16, 32, 64):
            mm = m & (np.maximum(w, h) == s_)
            if mm.any():
                print("  %-6s max side %2d: %5d steps, run mean %.2f us, median %.2f" % (nm, s_, mm.sum(), run[mm].mean(), np.median(run[mm])))
    ph = np.stack([(a[:, 3] >> (16 * k)) & 0xffff for k in range(4)] + [(a[:, 4] >> (16 * k)) & 0xffff for k in range(4)], 1).astype(float)
    dph = np.diff(np.concatenate([np.zeros((len(a), 1)), ph], 1), axis=1)
    print("phase cycles median (ps1..ps8 deltas):", [int(v) for v in np.median(dph, 0)], "mean:", [int(v) for v in dph.mean(0)])


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    elif sys.argv[1] == "summary":
        summary(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "ra1080_q32")
