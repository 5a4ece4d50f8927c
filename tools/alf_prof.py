"""Diagnostics: per-workgroup phase stamps of k_alf (VVCR_ALF_PROF build) on a stream's pictures.

  python tools/alf_prof.py build               # here: builds vvc_amd/libvvcr_alfprof.so
  python tools/alf_prof.py run [stream]        # GPU box: one ALF launch per picture (all stages prepared),
                                               # prints the phase durations and the dispatch spread
Phases: 0 start, 1 staged (first barrier), 2 classified (second barrier), 3 luma filtered, 4 end.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.path.join(ROOT, "vvc_amd", "libvvcr_alfprof.so")


def build():
    sys.path.insert(0, ROOT)
    from vvc_amd import build as B
    B.build_lib(extra=["-DVVCR_ALF_PROF"], obj_dir=os.path.join(ROOT, "build", "alfprof", "obj"), lib=PROF_LIB)


def run(stream):
    os.environ["VVCR_LIB"] = PROF_LIB
    sys.path.insert(0, ROOT)
    import ctypes as C
    import numpy as np
    from vvc_amd import native as N, stream as S
    L = N.lib()
    L.vvcr_alf_prof_read.argtypes = [C.c_void_p, C.c_int]
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", stream), max_pics=3)
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=8)
    alloc = S.SlotAllocator(pics, 8)
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
        S.submit(ctx, p)
        S.set_loop_filter_params(ctx, p)
        h = ctx.prepare(N.STAGE_ALL)
        buf = np.zeros((1 << 15, 6), np.uint64)
        for rep in range(2):
            ctx.launch(h)
            ctx.sync()
        L.vvcr_alf_prof_read(buf.ctypes.data, buf.shape[0])
        b = buf[buf[:, 4] > 0].astype(np.int64)
        # the last launch's workgroups only: stamps after the previous launch's last end
        b = b[b[:, 0] >= b[:, 0].max() - 5_000_000]
        t0 = b[:, 0].min()
        ph = np.diff(b[:, :5], axis=1) / 100.0
        st = (b[:, 0] - t0) / 100.0
        life = (b[:, 4] - b[:, 0]) / 100.0
        print("POC %d: %d WGs, span %.1f us, start spread %.1f us, WG life median %.2f p90 %.2f us" % (
            p["hdr"]["poc"], len(b), (b[:, 4].max() - t0) / 100.0, st.max(), np.median(life), np.percentile(life, 90)))
        print("   phase medians us (stage, classify, luma, chroma):", [round(float(v), 2) for v in np.median(ph, 0)],
              " p90:", [round(float(v), 2) for v in np.percentile(ph, 90, 0)])
        ctx.release(h)
    ctx.close()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "ra2160l_q27")
