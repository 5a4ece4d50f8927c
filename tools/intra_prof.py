"""Diagnostics: phase timestamps of every k_intra step (VVCR_INTRA_PROF build).

  python tools/intra_prof.py build [-Dxx]     # here: builds build/prof/libvvcr_prof.so (extra defines)
  python tools/intra_prof.py run [stream]    # GPU box: decodes the stream, writes gpurun_out/iprof_<stream>.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.environ.get("VVCR_PROF_LIB") or os.path.join(ROOT, "build", "prof", "libvvcr_prof.so")


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


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "ra1080_q32")
