"""Summarise gpurun_out/iprof_<stream>.npz (tools/intra_prof.py).

Record per step: [0..2] s_memrealtime (100 MHz) at take / dependencies met / done, [3],[4] eight 16-bit
phase stamps, [5] comp,w,h,flags,mode,xcc, [6] step | block << 32,
[7] number of dependencies, [8] picture, [9] repetition."""
import sys
import numpy as np
a = np.load(sys.argv[1])['prof']
a = a[a[:, 9] == a[:, 9].max()]
info = a[:, 5]
comp = info & 0xff; w = (info >> 8) & 0xff; h = (info >> 16) & 0xff; flags = (info >> 24) & 0xff; mode = (info >> 32) & 0xff
m16 = np.uint64(0xffff)
st = np.stack([(a[:, 3 + q // 4] >> np.uint64(16 * (q % 4))) & m16 for q in range(8)], 1).astype(np.int64)
print("stamps (cycles from start, 16-bit): job, resid, fill-loads, fill, refs, params, predict, end")
print("  mean", st.mean(0).round(0), " median", np.median(st, 0))
ph = st[:, [4, 5, 6, 7]]
d = np.diff(np.concatenate([np.zeros((len(a), 1), np.int64), ph], 1), axis=1)
t0, t1, t2 = (a[:, k].astype(np.int64) for k in range(3))
print("steps", len(a), "phase cycles [refs, params, predict, recon]", d.mean(0).round(0), "total", ph[:, 3].mean().round(0))
print("wait (us) mean %.2f  run (us) mean %.2f  median run %.2f" % (((t1 - t0) * 0.01).mean(), ((t2 - t1) * 0.01).mean(), np.median((t2 - t1) * 0.01)))
for pic in np.unique(a[:, 8]):
    m = a[:, 8] == pic
    span = (t2[m].max() - t0[m].min()) * 0.01
    print("picture %d: %d steps, span %.1f us, mean run %.2f us" % (pic, m.sum(), span, ((t2[m] - t1[m]) * 0.01).mean()))
for c in range(3):
    m = comp == c
    print("comp", c, m.sum(), d[m].mean(0).round(0), ph[m, 3].mean().round(0))
for f, name in [(1, 'MIP'), (8, 'CIIP'), (0x30, 'ISP'), (4, 'BDPCM')]:
    m = (flags & f) != 0
    if m.sum():
        print(name, m.sum(), d[m].mean(0).round(0), ph[m, 3].mean().round(0))
m = (comp > 0) & (mode >= 67)
print('CCLM', m.sum(), d[m].mean(0).round(0), ph[m, 3].mean().round(0))
for sz in [4, 8, 16, 32, 64]:
    m = (np.maximum(w, h) == sz)
    if m.sum():
        print('max dim', sz, m.sum(), d[m].mean(0).round(0), ph[m, 3].mean().round(0))
