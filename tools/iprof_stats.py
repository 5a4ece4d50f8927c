"""Summarise gpurun_out/iprof_<stream>.npz (tools/intra_prof.py): phase cycles per step type."""
import sys
import numpy as np
a = np.load(sys.argv[1])['prof']
a = a[a[:, 7] == a[:, 7].max()]
info = a[:, 5]
comp = info & 0xff; w = (info >> 8) & 0xff; h = (info >> 16) & 0xff; flags = (info >> 24) & 0xff; mode = (info >> 32) & 0xff
ph = a[:, 1:5].astype(np.int64)
d = np.diff(np.concatenate([np.zeros((len(a), 1), np.int64), ph], 1), axis=1)
print("steps", len(a), "phase cycles [refs, params, predict, recon]", d.mean(0).round(0), "total", ph[:, 3].mean().round(0))
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
