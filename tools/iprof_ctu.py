"""Summarise gpurun_out/iprof_<stream>.npz of the CTU-resident k_intra (tools/intra_prof.py):
per-step wait / run and the phase split of run_step (cycle stamps)."""
import sys
import numpy as np
a = np.load(sys.argv[1])['prof']
a = a[(a[:, 9] == a[:, 9].max()) & (a[:, 8] == 0)]
t0, t1, t2 = (a[:, k].astype(np.int64) for k in range(3))
print("steps", len(a), "span us %.0f" % ((t2.max() - t0.min()) * 0.01))
w = (t1 - t0) * 0.01; r = (t2 - t1) * 0.01
print("wait mean %.2f med %.2f | run mean %.2f med %.2f p90 %.2f" % (w.mean(), np.median(w), r.mean(), np.median(r), np.percentile(r, 90)))
m16 = np.uint64(0xffff)
st = np.stack([(a[:, 3 + q // 4] >> np.uint64(16 * (q % 4))) & m16 for q in range(6)], 1).astype(np.int64)
names = ["wait+resid", "fill", "store_resid", "params+filter", "predict", "recon+ISP"]
d = np.diff(np.concatenate([np.zeros((len(a), 1), np.int64), st], 1), axis=1)
ok = (d >= 0).all(1)
print("phase cycles (median over %d steps):" % ok.sum(), dict(zip(names, np.median(d[ok], 0).round(0))))
print("phase cycles (mean):", dict(zip(names, d[ok].mean(0).round(0))))
info = a[:, 5]; W = (info >> 8) & 0xff; H = (info >> 16) & 0xff
for sz in [4, 8, 16, 32]:
    mm = ok & (np.maximum(W, H) == sz)
    print("maxdim", sz, mm.sum(), np.median(d[mm], 0).round(0))
