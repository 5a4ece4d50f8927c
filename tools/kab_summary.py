"""Summary of a tools/gpu_kab.sh run: parity log tail, per-kernel average time new vs old library,
and the bench-line A/B values. Usage: python tools/kab_summary.py <tag> [kernel-substring ...]"""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
pats = sys.argv[2:]
out = "gpurun_out"
lp = os.path.join(out, "pytest_%s.log" % tag)
log = open(lp).read().strip().splitlines() if os.path.exists(lp) else []
print(log[-1] if log else "(no pytest log)")
stats = {}
for v in ("new", "old"):
    f = os.path.join(out, "kab_%s_%s" % (tag, v), "run_kernel_stats.csv")
    if os.path.exists(f):
        stats[v] = {r["Name"]: r for r in csv.DictReader(open(f))}
if stats:
    names = sorted(stats.get("new", {}), key=lambda n: -float(stats["new"][n]["TotalDurationNs"]))
    tot = {v: sum(float(r["TotalDurationNs"]) for r in s.values()) / 1e6 for v, s in stats.items()}
    print("total kernel ms: " + "  ".join("%s %.2f" % kv for kv in tot.items()))
    for n in names:
        short = n.replace("(anonymous namespace)::", "")[:40]
        if pats and not any(p in n for p in pats):
            continue
        row = ["%-40s" % short]
        for v in ("new", "old"):
            r = stats.get(v, {}).get(n)
            row.append("%s %5s x %7.1f us" % (v, r["Calls"], float(r["AverageNs"]) / 1e3) if r else "%s -" % v)
        print("  ".join(row))
vals = {}
for f in sorted(glob.glob(os.path.join(out, "bab_%s_*.json" % tag))):
    env = open(f[:-5] + ".env").read().strip()
    try:
        vals.setdefault(env, []).append(json.loads(open(f).read().strip().splitlines()[-1])["value"])
    except Exception as e:  # noqa: BLE001
        vals.setdefault(env, []).append(str(e))
for k, v in vals.items():
    print("bench %-40s %s" % (k, v))
