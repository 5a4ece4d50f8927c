"""Summary of one tools/gpu_mc.sh run: per-picture MC kernel time and algorithmic GB/s from mc_bench.py,
and the per-kernel rocprofv3 durations (grid size distinguishes the kernels):
python tools/mc_summary.py <tag>"""
import glob
import json
import sqlite3
import sys

tag = sys.argv[1]
for line in open("gpurun_out/mcb_%s.json" % tag):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print(d["stream"], {n: (round(v["us_per_launch"] * v["launches"] / d["pictures"], 1), v["alg_GBps"]) for n, v in d["kernels"].items()})
for pat in ("gpurun_out/mcprof_%s/**/*.db", "gpurun_out/mcprof1080_%s/**/*.db"):
    dbs = sorted(glob.glob(pat % tag, recursive=True))
    if not dbs:
        continue
    print(pat.split("/")[1].split("_")[0])
    c = sqlite3.connect(dbs[0])
    for r in c.execute("select name, count(*), avg(duration), grid_x/workgroup_x, workgroup_x from kernels where name like '%mc%' group by name, grid_x"):
        print("  %-12s n=%d %8.2f us  wgs=%d x %d" % (r[0].split("::")[-1].split("(")[0], r[1], r[2] / 1e3, r[3], r[4]))
