"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite database or kernel_stats/kernel_trace CSV) into
the per-kernel table committed under profiles/:  name, calls, total ms, average us, min us, max us, share.

  python tools/prof_summary.py gpurun_out/prof_r01b/run_results.db > profiles/r01_rocprof_stats.txt
"""
import csv
import re
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    out = {}
    for name, dur, vg, sg, lds in c.execute(
            "select name, duration, vgpr_count, sgpr_count, lds_size from kernels"):
        r = out.setdefault(name, {"durs": [], "vgpr": vg, "sgpr": sg, "lds": lds})
        r["durs"].append(dur)
    return out


def rows_from_csv(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e = out.setdefault(r["Kernel_Name"], {"durs": [], "vgpr": r.get("VGPR_Count"),
                                                  "sgpr": r.get("SGPR_Count"), "lds": r.get("LDS_Block_Size")})
            e["durs"].append(d)
    return out


def main(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = (dbs or csvs)[0]
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    total = sum(sum(r["durs"]) for r in rows.values())
    print("# rocprofv3 --kernel-trace --stats summary of %s" % path)
    print("# %-60s %7s %11s %10s %10s %10s %6s  vgpr sgpr lds" %
          ("kernel", "calls", "total_ms", "avg_us", "min_us", "max_us", "pct"))
    for name, r in sorted(rows.items(), key=lambda kv: -sum(kv[1]["durs"])):
        d = r["durs"]
        short = name.replace("(anonymous namespace)::", "")
        short = re.sub(r"^void ", "", short).split("(")[0][:60]
        print("  %-60s %7d %11.3f %10.2f %10.2f %10.2f %6.2f  %4s %4s %s" % (
            short, len(d), sum(d) / 1e6, sum(d) / len(d) / 1e3, min(d) / 1e3, max(d) / 1e3,
            100.0 * sum(d) / total, r["vgpr"], r["sgpr"], r["lds"]))


if __name__ == "__main__":
    main(sys.argv[1])
