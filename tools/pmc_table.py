"""Per-kernel sums of rocprofv3 --pmc counter CSVs (run_counter_collection.csv of each pass directory),
divided by the dispatch count: python tools/pmc_table.py gpurun_out/pmcmc_new [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    tab = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            tab[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((os.path.dirname(f), r["Dispatch_Id"]))
    return tab, disp


if __name__ == "__main__":
    tab, disp = load(sys.argv[1])
    keys = sys.argv[2:] or list(tab)
    for k in tab:
        if not any(s in k for s in keys):
            continue
        c = tab[k]
        n = max(1, len({x[1] for x in disp[k]}))
        w = c.get("SQ_WAVES", 0) or 1
        print(k[:40], "dispatches~%d" % n)
        for name in sorted(c):
            v = c[name]
            extra = ("  per wave %.1f" % (v / w)) if name.startswith("SQ_") and name not in ("SQ_WAVES", "SQ_BUSY_CYCLES") else ""
            print("   %-24s %14.0f%s" % (name, v, extra))
