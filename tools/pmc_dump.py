"""Every counter of a rocprofv3 --pmc run directory (or several), per kernel, averaged per dispatch.
  python tools/pmc_dump.py gpurun_out/pmcmc_TAG/a gpurun_out/pmcmc_TAG/b ..."""
import collections
import csv
import glob
import os
import re
import sys


def main(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
                    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[k][r["Counter_Name"]].add((path, r["Dispatch_Id"]))
    for k in sorted(agg):
        if k.startswith("__amd"):
            continue
        print(k)
        for c in sorted(agg[k]):
            n = max(len(disp[k][c]), 1)
            print("   %-34s %16.1f per dispatch (%d)" % (c, agg[k][c] / n, n))


if __name__ == "__main__":
    main(sys.argv[1:])
