"""Per-kernel instruction mix and stall share from tools/pmc_sq.sh (rocprofv3 SQ counters, one pass per
group of 8): VALU / LDS / VMEM-read / SALU instructions per wave, and the share of wave-cycles spent
waiting for an instruction to issue (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).

  python tools/sq_summary.py gpurun_out/pmcsq_r01 > profiles/r01_sq_counters.txt
"""
import collections
import csv
import os
import re
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return agg, disp


def main(d):
    a, da = load(os.path.join(d, "a", "run_counter_collection.csv"))
    b, _ = load(os.path.join(d, "b", "run_counter_collection.csv"))
    print("# SQ counters per kernel (sum over dispatches of one bench step, --segments 1 --sync-pictures): %s" % d)
    print("# %-22s %5s %8s %9s %9s %9s %9s %9s %11s" % ("kernel", "disp", "waves", "VALU/wave", "LDS/wave", "VMEM/wave",
                                                         "SALU/wave", "wait%", "LDS_conflict"))
    for k in sorted(a, key=lambda k: -a[k].get("SQ_WAVE_CYCLES", 0)):
        if k.startswith("__amd"):
            continue
        w = max(a[k].get("SQ_WAVES", 0), 1)
        wc = max(a[k].get("SQ_WAVE_CYCLES", 0), 1)
        print("  %-22s %5d %8d %9.0f %9.0f %9.1f %9.0f %8.1f%% %11.3g" % (
            k[:22], len(da[k]), w, a[k].get("SQ_INSTS_VALU", 0) / w, a[k].get("SQ_INSTS_LDS", 0) / w,
            a[k].get("SQ_INSTS_VMEM_RD", 0) / w, b[k].get("SQ_INSTS_SALU", 0) / w,
            100 * a[k].get("SQ_WAIT_INST_ANY", 0) / wc, b[k].get("SQ_LDS_BANK_CONFLICT", 0)))


if __name__ == "__main__":
    main(sys.argv[1])
