"""Per-kernel statistics of the bench's kernel-table steps from a rocprofv3 kernel trace.

bench.py --kernel-table-only run with VVCR_TRACE_MARKERS=1 launches a one-block torch scan kernel right
before and right after its synced steps; this cuts the trace's dispatches between the two markers and
summarises them per kernel (count, average / median / min / max duration in microseconds), so the
trace's averages can be set beside the bench's HIP-event medians of the same launches.
  python tools/kt_trace.py gpurun_out/prof_x/run_kernel_trace.csv [--alg bench.json] > summary.json"""
import argparse
import csv
import json
import re
import statistics
import sys


def short(name):
    m = re.search(r"\b(k_\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--alg", help="bench.py --kernel-table-only JSON of the same run: adds algorithmic GB/s")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "scan" in r[2].lower()]
    if len(marks) < 2:
        sys.exit("kt_trace: fewer than two marker kernels in the trace")
    sel = rows[marks[0] + 1:marks[-1]]
    per = {}
    for s, e, n in sel:
        per.setdefault(short(n), []).append((e - s) / 1e3)
    out = {"trace": a.trace, "dispatches": len(sel), "window_ms": round((rows[marks[-1]][0] - rows[marks[0]][1]) / 1e6, 3),
           "kernels": {k: {"count": len(v), "avg_us": round(sum(v) / len(v), 2), "median_us": round(statistics.median(v), 2),
                           "min_us": round(min(v), 2), "max_us": round(max(v), 2)} for k, v in sorted(per.items())}}
    if a.alg:
        with open(a.alg) as f:
            b = json.load(f)
        for key, blk in (("mc_roofline", b.get("mc_roofline")), ("north_star_mc", b.get("north_star_mc"))):
            if not blk:
                continue
            for k in ("mc", "mc_bidir", "mc_affine"):
                kn = "k_" + k
                if kn in out["kernels"] and k in blk:
                    mb = blk[k]["alg_MB_per_launch"]
                    t = out["kernels"][kn]["avg_us"]
                    out["kernels"][kn]["alg_MB_per_launch"] = mb
                    out["kernels"][kn]["alg_GBps_at_avg"] = round(mb / t * 1e3, 1)
                    out["kernels"][kn]["hbm_frac_at_avg"] = round(mb / t * 1e3 / 8000.0, 4)
                    out["kernels"][kn]["bench_event_median_us"] = blk[k]["us_per_launch"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
