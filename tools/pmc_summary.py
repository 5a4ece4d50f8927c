"""Per-kernel HBM traffic from the rocprofv3 PMC passes of tools/pmc.sh, per launch, corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes read, so it is doubled. The guide establishes the factor for 16 B/lane
streaming reads; tools/probe/fetch_cal.hip measured it for every width the kernels use (2, 4, 8 and 16 B
per lane, and 8-byte chunks of 2-D windows as the MC gathers read them): exactly 0.500 in each case
(profiles/r03_fetch_calibration.txt), so the doubled figure is the read traffic, not an upper bound.

  python tools/pmc_summary.py gpurun_out/pmc_r01 [stream] > profiles/r01_traffic.json
"""
import collections
import csv
import json
import os
import re
import sys


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in agg.items()}, {k: len(v) for k, v in disp.items()}


def main(d, stream="ra1080_q32"):
    fetch, nf = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"))
    write, nw = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"))
    out = {"source": d, "stream": stream, "unit": "bytes per launch",
           "note": "read = 2 x FETCH_SIZE (gfx950 wide-read correction), write = WRITE_SIZE; KiB -> bytes",
           "per_launch_bytes": {}, "detail": {}}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd"):
            continue
        f = fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024
        w = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        out["per_launch_bytes"][k] = round(2 * f + w)
        out["detail"][k] = {"fetch_raw": round(f), "read_corrected": round(2 * f), "write": round(w),
                            "launches_sampled": nf.get(k, 0)}
    # kernel-group names used by bench.py (vvcr_kernel_stats groups)
    groups = {"resid": ["k_resid"], "intra": ["k_intra"], "mc": ["k_mc"],
              "mc_bidir": ["k_mc_bidir"], "mc_affine": ["k_mc_affine"], "recon_inter": ["k_recon_inter"],
              "sao": ["k_sao"], "alf": ["k_alf"], "deblock": ["k_dbk<0>", "k_dbk<1>"]}
    out["per_group_launch_bytes"] = {g: round(sum(out["per_launch_bytes"].get(k, 0) for k in ks))
                                     for g, ks in groups.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
