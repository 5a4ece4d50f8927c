"""Per-rank CABAC time of the config-4 shard split (host only, no GPU): for N = 1, 2, 4, 8 ranks of the 8K
tile-row stream, each rank's parser covers only the tiles around its rows (vvcp_set_parse_rows, the bench's
shard leg: shard.parse_rows) and the CABAC pass of every picture is timed (min of --reps). Prints one JSON
line: per N the per-rank milliseconds and the slowest rank against N = 1 (the strong-scaling bound of the
parse phase).

  VVCP_TILE_THREADS=1 python tools/shard_parse_split.py     (work per rank; default threads: latency)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vvc_amd import parser as PZ  # noqa: E402
from vvc_amd import shard as SH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="ra4320t_q32")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "streams", a.stream + ".bin"), "rb") as f:
        data = f.read()
    ps = PZ.Stream(data)
    inf, pp, n = ps.info(0), ps.pic_params(0), len(ps)
    ps.close()
    ctu = 1 << inf["ctu_log2"]
    for _ in range(2):   # warm-up: the first streams of a process pay the first touch of their pages
        s = PZ.Stream(data)
        for i in range(n):
            s.parse(i)
        s.close()
    out = {"stream": a.stream, "pictures": n, "tile_threads": os.environ.get("VVCP_TILE_THREADS", "default"), "ranks": {}}
    for world in (1, 2, 4, 8):
        rows = SH.stream_shard_rows(pp, inf["height"], inf["ctu_log2"], world)
        per = []
        for y0, y1 in rows:
            best = None
            for _ in range(a.reps):
                s = PZ.Stream(data)
                if world > 1:
                    s.set_parse_rows(*SH.parse_rows(y0, y1, ctu))
                t0 = time.perf_counter()
                for i in range(n):
                    s.parse(i)
                t = (time.perf_counter() - t0) * 1e3
                s.close()
                best = t if best is None else min(best, t)
            per.append(round(best, 1))
        out["ranks"][world] = {"rows": rows, "parse_ms": per, "slowest_ms": max(per)}
    base = out["ranks"][1]["slowest_ms"]
    for w, v in out["ranks"].items():
        v["speedup_vs_1"] = round(base / v["slowest_ms"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
