"""Only bench.py's sharded leg (BASELINE config 4, the `shard` object of the bench line), for iterating on it.

  python tools/shard_leg.py [--shard-stream ra4320t_q32] [--shard-steps 3]
  (N ranks: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/shard_leg.py)

Prints the `shard` object as one JSON line on rank 0, plus the per-phase host timings of one more
decode when VVCP_PHASES=1.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from vvc_amd import dist as V  # noqa: E402


def phases(a, R):
    """one more decode with every phase of StreamShardRank timed (host wall clock, ms per picture)"""
    import time
    from vvc_amd import native as N
    from vvc_amd import parser as PZ
    from vvc_amd import shard as SH
    acc = {}

    def timed(name, f):
        def g(*args, **kw):
            t = time.perf_counter()
            try:
                return f(*args, **kw)
            finally:
                acc.setdefault(name, []).append(round((time.perf_counter() - t) * 1e3, 2))
        return g
    for name in ("parse", "local_deltas", "refine", "plan", "launch_recon", "launch_lf"):
        setattr(SH.StreamShardRank, name, timed(name, getattr(SH.StreamShardRank, name)))
    data = open(os.path.join(ROOT, "tests", "golden", "streams", a.shard_stream + ".bin"), "rb").read()
    ps = PZ.Stream(data)
    inf = ps.info(0)
    ps.close()
    ctx = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=8,
                    device=int(os.environ.get("VVCR_DEVICE", R.local)))
    ctx.set_timing(False)
    comm = SH.TorchComm(R.device) if R.world > 1 else None
    for k in range(2):
        acc.clear()
        t0 = time.perf_counter()
        rk = SH.StreamShardRank(ctx, data, R.rank, R.world, 8)
        acc["open"] = [round((time.perf_counter() - t0) * 1e3, 2)]
        for i in range(rk.n):
            SH.decode_stream_picture(rk, comm, i)
        ctx.sync()
        total = (time.perf_counter() - t0) * 1e3
        rk.release()
    ctx.close()
    return {"total_ms": round(total, 2), "phases_ms": acc}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-stream", default="ra4320t_q32")
    ap.add_argument("--shard-steps", type=int, default=3)
    a = ap.parse_args()
    R = V.Ranks()
    out = bench.shard_bench(a, R)
    if R.rank == 0:
        print(json.dumps(out))
    if os.environ.get("VVCP_PHASES"):
        ph = phases(a, R)
        if R.rank == 0:
            print(json.dumps(ph))
    R.close()


if __name__ == "__main__":
    main()
