"""The N>1 bench plumbing (vvc_amd/dist.py) over gloo with world_size 2 on CPU: barrier, max-over-ranks of
the elapsed time, whole-job throughput = units of all ranks / slowest rank's time."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, %r)
from vvc_amd import dist as V
R = V.Ranks()
R.barrier()
el = R.max_over_ranks(1.0 + R.rank)          # rank r took 1 + r seconds
val = V.job_throughput(100.0 * (R.rank + 1), el, R)
print(json.dumps({"rank": R.rank, "world": R.world, "elapsed": el, "value": val}))
R.close()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_timing_and_throughput():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), VVCR_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER % ROOT], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    import json
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for o in outs:
        assert o["world"] == 2
        assert o["elapsed"] == 2.0                  # the slowest rank
        assert abs(o["value"] - 300.0 / 2.0) < 1e-9 # (100 + 200) units / 2 s
