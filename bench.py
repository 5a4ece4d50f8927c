"""Decode throughput of the MI355X path on BASELINE.json configs[2], the largest single-GPU
configuration: 4K 3840x2160 random access QP27 (the north star's QP32 is --stream ra2160l_q32).

value (the headline) is END TO END FROM THE BITSTREAM: every step decodes the .bin again from its first
NAL unit - header parsing, the CABAC pass of every picture (host threads), motion derivation in decoding
order with each collocated picture's DMVR deltas read back from the GPU, host planning (work lists,
intra dependency plan, deblocking edges), upload (vvcr_prepare_planned) and the GPU (residuals, motion
compensation with DMVR/BDOF/affine-PROF/GEO/CIIP, intra, deblocking, SAO, ALF/CC-ALF) - all inside the
timed region. One step = `--segments` independent decodes of the whole stream, all in flight at once (a
serving process decoding that many streams; vvc_amd/bitstream.py), so `steps` x `segments` decodes are timed
and the rate is a steady state, not the latency of the first intra pictures.
The `resident` object is the same reconstruction with every picture already planned and resident in
HBM (launch only): the GPU-side rate. Output is checked bit-exact against DecoderApp: the YUV file MD5
of one decode, and the plane MD5s of every segment's pictures after the timed steps.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--stream ra2160l_q27] [--no-cpu]

Multi-GPU: one process per GPU (torch.distributed.run; a plain `python bench.py --gpus N` spawns the N
ranks itself before anything touches the GPU). N ranks decode N independent replicas of the stream
(weak scaling, no data-path collective); the timing barrier and max-over-ranks use torch.distributed.
"""
import os
import sys

USER_LANES = "VVCR_LANES" in os.environ or "VVCR_INTRA_LANES" in os.environ


def _spawn_ranks():
    """`python bench.py --gpus N` outside torch.distributed.run: start the N ranks as child processes
    (nothing here has touched the GPU yet) and exit with their status."""
    import argparse
    import socket
    import subprocess
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != a.gpus:
            sys.exit("bench: --gpus %d but WORLD_SIZE=%s" % (a.gpus, world))
        return
    if a.gpus <= 1:
        return
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def _default_stream():
    root = os.path.dirname(os.path.abspath(__file__))
    # the longest 4K RA QP27 stream captured: 17 pictures (I + GOP 16), 9 (I + 8), else the 3-picture one
    for n in ("ra2160l_q27", "ra2160n_q27", "ra2160_q27"):
        if os.path.isdir(os.path.join(root, "tests", "golden", n)):
            return n
    return "ra2160_q27"


def _lanes_for(stream):
    """Execution lanes (libvvcr reads VVCR_LANES / VVCR_INTRA_LANES at vvcr_create) and the HIP hardware
    queues they need: each lane, the library's copy stream and torch's stream on a queue of its own, so
    GPU_MAX_HW_QUEUES = lanes + 2 (the box exports HIP's default of 4; the limit here is 32). Measured:
    4K 12 lanes (7 intra) 9.0 vs 8 (5) 8.6 Gpx/s; 1080p 9 (5) 11.2-12.3 vs 8 (5) 10.5-12.2, 12 (7) 10.7."""
    small = any(t in stream for t in ("1080", "480", "416", "412"))
    lanes, intra = (9, 5) if small else (12, 7)
    if not USER_LANES:
        os.environ["VVCR_LANES"], os.environ["VVCR_INTRA_LANES"] = str(lanes), str(intra)
    lanes = int(os.environ.get("VVCR_LANES", lanes))
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < lanes + 2:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, lanes + 2))


if __name__ == "__main__":
    _spawn_ranks()
    import argparse as _ap
    _p = _ap.ArgumentParser(add_help=False)
    _p.add_argument("--stream", default=None)
    _lanes_for(_p.parse_known_args()[0].stream or _default_stream())

import argparse
import hashlib
import glob
import json
import os
import subprocess
import sys
import resource
import time

import numpy as np
import torch  # noqa: F401  (before any libvvcr context: torch's HIP runtime must load first)

ROOT = os.path.dirname(os.path.abspath(__file__))


def _thread_cpu():
    """{tid: (name, user + system CPU seconds)} of this process's threads (/proc, diagnostics)"""
    out, tick = {}, os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            st = open("/proc/self/task/%s/stat" % t).read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        out[int(t)] = (name, (int(f[11]) + int(f[12])) / tick)
    return out
sys.path.insert(0, ROOT)

from vvc_amd import native as N  # noqa: E402
from vvc_amd import stream as S  # noqa: E402
from vvc_amd import decode as D  # noqa: E402
from vvc_amd import dist as V  # noqa: E402

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E peak (guides/MI355X_MICROARCH.md)


def cpu_baseline(stream_bin, pixels_per_run, min_seconds=10.0, max_runs=40):
    """VTM DecoderApp (the reference, built here from /root/reference by oracle/ref.mk) on the same
    bitstream, single-threaded, no output file and no decoded-picture-hash check (-dph 0, as BASELINE.md
    §2 times it: SEIDecodedPictureHash defaults to on, DecAppCfg.cpp:91, ~11 % of VTM's time); repeated
    until ~min_seconds of CPU work."""
    exe = os.path.join(ROOT, "oracle", "_ref", "DecoderApp")
    if not os.path.exists(exe):
        return None
    runs, total = 0, 0.0
    while total < min_seconds and runs < max_runs:
        t0 = time.perf_counter()
        r = subprocess.run([exe, "-b", stream_bin, "-dph", "0"], capture_output=True, text=True)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            return None
        runs += 1
        total += dt
    return {"value": round(pixels_per_run * runs / total / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "reference",
            "sample": "VTM-7.3 DecoderApp -b %s.bin -dph 0 (x86 SIMD, 1 thread, no output file, no hash check), %d runs (%.1f s), parse + reconstruction"
                      % (os.path.basename(stream_bin)[:-4], runs, total)}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_all_cores(stream_bin, pixels_per_run, procs, runs_each=2):
    """The like-for-like comparator of the headline's `procs` host threads:
    `procs` VTM DecoderApp processes (-dph 0, one thread each) decoding the same bitstream at once, each
    `runs_each` times back to back; total pixels of every run / wall time from the first start to the last
    end."""
    import threading
    exe = os.path.join(ROOT, "oracle", "_ref", "DecoderApp")
    if not os.path.exists(exe):
        return None
    fails = []

    def worker():
        for _ in range(runs_each):
            r = subprocess.run([exe, "-b", stream_bin, "-dph", "0"], capture_output=True, text=True)
            if r.returncode != 0:
                fails.append(r.returncode)
    th = [threading.Thread(target=worker) for _ in range(procs)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    if fails:
        return None
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"value": round(pixels_per_run * procs * runs_each / wall / 1e6, 3), "unit": "Mpixels/s", "cores": procs,
            "kind": "reference", "cpu": cpu_model(), "affinity_cpus": aff,
            "sample": "%d concurrent VTM-7.3 DecoderApp processes (x86 SIMD, 1 thread each, -dph 0, no output file), "
                      "each decoding %s.bin %d times; %.1f s wall" % (procs, os.path.basename(stream_bin)[:-4], runs_each, wall)}


class _Roctx:
    """Bracketing of the kernel-table steps for a rocprofv3 kernel trace of the same command:
    * VVCR_ROCTX_REGIONS=1: roctxProfilerResume(0) / roctxProfilerPause(0) (rocprofv3 --selected-regions
      collects only between them);
    * VVCR_TRACE_MARKERS=1: a one-block torch cumsum kernel on the device right before and right after the
      steps (host-synchronised), so tools/kt_trace.py can cut the steps' launches out of any kernel trace."""
    L = None

    @classmethod
    def _lib(cls):
        if cls.L is None and os.environ.get("VVCR_ROCTX_REGIONS") == "1":
            import ctypes
            cls.L = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
        return cls.L

    @staticmethod
    def _marker():
        if os.environ.get("VVCR_TRACE_MARKERS") == "1":
            torch.cuda.synchronize()
            torch.arange(8, device="cuda").cumsum(0)
            torch.cuda.synchronize()

    @classmethod
    def resume(cls):
        cls._marker()
        if cls._lib() is not None:
            cls.L.roctxProfilerResume(0)

    @classmethod
    def pause(cls):
        if cls._lib() is not None:
            cls.L.roctxProfilerPause(0)
        cls._marker()


def kernel_table(ctx, groups, reps, sync="picture"):
    """Per-kernel HIP-event durations (events on the library's lanes, vvcr_kernel_stats) of one decode's
    resident pictures, launched as the decode loop launches them (`groups`: single pictures and
    frame-batched pairs, bitstream.launch_groups): `reps` steps, each launching every group with a host sync
    after it (no kernel overlaps another group's), summed per kernel and step; the table keeps the MEDIAN
    step's time per kernel and its min / max across the steps. These are the launches a
    `VVCR_ROCTX_REGIONS=1 rocprofv3 --selected-regions` trace of the same command records. Returns {name:
    [launches, ms, alg_bytes, ms_min, ms_max, pictures]} (per step; pictures: the pictures the kernel's
    launches carried, > launches for the frame-batched k_mc)."""
    from vvc_amd import bitstream as B
    ctx.set_timing(True)
    steps = []
    _Roctx.resume()
    for _ in range(max(1, reps)):
        for g in groups:
            B.launch_group(ctx, g)
            if sync == "picture":
                ctx.sync()
        ctx.sync()
        rep = {}
        for g in groups:
            for hnd in g:
                for name, launches, ms, alg, pics in ctx.kernel_stats(hnd):
                    k = rep.setdefault(name, [0, 0.0, 0.0, 0])
                    k[0] += launches
                    k[1] += ms
                    k[2] += alg
                    k[3] += pics if launches else 0
        steps.append(rep)
    _Roctx.pause()
    ctx.set_timing(False)
    out = {}
    for name in sorted(set().union(*steps)):
        v = [s[name] for s in steps if name in s and s[name][0]]
        if not v:
            continue
        ms = sorted(x[1] for x in v)
        out[name] = [v[0][0], float(np.median(ms)), v[0][2], ms[0], ms[-1], v[0][3]]
    return out


def resident_handles(ctx, data, per, base=0):
    """One decode of the stream on slots [base, base + per), its prepared pictures kept: their launch groups
    (decoding order, frame-batched pairs as vvcp_decode launches them), handles and (poc, slot)s."""
    from vvc_amd import bitstream as B
    seq = B.SequenceDecode(ctx, data, nslots=per, base=base, threads=8)
    _, handles = seq.run(keep_handles=True)
    ctx.sync()
    return B.launch_groups(handles, seq.batch), handles, [(inf["poc"], seq.slot[i]) for i, inf in enumerate(seq.info)]


def mc_roofline(kern, note):
    out = {"peak": PEAK_HBM_GBS, "unit": "GB/s", "note": note}
    tot = [0.0, 0.0]
    for k in ("mc", "mc_affine", "mc_bidir"):
        v = kern.get(k, [0, 0.0, 0.0, 0.0, 0.0, 0])
        g = v[2] / (v[1] / 1e3) / 1e9 if v[1] > 0 else 0.0
        out[k] = {"achieved": round(g, 2), "frac": round(g / PEAK_HBM_GBS, 4),
                  "us_per_launch": round(v[1] / max(v[0], 1) * 1e3, 2),
                  "us_per_launch_min_max": [round(v[3] / max(v[0], 1) * 1e3, 2), round(v[4] / max(v[0], 1) * 1e3, 2)],
                  "alg_MB_per_launch": round(v[2] / max(v[0], 1) / 1e6, 3), "launches_per_step": v[0],
                  "pictures_per_step": v[5], "us_per_picture": round(v[1] / max(v[5], 1) * 1e3, 2)}
        tot[0] += v[2]
        tot[1] += v[1]
    g = tot[0] / (tot[1] / 1e3) / 1e9 if tot[1] > 0 else 0.0
    out["mc_stage"] = {"achieved": round(g, 2), "frac": round(g / PEAK_HBM_GBS, 4), "ms_per_step": round(tot[1], 4)}
    return out


def north_star_mc(ctx, stream, per, reps, sync="picture"):
    """north_star's MC target is quoted on 4K RA QP32: the same kernel table on that stream."""
    p = os.path.join(ROOT, "tests", "golden", "streams", stream + ".bin")
    if not os.path.exists(p):
        return None
    with open(p, "rb") as f:
        data = f.read()
    groups, handles, slots = resident_handles(ctx, data, per)
    meta = S.load_meta(os.path.join(ROOT, "tests", "golden", stream))
    kern = kernel_table(ctx, groups, reps, sync)
    ok = check_slots(ctx, {slot: poc for poc, slot in slots}, meta)
    for h in handles:
        ctx.release(h)
    r = mc_roofline(kern, "%s, one segment, a host sync after every picture, median of %d steps (HIP events)" % (stream, reps))
    r["stream"] = stream
    r["bitexact_vs_reference"] = bool(ok)
    return r


def shard_bench(a, R):
    """BASELINE config 4 end to end from the bitstream: one tile-row stream decoded by all ranks together
    (vvc_amd/shard.py StreamShardRank). Every rank parses the .bin (CABAC, motion derivation with the
    all-gathered DMVR deltas of each reference), plans and reconstructs its own tile rows, and exchanges
    only the loop-filter halo (24 pre-deblocking rows per edge) and, per picture, the motion reach of its
    references with its neighbours over torch.distributed (RCCL on the GPU box). Strong scaling: the whole
    job decodes every picture once per step; parse + derive + plan + upload + GPU are all in the timed
    region. Checked bit-exact afterwards: rank 0 gathers every rank's rows of each picture and compares
    its MD5s."""
    from vvc_amd import parser as PZ
    from vvc_amd import shard as SH
    path = os.path.join(ROOT, "tests", "golden", "streams", a.shard_stream + ".bin")
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    meta = S.load_meta(os.path.join(ROOT, "tests", "golden", a.shard_stream))
    ps = PZ.Stream(data)
    inf = ps.info(0)
    npic = len(ps)
    ps.close()
    W, H = inf["width"], inf["height"]
    slots = 8
    ctx = N.Context(W, H, bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=slots,
                    device=int(os.environ.get("VVCR_DEVICE", R.local)))
    comm = SH.TorchComm(R.device) if R.world > 1 else None
    ctx.set_timing(False)

    def decode(check):
        rk = SH.StreamShardRank(ctx, data, R.rank, R.world, slots)
        ok = True
        for i in range(rk.n):
            SH.decode_stream_picture(rk, comm, i)
            if check:
                SH.gather_to_root(rk, comm, rk.slots[i])
                if R.rank == 0:
                    got = D.plane_md5s([ctx.read_plane(N.BUF_RECO, rk.slots[i], c) for c in range(3)])
                    ok = ok and got == meta["poc_plane_md5"][str(rk.info[i]["poc"])]
        ctx.sync()
        rows, reach = rk.rows, rk.reach
        rk.release()
        return ok, rows, reach
    ok, rows, reach = decode(True)   # warm-up and parity
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(a.shard_steps):
        decode(False)
    t1 = time.perf_counter()
    R.barrier()
    elapsed = R.max_over_ranks(t1 - t0)
    ctx.close()
    px = W * H * npic * a.shard_steps
    return {"value": round(px / elapsed / 1e6, 2), "unit": "Mpixels/s", "n_gpus": R.world, "scaling": "strong",
            "stream": a.shard_stream, "picture": "%dx%d" % (W, H), "pictures_per_step": npic, "steps": a.shard_steps,
            "ms_per_step": round(elapsed / a.shard_steps * 1e3, 3), "shard_rows": [b - y for y, b in rows],
            "lf_halo_rows": SH.LF_HALO, "max_ref_reach_rows": reach, "bitexact_vs_reference": bool(ok) if R.rank == 0 else None,
            "scope": "from the bitstream: parse + motion derivation + shard planning + upload + GPU + halo exchanges",
            "note": "tile-row shards, halos over torch.distributed %s point to point, DMVR deltas all-gathered" % (
                R.dist.get_backend() if R.dist else "-")}


class BitstreamE2E:
    """The headline: bitstream in, pictures out, everything in the timed region.

    Every step decodes the .bin again from its first NAL: a fresh host parser (vvcp_open: NAL split and
    every header), then one native decode loop (vvcp_decode, GIL released): the CABAC pass of each
    picture on threads // segments parser threads, motion derivation in decoding order with each
    collocated picture's DMVR deltas from the GPU, native planning (vvcp_plan_picture), upload
    (vvcr_prepare_planned) and the GPU. Steps run as `segments` independent decodes in flight at once,
    each on its own DPB slot range and host thread (a serving process decoding several streams)."""

    def __init__(self, ctx, data, per, segments, threads):
        import concurrent.futures as cf
        import threading
        from vvc_amd import bitstream as B
        self.B, self.ctx, self.data, self.per, self.segments = B, ctx, data, per, segments
        self.parse_threads = max(1, threads // segments)   # parser threads per decode (vvcp_decode)
        self.seg_ex = cf.ThreadPoolExecutor(segments)
        self.final = [None] * segments   # per segment: {slot: poc} after its last decode
        self.times = {}                  # summed per-phase seconds of the decode threads
        self.tlock = threading.Lock()

    def _decode(self, c):
        seq = self.B.SequenceDecode(self.ctx, self.data, nslots=self.per, base=self.per * c, threads=self.parse_threads)
        seq.run()
        with self.tlock:
            for k, v in seq.times.items():
                self.times[k] = self.times.get(k, 0.0) + v
        owner = {}
        for i, inf in enumerate(seq.info):
            owner[seq.slot[i]] = inf["poc"]
        self.final[c] = owner

    def _segment(self, c, n):
        for _ in range(n):
            self._decode(c)

    def run(self, steps):
        """`steps` steps: every segment decodes the stream `steps` times (one step = `segments` decodes of the
        whole stream, all in flight); returns when every picture is launched (not finished)."""
        futs = [self.seg_ex.submit(self._segment, c, steps) for c in range(self.segments)]
        for f in futs:
            f.result()

    def close(self):
        self.ctx.sync()
        self.seg_ex.shutdown()


def e2e_legs(ctx, data, meta, per, segments, steps, warmup, single_steps, threads, R, px_seq, npic):
    """The end-to-end legs of one stream: `segments` decodes in flight (steps x segments decodes timed) and
    one decode in flight (single_steps decodes timed), both from the bitstream; every segment's pictures
    checked against the reference's MD5s afterwards. Returns (value Mpx/s, ms per step, host ms per picture,
    host rusage, single-stream object, bit-exact)."""
    bitexact = True
    e2e = BitstreamE2E(ctx, data, per, segments, threads)
    if warmup > 0:
        e2e.run(warmup)
        ctx.sync()
    e2e.times = {}
    R.barrier()
    ctx.sync()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    th0 = _thread_cpu() if os.environ.get("VVCR_BENCH_THREADS") else None
    t0 = time.perf_counter()
    e2e.run(steps)
    ctx.sync()
    t1 = time.perf_counter()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    if th0 is not None:   # diagnostics: CPU of every thread of the process over the timed steps
        th1 = _thread_cpu()
        d = sorted(((th1[k][1] - th0.get(k, (None, 0))[1], k, th1[k][0]) for k in th1), reverse=True)
        print("threads: %d, CPU s over the timed steps: total %.2f; top: %s" % (
            len(d), sum(x[0] for x in d), ", ".join("%s/%d %.2f" % (n, k, v) for v, k, n in d[:24])), file=sys.stderr)
    R.barrier()
    elapsed = R.max_over_ranks(t1 - t0)
    npic_timed = steps * segments * npic
    # the process's CPU over the timed steps (all threads, this rank): user / system ms and page faults per picture
    host_rusage = {"user_ms_per_picture": round((ru1.ru_utime - ru0.ru_utime) / npic_timed * 1e3, 3),
                   "sys_ms_per_picture": round((ru1.ru_stime - ru0.ru_stime) / npic_timed * 1e3, 3),
                   "minor_faults_per_picture": round((ru1.ru_minflt - ru0.ru_minflt) / npic_timed, 1),
                   "cores_busy": round(((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / (t1 - t0), 2)}
    for owner in e2e.final:
        if owner is not None:
            bitexact = bitexact and check_slots(ctx, owner, meta)
    e2e.close()
    host_ms = {k: round(v / npic_timed * 1e3, 3) for k, v in e2e.times.items()}
    value = V.job_throughput(px_seq * segments * steps, elapsed, R) / 1e6
    # single stream: one decode at a time (latency view of the same path)
    single = None
    if single_steps > 0:
        ss = BitstreamE2E(ctx, data, per, 1, threads)
        ss.run(1)
        ctx.sync()
        ss.times = {}
        R.barrier()
        s0 = time.perf_counter()
        ss.run(single_steps)
        ctx.sync()
        s1 = time.perf_counter()
        R.barrier()
        s_el = R.max_over_ranks(s1 - s0)
        for owner in ss.final:
            if owner is not None:
                bitexact = bitexact and check_slots(ctx, owner, meta)
        ss.close()
        single = {"value": round(V.job_throughput(px_seq * single_steps, s_el, R) / 1e6, 2), "unit": "Mpixels/s",
                  "decodes": single_steps, "ms_per_decode": round(s_el / single_steps * 1e3, 3),
                  "host_ms_per_picture": {k: round(v / (single_steps * npic) * 1e3, 3) for k, v in ss.times.items()},
                  "note": "one decode in flight (%d worker threads: CABAC ahead, plan + upload pipelined; motion derivation "
                          "in decoding order), end to end from the bitstream like value" % threads}
    return value, elapsed / steps * 1e3, host_ms, host_rusage, single, bitexact


def cpu_ratios(value, single, cb, ca, threads):
    """vs_cpu_baseline (one DecoderApp core) and vs_cpu_baseline_all_cores (`threads` DecoderApp processes)."""
    out = {}
    if cb and cb.get("value"):
        out["vs_cpu_baseline"] = {"value": round(value / cb["value"], 1),
                                  "single_stream": round(single["value"] / cb["value"], 1) if single else None}
    if ca and ca.get("value"):
        out["vs_cpu_baseline_all_cores"] = {"value": round(value / ca["value"], 2),
                                            "single_stream": round(single["value"] / ca["value"], 2) if single else None,
                                            "note": "value uses %d host threads + the GPU; the comparator %d DecoderApp "
                                                    "processes on %d cores" % (threads, ca["cores"], ca["cores"])}
    return out


def north_star_e2e(ctx, a, R, per):
    """north_star's target is quoted on 4K RA QP32 (>= 20x VTM CPU decode at 1 MI355X): the headline's legs
    on that stream, end to end from the bitstream, with its own CPU baselines (rank 0, one GPU)."""
    name = a.north_star_stream
    p = os.path.join(ROOT, "tests", "golden", "streams", name + ".bin")
    if not os.path.exists(p):
        return None
    with open(p, "rb") as f:
        data = f.read()
    meta = S.load_meta(os.path.join(ROOT, "tests", "golden", name))
    from vvc_amd import parser as P
    ps = P.Stream(data)
    infos = [ps.info(i) for i in range(len(ps))]
    ps.close()
    W, H = infos[0]["width"], infos[0]["height"]
    if (W, H) != (ctx.width, ctx.height):
        return {"error": "north-star stream %dx%d differs from the headline context" % (W, H)}
    px_seq = W * H * len(infos)
    value, ms_step, host_ms, rus, single, ok = e2e_legs(ctx, data, meta, per, a.segments, a.north_star_steps, 1,
                                                        a.single_steps, a.e2e_threads, R, px_seq, len(infos))
    out = {"stream": name, "value": round(value, 2), "unit": "Mpixels/s",
           "workload": "%s: %dx%d random access QP32, %d pictures per decode, %d decodes per step" % (name, W, H, len(infos), a.segments),
           "steps": a.north_star_steps, "ms_per_step": round(ms_step, 3), "host_ms_per_picture": host_ms, "host_rusage": rus,
           "single_stream": single, "bitexact_vs_reference": bool(ok)}
    if R.rank == 0 and R.world == 1 and not a.no_cpu:
        cb = out["cpu_baseline"] = cpu_baseline(p, px_seq)
        ca = out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(p, px_seq, a.e2e_threads)
        out.update(cpu_ratios(value, single, cb, ca, a.e2e_threads))
    return out


def output_yuv_md5(ctx, data, meta):
    """One decode with DecoderApp's output: the YUV file's MD5 (vvcr_write_output, output order) and
    every output picture's plane MD5s, compared with the reference's."""
    from vvc_amd import bitstream as B
    from vvc_amd import parser as P
    s = P.Stream(data)
    inf = s.info(0)
    s.close()
    op = N.OutputParams(0, inf["conf_left"], inf["conf_right"], inf["conf_top"], inf["conf_bottom"], 0)
    yuv, ok = hashlib.md5(), [True]

    def on_output(poc, slot):
        yuv.update(ctx.write_output(slot, op).tobytes())
        exp = meta["poc_plane_md5"].get(str(poc))
        if exp is not None and D.plane_md5s([ctx.read_plane(N.BUF_RECO, slot, c) for c in range(3)]) != exp:
            ok[0] = False
    B.SequenceDecode(ctx, data, nslots=min(16, ctx.dpb_slots), threads=8).run(on_output)
    ctx.sync()
    return ok[0] and yuv.hexdigest() == meta["yuv_md5"]


def read_slot(ctx, slot):
    return [ctx.read_plane(N.BUF_RECO, slot, c) for c in range(3)]


def check_slots(ctx, owner, meta):
    return all(D.plane_md5s(read_slot(ctx, slot)) == meta["poc_plane_md5"][str(poc)] for slot, poc in owner.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--stream", default=_default_stream())
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--segments", type=int, default=0,
                    help="independent decodes in flight; one step = each of them decodes the whole stream once (<= 32). "
                         "Default: 16 at 4K and above, 12 below (4K 9-picture stream, end to end: 12 / 16 / 20 in flight "
                         "2545 / 2763 / 2572 Mpx/s; 1080p 33 pictures: 12 / 16 2372 / 2122)")
    ap.add_argument("--resident-steps", type=int, default=20, help="timed steps of the resident (pre-planned) pass, 0 = skip")
    ap.add_argument("--single-steps", type=int, default=5, help="timed decodes of the single-stream pass (one decode in flight), 0 = skip")
    ap.add_argument("--kernel-table-reps", type=int, default=7,
                    help="one-segment steps of the kernel table / roofline (a sync after every picture); each kernel "
                         "reports its median step with the min / max")
    ap.add_argument("--kernel-table-only", action="store_true",
                    help="profiling: only the kernel table of --stream and of --north-star-stream (with "
                         "VVCR_ROCTX_REGIONS=1 under rocprofv3 --selected-regions the trace holds exactly those steps)")
    ap.add_argument("--kernel-table-sync", choices=("picture", "step"), default="picture",
                    help="host sync after every picture of a kernel-table step, or only after the step")
    ap.add_argument("--north-star-stream", default="ra2160l_q32",
                    help="north_star's MC target stream (4K RA QP32): its MC kernel table goes into `north_star_mc`")
    ap.add_argument("--sync-pictures", action="store_true",
                    help="host sync after every picture of the resident pass (profiling: kernel durations without overlap)")
    ap.add_argument("--e2e-threads", type=int, default=16,
                    help="host planning threads (the GPU box's CPU share is 16)")
    ap.add_argument("--north-star-steps", type=int, default=4,
                    help="timed steps of the north-star stream's end-to-end leg (`north_star_e2e`, 0 = skip)")
    ap.add_argument("--shard-stream", default="ra4320t_q32",
                    help="tile-row stream of the spatially sharded pass (BASELINE config 4: 8K, one shard per rank)")
    ap.add_argument("--shard-steps", type=int, default=3, help="timed steps of the sharded pass (0 = skip it)")
    ap.add_argument("--shard-timeout", type=int, default=300,
                    help="N > 1: seconds the sharded pass may take before the line is printed without it (0 = no limit)")
    a = ap.parse_args()

    R = V.Ranks()
    world, rank, local = R.world, R.rank, R.local
    if world != a.gpus:
        sys.exit("bench: --gpus %d but %d ranks" % (a.gpus, world))

    d = os.path.join(ROOT, "tests", "golden", a.stream)
    meta = S.load_meta(d)
    with open(os.path.join(ROOT, "tests", "golden", "streams", a.stream + ".bin"), "rb") as f:
        data = f.read()
    from vvc_amd import parser as P
    ps = P.Stream(data)
    infos = [ps.info(i) for i in range(len(ps))]
    ps.close()
    W, H = infos[0]["width"], infos[0]["height"]
    if a.segments <= 0:
        a.segments = 16 if W * H >= 3840 * 2160 else 12
    px_seq = W * H * len(infos)
    nI = sum(1 for inf in infos if inf["slice_type"] == 2)

    per = min(16, 256 // a.segments)   # DPB slots per copy (at most 256 in all)
    # k_intra workgroups (VVCR_INTRA_WG, read at vvcr_create): the library's default sizes one intra picture at
    # a time (32 at 1080p, 60 at 4K); with several intra pictures in flight 32 each is better (4K 7.6 -> 8.6
    # Gpx/s). The 8K shard pass, one picture at a time, keeps the default.
    saved = os.environ.get("VVCR_INTRA_WG")
    os.environ.setdefault("VVCR_INTRA_WG", "32")
    ctx = N.Context(W, H, bit_depth=infos[0]["bit_depth"], ctu_log2=infos[0]["ctu_log2"], dpb_slots=per * a.segments,
                    device=int(os.environ.get("VVCR_DEVICE", local)))   # VVCR_DEVICE: rehearsal of N ranks on one GPU
    lanes_cfg = "%s lanes (%s intra) on %s hardware queues, %s k_intra workgroups" % (
        os.environ["VVCR_LANES"], os.environ["VVCR_INTRA_LANES"], os.environ.get("GPU_MAX_HW_QUEUES", "4"),
        os.environ["VVCR_INTRA_WG"])
    if saved is None:
        os.environ.pop("VVCR_INTRA_WG", None)

    if a.kernel_table_only:
        ctx.set_timing(False)
        groups, handles, slots = resident_handles(ctx, data, per)
        kern = kernel_table(ctx, groups, a.kernel_table_reps, a.kernel_table_sync)
        ok = check_slots(ctx, {slot: poc for poc, slot in slots}, meta)
        for h in handles:
            ctx.release(h)
        out = {"stream": a.stream, "reps": a.kernel_table_reps, "sync": a.kernel_table_sync, "bitexact_vs_reference": bool(ok),
               "mc_roofline": mc_roofline(kern, "median of %d synced steps" % a.kernel_table_reps),
               "kernels": {k: {"us_per_launch": round(v[1] / max(v[0], 1) * 1e3, 2), "launches_per_step": v[0],
                               "ms_per_step": round(v[1], 4), "ms_min_max": [round(v[3], 4), round(v[4], 4)],
                               "alg_MB_per_launch": round(v[2] / max(v[0], 1) / 1e6, 3), "pictures_per_step": v[5]}
                           for k, v in kern.items()}}
        if a.north_star_stream and a.north_star_stream != a.stream:
            out["north_star_mc"] = north_star_mc(ctx, a.north_star_stream, per, a.kernel_table_reps, a.kernel_table_sync)
        ctx.close()
        print(json.dumps(out))
        R.close()
        return

    # ---- headline: end to end from the bitstream (parse + derive + plan + upload + GPU in the timed region)
    ctx.set_timing(False)
    bitexact = output_yuv_md5(ctx, data, meta)      # one decode writing DecoderApp's output file: its MD5
    value, ms_step, host_ms, host_rusage, single, ok = e2e_legs(ctx, data, meta, per, a.segments, a.steps, a.warmup,
                                                                 a.single_steps, a.e2e_threads, R, px_seq, len(infos))
    bitexact = bitexact and ok

    # ---- resident: every picture planned and uploaded once, the steps only launch (GPU-side rate)
    resident = None
    kern = {}
    if a.resident_steps > 0:
        from vvc_amd import bitstream as B
        copies = []
        t_prep = time.perf_counter()
        for c in range(a.segments):
            seq = B.SequenceDecode(ctx, data, nslots=per, base=per * c, threads=8)
            _, handles = seq.run(keep_handles=True)
            copies.append((B.launch_groups(handles, seq.batch), [(inf["poc"], seq.slot[i]) for i, inf in enumerate(seq.info)]))
        ctx.sync()
        t_prep = (time.perf_counter() - t_prep) / a.segments
        res_ok = True
        nstep = [0]

        def run_step():
            for g in copies[nstep[0] % a.segments][0]:
                B.launch_group(ctx, g)
                if a.sync_pictures:
                    ctx.sync()
            nstep[0] += 1
        for _ in range(a.warmup):
            run_step()
        ctx.sync()
        R.barrier()
        r0 = time.perf_counter()
        for _ in range(a.resident_steps):
            run_step()
        ctx.sync()
        r1 = time.perf_counter()
        R.barrier()
        r_el = R.max_over_ranks(r1 - r0)
        # every copy launched back to back (as timed), then each copy's slots checked
        for groups, _ in copies:
            for g in groups:
                B.launch_group(ctx, g)
        ctx.sync()
        for _, slots in copies:
            res_ok = res_ok and check_slots(ctx, {slot: poc for poc, slot in slots}, meta)
        # serial view: one step at a time
        s0 = time.perf_counter()
        for _ in range(max(1, a.resident_steps // 2)):
            run_step()
            ctx.sync()
        s_el = (time.perf_counter() - s0) / max(1, a.resident_steps // 2)
        # per-kernel HIP events: the kernel table and roofline (kernel_table: one segment, a host sync after
        # every picture, the median step of --kernel-table-reps)
        kern.update(kernel_table(ctx, copies[nstep[0] % a.segments][0], a.kernel_table_reps, a.kernel_table_sync))
        for groups, _ in copies:
            for g in groups:
                for hnd in g:
                    ctx.release(hnd)
        bitexact = bitexact and res_ok
        resident = {"value": round(V.job_throughput(px_seq * a.resident_steps, r_el, R) / 1e6, 2), "unit": "Mpixels/s",
                    "steps": a.resident_steps, "ms_per_step": round(r_el / a.resident_steps * 1e3, 3),
                    "serial_ms_per_step": round(s_el * 1e3, 3),
                    "serial_value": round(px_seq / s_el / 1e6, 2),
                    "host_prepare_s_per_sequence": round(t_prep, 3), "bitexact_vs_reference": bool(res_ok),
                    "note": "GPU reconstruction + loop filters of pictures planned and uploaded beforehand "
                            "(descriptors and work lists resident in HBM), %d segments in flight; serial = one "
                            "step at a time" % a.segments}

    roof = None
    if kern:
        dom = max(kern, key=lambda k: kern[k][1])
        dl, dms, dalg = kern[dom][:3]
        per_launch_s = dms / 1e3 / max(dl, 1)
        achieved = dalg / max(dl, 1) / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
        traffic = None
        tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_traffic*.json")))
        for tf in reversed(tfs):   # the newest PMC summary taken on this workload
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("stream") == a.stream:
                traffic = tj.get("per_group_launch_bytes", {}).get(dom)
                break
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic,
                "us_per_launch": round(per_launch_s * 1e6, 2)}
    mc_roof = mc_roofline(kern, "MC interpolation kernels, HIP events, one segment, a sync after every picture, median of %d steps"
                          % a.kernel_table_reps)
    ns_mc = None
    if a.resident_steps > 0 and a.north_star_stream and a.north_star_stream != a.stream:
        ns_mc = north_star_mc(ctx, a.north_star_stream, per, a.kernel_table_reps, a.kernel_table_sync)
        bitexact = bitexact and (ns_mc is None or ns_mc["bitexact_vs_reference"])

    # ---- the north star's stream (4K RA QP32) end to end, with its own CPU baselines
    ns_e2e = None
    if a.north_star_steps > 0 and a.north_star_stream and a.north_star_stream != a.stream:
        ns_e2e = north_star_e2e(ctx, a, R, per)
        bitexact = bitexact and (ns_e2e is None or "error" in ns_e2e or ns_e2e["bitexact_vs_reference"])

    kind, qp = a.stream.split("_")[0], a.stream.split("_")[-1]
    desc = "%s %s" % ("random access" if kind.startswith("ra") else "all intra", qp.replace("q", "QP"))
    line = {
        "metric": "decode Mpixels/sec (CABAC on host), bit-exact YUV vs DecoderApp, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (VTM-7.3-encoded synthetic %dx%d %s stream)" % (W, H, desc),
        "config": {"workload": "%s: %dx%d %s, %d pictures (%d intra) per decode, %d decodes per step, reconstruction + "
                                   "DBK/SAO/ALF" % (a.stream, W, H, desc, len(infos), nI, a.segments),
                   "parallelism": "replicas%d" % world, "segments": a.segments, "lanes": lanes_cfg,
                   "host_threads": a.e2e_threads, "bitexact_vs_reference": bool(bitexact)},
        "value_scope": "end to end from the bitstream: NAL/header parsing, CABAC (host threads), motion derivation "
                       "with the GPU's DMVR feedback, host planning, upload, GPU reconstruction and loop filters, every "
                       "picture of every step; a step = %d independent decodes of the stream, all in flight" % a.segments,
        "host_ms_per_picture": host_ms,
        "host_rusage": host_rusage,
        "roofline": roof,
        "cpu_baseline": None,
        "single_stream": single,
        "resident": resident,
        # the GPU time the end-to-end run needs, as a fraction of its wall time: value / the GPU-only rate
        # of the same pictures (resident); the rest of the time the GPU waits for the host
        "gpu_busy_est": round(value / resident["value"], 3) if resident and resident["value"] > 0 else None,
        "mc_roofline": mc_roof,
        "north_star_mc": ns_mc,
        "north_star_e2e": ns_e2e,
        "kernels": {k: {"ms_per_step": round(v[1], 4), "ms_min_max": [round(v[3], 4), round(v[4], 4)], "launches_per_step": v[0],
                        "alg_GBps": round(v[2] / (v[1] / 1e3) / 1e9, 2) if v[1] > 0 else 0.0} for k, v in kern.items()},
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"] = cpu_baseline(os.path.join(ROOT, "tests", "golden", "streams", a.stream + ".bin"), px_seq)
        cb = line["cpu_baseline"]
        ca = line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(
            os.path.join(ROOT, "tests", "golden", "streams", a.stream + ".bin"), px_seq, a.e2e_threads)
        line.update(cpu_ratios(value, single, cb, ca, a.e2e_threads))
    ctx.close()
    if a.shard_steps > 0:
        # With N > 1 the shard leg is the only point-to-point traffic of the run (halo rows over RCCL): a
        # watchdog on every rank bounds it, so that a stuck exchange costs the shard object, never the line
        # (rank 0 prints it with the error; every rank then ends its own process)
        dog = None
        if world > 1 and a.shard_timeout > 0:
            import threading
            gate, state = threading.Lock(), {"done": False}

            def expire():
                gate.acquire()   # held until the process ends: the main thread's line can no longer print
                if state["done"]:
                    gate.release()
                    return
                if rank == 0:
                    line["shard"] = {"error": "no result within %d s (watchdog)" % a.shard_timeout}
                    print(json.dumps(line), flush=True)
                sys.stderr.flush()
                os._exit(0 if bitexact else 1)
            dog = threading.Timer(a.shard_timeout, expire)
            dog.daemon = True
            dog.start()
        try:
            line["shard"] = shard_bench(a, R)
        except Exception as e:   # reported, never silently dropped: the line above stays valid
            line["shard"] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
        if dog is not None:
            with gate:
                state["done"] = True
            dog.cancel()
    if rank == 0:
        print(json.dumps(line))
    R.close()
    if not bitexact:
        sys.exit("bench: output is not bit-exact to the reference decoder")


if __name__ == "__main__":
    main()
