"""Decode throughput of the MI355X reconstruction path (BASELINE.json configs[1]: 1080p random-access
QP32, 1 GPU): all pictures of the stream reconstructed by libvvcr in decoding order — residuals, motion
compensation (DMVR/BDOF/affine-PROF/GEO/CIIP), intra waves, deblocking, SAO, ALF/CC-ALF — with every
input (parsed descriptors, work lists, loop-filter parameters) resident in HBM when the timed region
starts (vvcr_prepare_picture once, vvcr_launch_picture per step). One step = one decode of the whole
sequence. The output of the first pass is checked bit-exact against the reference decoder's MD5s.
Steps cycle through --segments (default 4) copies of the sequence on disjoint DPB slots, as consecutive
intra-started segments of one long stream: the library runs each picture once its reference / slot
dependencies are met, so a segment's intra picture may overlap the previous segment's B pictures.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--stream ra1080_q32] [--segments 4] [--no-cpu]

Multi-GPU (torch.distributed.run, one process per GPU): the path has no intra-picture work split in
this round, so N ranks decode N independent replicas (weak scaling, no data-path collective); the
timing barrier and max-over-ranks use torch.distributed.
"""
import os

# Execution lanes (libvvcr reads VVCR_LANES / VVCR_INTRA_LANES at vvcr_create): 5 intra lanes + 4 B lanes,
# each on its own hardware queue, so that five intra-started segments and the B pictures of four others
# overlap; HIP's default is 4 hardware queues per process, so the bench asks for 12 before the runtime
# starts. Measured on 1080p with 12 segments in flight (lanes (intra lanes)): one sweep 8 (4) 11.5,
# 8 (5) 12.2, 9 (5) 12.3, 10 (5) 11.5, 10 (4) 10.8, 12 (6) 12.0 Gpx/s; interleaved A/B on one box, twice
# each: 8 (5) 10.5-10.7, 9 (5) 11.2, 10 (5) 10.6 Gpx/s. (Until late r02 the library clamped VVCR_LANES to 8:
# the "10 lanes" of earlier r02 lines were 8.)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 12:   # the box exports HIP's default of 4
    os.environ["GPU_MAX_HW_QUEUES"] = "12"
USER_LANES = "VVCR_LANES" in os.environ or "VVCR_INTRA_LANES" in os.environ
os.environ.setdefault("VVCR_LANES", "9")
os.environ.setdefault("VVCR_INTRA_LANES", "5")

import argparse
import hashlib
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch  # noqa: F401  (before any libvvcr context: torch's HIP runtime must load first)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vvc_amd import native as N  # noqa: E402
from vvc_amd import stream as S  # noqa: E402
from vvc_amd import decode as D  # noqa: E402
from vvc_amd import dist as V  # noqa: E402

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E peak (guides/MI355X_MICROARCH.md)


def cpu_baseline(stream_bin, pixels_per_run, min_seconds=10.0, max_runs=40):
    """VTM DecoderApp (the reference, built here from /root/reference by oracle/ref.mk) on the same
    bitstream, single-threaded, no output file; repeated until ~min_seconds of CPU work."""
    exe = os.path.join(ROOT, "oracle", "_ref", "DecoderApp")
    if not os.path.exists(exe):
        return None
    runs, total = 0, 0.0
    while total < min_seconds and runs < max_runs:
        t0 = time.perf_counter()
        r = subprocess.run([exe, "-b", stream_bin], capture_output=True, text=True)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            return None
        runs += 1
        total += dt
    return {"value": round(pixels_per_run * runs / total / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "reference",
            "sample": "VTM-7.3 DecoderApp (x86 SIMD, 1 thread) decoding %s.bin %d times (%.1f s), parse + reconstruction"
                      % (os.path.basename(stream_bin)[:-4], runs, total)}


def shard_bench(a, R):
    """BASELINE config 4: one tile-row stream decoded by all ranks together, each rank reconstructing and
    filtering its own rows (vvc_amd/shard.py) and exchanging only the loop-filter halo (24 pre-deblocking
    rows per edge) and the motion-reach rows of reference pictures with its neighbours over RCCL.
    Strong scaling: the whole job decodes every picture once per step. Checked bit-exact afterwards:
    rank 0 gathers every rank's rows of each slot's last picture and compares its MD5s."""
    from vvc_amd import shard as SH
    d = os.path.join(ROOT, "tests", "golden", a.shard_stream)
    if not os.path.isdir(d):
        return None
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    h0 = pics[0]["hdr"]
    W, H = h0["width"], h0["height"]
    slots = 8
    ctx = N.Context(W, H, bit_depth=h0["bitdepth_y"], ctu_log2=h0["ctu_log2"], dpb_slots=slots,
                    device=int(os.environ.get("VVCR_DEVICE", R.local)))
    t0 = time.perf_counter()
    rk = SH.ShardRank(ctx, pics, R.rank, R.world, slots)
    t_plan = time.perf_counter() - t0
    comm = SH.TorchComm(R.device) if R.world > 1 else None
    M = SH.plan_and_reach([rk], comm)
    ctx.set_timing(False)

    def step():
        for i in range(len(pics)):
            SH.decode_picture(rk, comm, i)
        ctx.sync()
    for _ in range(max(1, a.warmup)):
        step()
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(a.shard_steps):
        step()
    t1 = time.perf_counter()
    R.barrier()
    elapsed = R.max_over_ranks(t1 - t0)
    owner = {}
    for i, p in enumerate(pics):
        owner[rk.slots[i]] = p["hdr"]["poc"]
    ok = True
    for slot, poc in sorted(owner.items()):
        SH.gather_to_root(rk, comm, slot)
        if R.rank == 0:
            got = D.plane_md5s([ctx.read_plane(N.BUF_RECO, slot, c) for c in range(3)])
            ok = ok and got == meta["poc_plane_md5"][str(poc)]
    rk.release()
    ctx.close()
    px = W * H * len(pics) * a.shard_steps
    heights = [b - y for y, b in rk.rows]
    return {"value": round(px / elapsed / 1e6, 2), "unit": "Mpixels/s", "n_gpus": R.world, "scaling": "strong",
            "stream": a.shard_stream, "picture": "%dx%d" % (W, H), "pictures_per_step": len(pics), "steps": a.shard_steps,
            "ms_per_step": round(elapsed / a.shard_steps * 1e3, 3), "shard_rows": heights, "lf_halo_rows": SH.LF_HALO,
            "ref_halo_rows": M, "host_plan_s": round(t_plan, 3), "bitexact_vs_reference": bool(ok) if R.rank == 0 else None,
            "note": "tile-row shards, halo exchange over torch.distributed %s point to point" % (R.dist.get_backend() if R.dist else "-")}


def end_to_end(ctx, dec, pics, meta, per, a, copies=4):
    """Descriptors (host arrays) -> reconstructed pictures, host planning included: a pool of
    --e2e-threads threads validates and plans pictures (vvcr_picture_*, no GIL inside the library) and
    uploads them (vvcr_prepare_planned) while this thread launches them in decoding order as soon as each
    is ready; `copies` consecutive segments of the sequence. Every picture is planned from scratch.
    CABAC parsing is not included: the descriptors are the capture of the reference's parser."""
    import concurrent.futures as cf
    jobs = []
    for c in range(copies):
        alloc = S.SlotAllocator(pics, per, base=per * (c % a.segments))
        for i, p in enumerate(pics):
            slot = alloc.assign(i, p["hdr"]["poc"])
            jobs.append((p, slot, dict(alloc.slot_of)))

    def work(job):
        p, slot, slot_of = job
        pic = S.plan_picture(p, slot, slot_of, dpb_slots=per * a.segments)
        h = ctx.prepare_planned(pic)
        pic.close()
        return h

    ctx.sync()
    with cf.ThreadPoolExecutor(a.e2e_threads) as ex:
        t0 = time.perf_counter()
        futs = [ex.submit(work, j) for j in jobs]
        handles = []
        for f in futs:
            h = f.result()
            ctx.launch(h)
            handles.append(h)
        ctx.sync()
        t1 = time.perf_counter()
    ok = True
    owner = {}
    for (p, slot, _) in jobs[-len(pics):]:
        owner[slot] = p["hdr"]["poc"]
    for slot, poc in owner.items():
        ok = ok and D.plane_md5s(dec.read(slot)) == meta["poc_plane_md5"][str(poc)]
    for h in handles:
        ctx.release(h)
    px = pics[0]["hdr"]["width"] * pics[0]["hdr"]["height"] * len(jobs)
    return {"value": round(px / (t1 - t0) / 1e6, 2), "unit": "Mpixels/s", "threads": a.e2e_threads,
            "pictures": len(jobs), "ms_per_sequence": round((t1 - t0) / copies * 1e3, 2), "bitexact_vs_reference": ok,
            "note": "host planning (validation, work lists, intra dependency plan, deblocking edges) + upload + GPU, "
                    "from parsed descriptors; CABAC parsing excluded"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stream", default="ra1080_q32")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--segments", type=int, default=12, help="copies of the sequence the steps cycle through (<= 12)")
    ap.add_argument("--kernels-inflight", action="store_true",
                    help="diagnostics: take the kernel table from a pass with every segment in flight")
    ap.add_argument("--sync-pictures", action="store_true",
                    help="host sync after every picture (profiling: kernel durations without overlap)")
    ap.add_argument("--e2e-threads", type=int, default=12,
                    help="host planning threads of the end-to-end pass (0 = skip it)")
    ap.add_argument("--shard-stream", default="ra4320t_q32",
                    help="tile-row stream of the spatially sharded pass (BASELINE config 4: 8K, one shard per rank)")
    ap.add_argument("--shard-steps", type=int, default=3, help="timed steps of the sharded pass (0 = skip it)")
    a = ap.parse_args()

    R = V.Ranks()
    world, rank, local = R.world, R.rank, R.local

    d = os.path.join(ROOT, "tests", "golden", a.stream)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    h0 = pics[0]["hdr"]
    W, H = h0["width"], h0["height"]
    px_seq = W * H * len(pics)

    # ---- prepare every picture once (host planning + upload), decoding order. The sequence is prepared
    # --segments times over disjoint DPB slot ranges and the steps cycle through these copies: step k+1
    # then decodes its segment like the next intra-started segment of a longer stream would be decoded
    # (its intra picture references nothing, so it may start while step k's B pictures still run —
    # the library orders pictures only by their DPB-slot dependencies). --segments 1 serialises steps.
    per = min(12, 64 // a.segments)   # DPB slots per copy (64 in all)
    # k_intra workgroups of this context (VVCR_INTRA_WG, read at vvcr_create): the library's default sizes
    # one intra picture at a time (four wavefront diagonals' worth: 32 at 1080p, 60 at 4K); with five intra
    # pictures in flight 32 each is better (4K 7.6 -> 8.6 Gpx/s, 1080p unchanged). The 8K shard pass, one
    # picture at a time, keeps the default (32 there: 5.4 -> 4.4 Gpx/s).
    # At 4K an intra picture takes ~11 ms (5 at 1080p): 12 lanes, 7 of them intra, keep more of them in
    # flight (interleaved A/B, 4K QP32: 9.0 vs 8.6 Gpx/s; at 1080p 12 / 7 loses: 10.7 vs 12.2).
    saved = {k: os.environ.get(k) for k in ("VVCR_INTRA_WG", "VVCR_LANES", "VVCR_INTRA_LANES")}
    if saved["VVCR_INTRA_WG"] is None:
        os.environ["VVCR_INTRA_WG"] = "32"
    if not USER_LANES and W * H >= 3840 * 2160:
        os.environ["VVCR_LANES"], os.environ["VVCR_INTRA_LANES"] = "12", "7"
    dec = D.Decoder(pics, dpb_slots=per * a.segments,
                    device=int(os.environ.get("VVCR_DEVICE", local)))   # VVCR_DEVICE: rehearsal of N ranks on one GPU
    lanes_cfg = "%s lanes (%s intra), %s k_intra workgroups" % (os.environ["VVCR_LANES"], os.environ["VVCR_INTRA_LANES"],
                                                              os.environ["VVCR_INTRA_WG"])
    for k, v in saved.items():   # the shard pass's context takes the library / process defaults
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    ctx = dec.ctx
    copies = []
    t_prep = time.perf_counter()
    for c in range(a.segments):
        alloc = S.SlotAllocator(pics, per, base=per * c)
        handles, slots = [], []
        for i, p in enumerate(pics):
            slot = alloc.assign(i, p["hdr"]["poc"])
            ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
            S.submit(ctx, p)
            S.set_loop_filter_params(ctx, p)
            handles.append(ctx.prepare(N.STAGE_ALL))
            slots.append((p["hdr"]["poc"], slot))
        copies.append((handles, slots))
    t_prep = (time.perf_counter() - t_prep) / a.segments

    # ---- first pass: bit-exactness of every copy against the reference decoder (untimed, one picture at
    # a time: every picture's planes and the YUV file MD5)
    bitexact = True
    for handles, slots in copies:
        yuv = hashlib.md5()
        outs = {}
        for hnd, (poc, slot) in zip(handles, slots):
            ctx.launch(hnd)
            planes = dec.read(slot)
            outs[poc] = D.plane_md5s(planes), planes
        bitexact = bitexact and all(outs[int(k)][0] == v for k, v in meta["poc_plane_md5"].items())
        for poc in sorted(outs):
            for pl in outs[poc][1]:
                yuv.update(np.ascontiguousarray(pl).astype("<u2").tobytes())
        bitexact = bitexact and yuv.hexdigest() == meta["yuv_md5"]
        outs = None
    nstep = [0]

    def check_in_flight():
        """The timed configuration itself: every segment copy launched back to back with no host sync in
        between (all segments in flight on the lanes), then the last picture of every DPB slot of every
        copy checked against the reference MD5s."""
        for handles, _ in copies:
            for hnd in handles:
                ctx.launch(hnd)
        ctx.sync()
        ok = True
        for _, slots in copies:
            owner = {slot: poc for poc, slot in slots}
            for slot, poc in owner.items():
                ok = ok and D.plane_md5s(dec.read(slot)) == meta["poc_plane_md5"][str(poc)]
        return ok

    def run_step():
        for hnd in copies[nstep[0] % a.segments][0]:
            ctx.launch(hnd)
            if a.sync_pictures:
                ctx.sync()
        nstep[0] += 1

    ctx.set_timing(False)   # the throughput passes record no per-kernel events (marker packets)
    for _ in range(a.warmup):
        run_step()
    ctx.sync()

    R.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run_step()
    t_sub = time.perf_counter()   # host submission done (the library never blocks the host on the GPU)
    ctx.sync()
    t1 = time.perf_counter()
    R.barrier()
    elapsed = R.max_over_ranks(t1 - t0)

    # ---- the same steps one segment at a time (each step synchronised before the next starts): the
    # latency-bound view, reported beside value
    ctx.sync()
    R.barrier()
    t2 = time.perf_counter()
    for _ in range(a.steps):
        run_step()
        ctx.sync()
    t3 = time.perf_counter()
    R.barrier()
    elapsed_serial = R.max_over_ranks(t3 - t2)
    # the timed configuration (all segments in flight, no per-kernel events), checked bit-exact
    inflight_ok = check_in_flight()
    bitexact = bitexact and inflight_ok
    # one more (untimed) step with per-kernel HIP events, one segment in flight: the kernel table and roofline
    ctx.set_timing(True)
    if a.kernels_inflight:   # every segment in flight (as timed), all steps' kernel tables summed below
        for _ in range(a.segments):
            run_step()
    else:
        run_step()
    ctx.sync()
    e2e = end_to_end(ctx, dec, pics, meta, per, a) if (world == 1 and a.e2e_threads > 0) else None

    # ---- per-kernel timing of the last step (HIP events on the library stream)
    kern = {}
    last = copies[(nstep[0] - 1) % a.segments][0]
    if a.kernels_inflight:
        last = [h for c in copies for h in c[0]]
    for hnd in last:
        for name, launches, ms, alg in ctx.kernel_stats(hnd):
            k = kern.setdefault(name, [0, 0.0, 0.0])
            k[0] += launches
            k[1] += ms
            k[2] += alg
    dom = max(kern, key=lambda k: kern[k][1])
    dl, dms, dalg = kern[dom]
    per_launch_bytes = dalg / max(dl, 1)
    per_launch_s = dms / 1e3 / max(dl, 1)
    achieved = per_launch_bytes / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    # the north-star's MC-interpolation kernels (plain and affine): algorithmic bytes / HIP-event time
    mc_roof = {"peak": PEAK_HBM_GBS, "unit": "GB/s",
               "note": "MC interpolation kernels on this workload (one segment in flight); "
                       "4K figures: profiles/r02_mc_kernels.json"}
    for k in ("mc", "mc_affine"):
        v = kern.get(k, [0, 0.0, 0.0])
        g = v[2] / (v[1] / 1e3) / 1e9 if v[1] > 0 else 0.0
        mc_roof[k] = {"achieved": round(g, 2), "frac": round(g / PEAK_HBM_GBS, 4), "us_per_launch": round(v[1] / max(v[0], 1) * 1e3, 2)}

    traffic = None
    tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_traffic.json")))   # the newest round's
    tf = tfs[-1] if tfs else ""
    if tf and os.path.exists(tf):
        with open(tf) as f:
            tj = json.load(f)
        if tj.get("stream", "ra1080_q32") == a.stream:   # the PMC passes were taken on this workload
            traffic = tj.get("per_group_launch_bytes", {}).get(dom)   # profiles/: tools/pmc.sh + tools/pmc_summary.py

    ms_step = elapsed / a.steps * 1e3
    kind, qp = a.stream.split("_")[0], a.stream.split("_")[-1]
    desc = "%s %s" % ("random access" if kind.startswith("ra") else "all intra", qp.replace("q", "QP"))
    value = V.job_throughput(px_seq * a.steps, elapsed, R) / 1e6
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
        "data": "synthetic (VTM-7.3-encoded synthetic %dx%d %s stream, parsed descriptors resident in HBM)" % (W, H, desc),
        "config": {"workload": "%s: %dx%d %s, %d pictures, reconstruction + DBK/SAO/ALF" % (a.stream, W, H, desc, len(pics)),
                   "parallelism": "replicas%d" % world, "segments_in_flight": a.segments, "lanes": lanes_cfg,
                   "bitexact_vs_reference": bool(bitexact)},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic},
        "kernels": {k: {"ms_per_step": round(v[1], 4), "launches_per_step": v[0],
                        "alg_GBps": round(v[2] / (v[1] / 1e3) / 1e9, 2) if v[1] > 0 else 0.0} for k, v in kern.items()},
        "host_submit_ms_per_step": round((t_sub - t0) / a.steps * 1e3, 3),
        "serial": {"value": round(V.job_throughput(px_seq * a.steps, elapsed_serial, R) / 1e6, 2),
                   "ms_per_step": round(elapsed_serial / a.steps * 1e3, 3),
                   "note": "one segment in flight (sync after every step)"},
        "mc_roofline": mc_roof,
        "host_prepare_s": round(t_prep, 3),
        "value_scope": "GPU reconstruction + loop filters of pre-planned pictures (descriptors and work lists resident "
                       "in HBM); host planning and CABAC parsing excluded - see end_to_end",
        "end_to_end": e2e,
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"] = cpu_baseline(os.path.join(ROOT, "tests", "golden", "streams", a.stream + ".bin"), px_seq)
    else:
        line["cpu_baseline"] = None
    for handles, _ in copies:
        for hnd in handles:
            ctx.release(hnd)
    dec.close()
    if a.shard_steps > 0:
        try:
            line["shard"] = shard_bench(a, R)
        except Exception as e:   # reported, never silently dropped: the replica line above stays valid
            line["shard"] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
    if rank == 0:
        print(json.dumps(line))
    R.close()
    if not bitexact:
        sys.exit("bench: output is not bit-exact to the reference decoder")


if __name__ == "__main__":
    main()
