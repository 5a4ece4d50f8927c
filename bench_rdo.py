"""BASELINE config 5 — the encoder's RDO inner loop on one MI355X: batched SAD +
Hadamard SATD (RdCost xGetSAD / xGetHADs) and DCT-2 forward transforms (TrQuant::xT) of every candidate
block of a 1080p picture, through libvvcr's C-ABI (vvcr_rd_run / vvcr_fwd_run on resident device buffers).

Candidate set (the same as `oracle/_ref/rdo_kat --bench`, the CPU baseline): every rectangle w x h with
w, h in {8, 16, 32, 64, 128}, on its own size grid inside each 128x128 CTU, clipped to the picture; SAD
and SATD for all of them, the forward DCT-2 for those with w, h <= 64. Synthetic 10-bit original and
prediction (uniform random original, prediction = original + noise in [-40, 40]).

  python bench_rdo.py [--steps K] [--warmup W] [--width 1920 --height 1080] [--no-cpu]

One JSON line: value = candidate samples per second (Msamples/s, each sample counted once per candidate
block it belongs to), roofline of the distortion kernel (algorithmic bytes: 2 B original + 2 B prediction
per sample, 8 B out per block), and the reference CPU baseline (one thread, x86 SIMD).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vvc_amd import native as N  # noqa: E402

PEAK_HBM_GBS = 8000.0


def blocks(W, H):
    out = []
    for cy in range(0, H, 128):
        for cx in range(0, W, 128):
            for w in (8, 16, 32, 64, 128):
                for h in (8, 16, 32, 64, 128):
                    for y in range(cy, cy + 128, h):
                        for x in range(cx, cx + 128, w):
                            if x + w <= W and y + h <= H:
                                out.append((x, y, w, h))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch

    W, H = a.width, a.height
    bl = blocks(W, H)
    rd = np.zeros(len(bl), N.RD_BLOCK)
    for i, (x, y, w, h) in enumerate(bl):
        rd[i] = (y * W + x, y * W + x, W, W, w, h)
    tr = [b for b in bl if b[2] <= 64 and b[3] <= 64]
    fw = np.zeros(len(tr), N.FWD_BLOCK)
    off = 0
    for i, (x, y, w, h) in enumerate(tr):
        fw[i] = (y * W + x, off, W, w, h, 0, 0, 0)
        off += w * h
    samples = float(sum(w * h for _, _, w, h in bl))
    tr_samples = float(off)

    rng = np.random.default_rng(5)
    org = rng.integers(0, 1024, (H, W)).astype(np.int16)
    cur = np.clip(org + rng.integers(-40, 41, (H, W)), 0, 1023).astype(np.int16)
    dev = torch.device("cuda", 0)
    d_org = torch.from_numpy(org).to(dev)
    d_cur = torch.from_numpy(cur).to(dev)
    d_res = (d_org - d_cur).contiguous()
    d_sad = torch.zeros(len(bl), dtype=torch.int32, device=dev)
    d_satd = torch.zeros(len(bl), dtype=torch.int32, device=dev)
    d_coef = torch.zeros(off, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    ctx = N.Context(W, H, dpb_slots=1)
    p_rd, p_fw = ctx.rd_plan(rd), ctx.fwd_plan(fw)

    def step():
        ctx.rd_run(p_rd, d_org.data_ptr(), d_cur.data_ptr(), d_sad.data_ptr(), d_satd.data_ptr())
        ctx.fwd_run(p_fw, d_res.data_ptr(), d_coef.data_ptr())

    # correctness spot check against the host-pointer path on a sample of blocks (same library, same kernels)
    step()
    ctx.sync()
    sub = rd[:: max(1, len(rd) // 500)]
    s_sad, s_satd = ctx.rd_dist(sub, org.ravel(), cur.ravel())
    idx = np.arange(0, len(rd), max(1, len(rd) // 500))[: len(sub)]
    consistent = bool(np.array_equal(d_sad.cpu().numpy()[idx].astype(np.uint32), s_sad) and
                      np.array_equal(d_satd.cpu().numpy()[idx].astype(np.uint32), s_satd))

    for _ in range(a.warmup):
        step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.sync()
    el = time.perf_counter() - t0
    # per-kernel-group times (each alone)
    t1 = time.perf_counter()
    for _ in range(a.steps):
        ctx.rd_run(p_rd, d_org.data_ptr(), d_cur.data_ptr(), d_sad.data_ptr(), d_satd.data_ptr())
    ctx.sync()
    rd_s = (time.perf_counter() - t1) / a.steps
    t2 = time.perf_counter()
    for _ in range(a.steps):
        ctx.fwd_run(p_fw, d_res.data_ptr(), d_coef.data_ptr())
    ctx.sync()
    fw_s = (time.perf_counter() - t2) / a.steps

    rd_bytes = samples * 4 + len(bl) * 8
    fw_bytes = tr_samples * (2 + 4)
    achieved = rd_bytes / rd_s / 1e9
    line = {
        "metric": "encoder RDO inner loop Msamples/s (SAD + Hadamard SATD + DCT-2 forward transform per candidate block)",
        "value": round(samples * a.steps / el / 1e6, 2),
        "unit": "Msamples/s",
        "n_gpus": 1,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True,
        "dtype": "int16",
        "data": "synthetic (uniform random 10-bit original, prediction = original + U[-40, 40])",
        "config": {"workload": "%dx%d picture, %d candidate blocks (8..128 rectangles on their grids per CTU), %d forward DCT-2"
                               % (W, H, len(bl), len(tr)), "consistent_with_host_path": consistent},
        "roofline": {"bound": "hbm", "kernel": "k_rd_tiles", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None},
        "kernels": {"rd_dist_ms": round(rd_s * 1e3, 4), "fwd_tr_ms": round(fw_s * 1e3, 4),
                    "fwd_tr_alg_GBps": round(fw_bytes / fw_s / 1e9, 2)},
    }
    kat = os.path.join(ROOT, "oracle", "_ref", "rdo_kat")
    if not a.no_cpu and os.path.exists(kat):
        r = subprocess.run([kat, "--bench", str(W), str(H), "10"], capture_output=True, text=True, timeout=120)
        cj = json.loads(r.stdout.strip().splitlines()[-1])
        line["cpu_baseline"] = {"value": cj["msamples_per_s"], "unit": "Msamples/s", "cores": 1, "kind": "reference",
                                "sample": "VTM-7.3 RdCost setDistParam/distFunc (x86 SIMD) + fastFwdTrans DCT-2, the same "
                                          "candidate set, %d passes in %.1f s" % (cj["passes"], cj["seconds"])}
    else:
        line["cpu_baseline"] = None
    ctx.rdo_release(p_rd)
    ctx.rdo_release(p_fw)
    ctx.close()
    print(json.dumps(line))


if __name__ == "__main__":
    main()
