"""Spatial sharding of a picture across GPUs: one rank per run of whole tile rows.

A stream coded with tile rows (and loop filtering across them) lets every rank reconstruct its own rows
without the others: intra prediction, CCLM, CIIP and LMCS never read across a tile edge (vvcr.h tiles;
CodingStructure::getCURestricted, CodingStructure.cpp:1519). Two things do cross shard edges, and they
are the only data a rank exchanges with its neighbours, point to point (RCCL send / recv over xGMI):

1. the loop filters (DecLib::executeLoopFilters, DecLib.cpp:560: deblocking LoopFilter.cpp:145, SAO
   SampleAdaptiveOffset.cpp:618, ALF AdaptiveLoopFilter.cpp:393) filter across tile edges: after
   reconstruction each rank sends the VVCR_LF_HALO (24) pre-deblocking luma rows (12 chroma) next to
   each edge to the neighbour, which rebuilds the deblocked / SAO samples its own rows' filters read;
2. motion compensation may read a reference picture anywhere (VTM 7.3 has no subpicture MC clamp,
   SURVEY.md finding 3): after its loop filters a rank sends the final rows within the sequence's
   motion reach M of each edge to the neighbour (M from the planned motion vectors, all-reduced once);
   if M exceeds a neighbour's height every rank sends its rows to every other one instead.

Shard rows are balanced over the tile rows. The transport is an argument: TorchComm (torch.distributed
point-to-point: nccl = RCCL on ROCm with device buffers, or gloo with host buffers) or LocalComm (ranks
emulated inside one process, each with its own context, e.g. on a one-GPU box).
"""
import numpy as np
# torch before any libvvcr context: torch's HIP runtime must be the process's first (a HIP runtime loaded
# after libvvcr initialised the system one sees no GPU)
import torch  # noqa: F401

from . import native as N
from . import stream as S

LF_HALO = 24
STAGES_RECON = N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA | N.STAGE_LMCS_INV
STAGES_LF = N.STAGE_DBK | N.STAGE_SAO | N.STAGE_ALF


def shard_rows(p, world):
    """[(y0, y1)] luma rows per rank: contiguous runs of whole tile rows, balanced by CTU rows."""
    h = p["hdr"]
    ctu, H = 1 << h["ctu_log2"], h["height"]
    bd = [int(v) for v in p["tile_row_bd"]] if "tile_row_bd" in p else [0, (H + ctu - 1) // ctu]
    ntile = len(bd) - 1
    if world > ntile:
        raise ValueError("%d ranks but only %d tile rows" % (world, ntile))
    total = bd[-1]
    cuts = [0]
    for r in range(1, world):   # the tile-row boundary nearest the ideal cut, leaving a tile row per later rank
        ideal = total * r / world
        lo, hi = cuts[-1] + 1, ntile - (world - r)
        cuts.append(min(range(lo, hi + 1), key=lambda k: (abs(bd[k] - ideal), k)))
    cuts.append(ntile)
    return [(bd[cuts[r]] * ctu, min(H, bd[cuts[r + 1]] * ctu)) for r in range(world)]


def referenced_later(pics):
    """decode index -> True if a later picture references it (only those need the reference halo)"""
    used = set()
    out = [False] * len(pics)
    for i in range(len(pics) - 1, -1, -1):
        out[i] = pics[i]["hdr"]["poc"] in used
        p = pics[i]
        for l in range(2):
            for r in range(p["hdr"]["num_ref_l%d" % l]):
                used.add(int(p["ref_poc"][l][r]))
    return out


class ShardGeom:
    """A rank's rows and its exchange lists (no device: the CPU tests drive the exchanges with it)."""

    def __init__(self, ctx, rank, rows, M=0):
        self.ctx, self.rank, self.rows, self.world = ctx, rank, rows, len(rows)
        self.y0, self.y1 = rows[rank]
        self.M = M

    def set_reach(self, M):
        self.M = int(-(-M // 8) * 8)   # rounded up to 8 rows

    # ---- exchange lists: (peer, first luma row, rows); sends are own rows, receives land next to them
    def lf_halo(self):
        sends, recvs = [], []
        for peer, (a, b) in enumerate(self.rows):
            if peer == self.rank - 1:
                n = min(LF_HALO, self.y1 - self.y0, b - a)
                sends.append((peer, self.y0, n)); recvs.append((peer, self.y0 - n, n))
            elif peer == self.rank + 1:
                n = min(LF_HALO, self.y1 - self.y0, b - a)
                sends.append((peer, self.y1 - n, n)); recvs.append((peer, self.y1, n))
        return sends, recvs

    def ref_halo(self):
        """final rows of a reference picture: the motion reach around each edge, or everything (all-gather)"""
        M = self.M
        heights = [b - a for a, b in self.rows]
        if M <= 0:
            return [], []
        sends, recvs = [], []
        if M <= min(heights):
            for peer, (a, b) in enumerate(self.rows):
                if peer == self.rank - 1:
                    sends.append((peer, self.y0, M)); recvs.append((peer, b - M, M))
                elif peer == self.rank + 1:
                    sends.append((peer, self.y1 - M, M)); recvs.append((peer, a, M))
        else:
            for peer, (a, b) in enumerate(self.rows):
                if peer != self.rank:
                    sends.append((peer, self.y0, self.y1 - self.y0)); recvs.append((peer, a, b - a))
        return sends, recvs


class ShardRank(ShardGeom):
    """One rank's part of a sharded decode: its context, rows, planned pictures and exchange lists."""

    def __init__(self, ctx, pics, rank, world, dpb_slots, rows=None):
        super().__init__(ctx, rank, rows or shard_rows(pics[0], world))
        self.pics = pics
        self.H = pics[0]["hdr"]["height"]
        self.alloc = S.SlotAllocator(pics, dpb_slots)
        self.slots, self.h_recon, self.h_lf, self.reach = [], [], [], 0
        for i, p in enumerate(pics):
            slot = self.alloc.assign(i, p["hdr"]["poc"])
            pp = S.pic_params(p, slot, self.alloc.slot_of)
            pp.shard_y0, pp.shard_y1 = self.y0, self.y1
            pic = S.plan_picture_pp(p, pp, dpb_slots=dpb_slots, stages=STAGES_RECON)
            c = pic.work_counts()
            if c["ref_y1"] > c["ref_y0"]:
                self.reach = max(self.reach, self.y0 - c["ref_y0"], c["ref_y1"] - self.y1)
            self.h_recon.append(ctx.prepare_planned(pic))
            pic.close()
            pic = S.plan_picture_pp(p, pp, dpb_slots=dpb_slots, stages=STAGES_LF)
            self.h_lf.append(ctx.prepare_planned(pic))
            pic.close()
            self.slots.append(slot)
        self.ref_later = referenced_later(pics)

    def release(self):
        for h in self.h_recon + self.h_lf:
            self.ctx.release(h)


def plan_and_reach(ranks, comm=None):
    """the sequence's motion reach: max over ranks (all-reduce when the ranks are in other processes)"""
    M = max(r.reach for r in ranks)
    if comm is not None:
        M = comm.max_int(M)
    for r in ranks:
        r.set_reach(M)
    return ranks[0].M


def exchange(rk, comm, lists, slot):
    """export the sends, swap through comm, import the receives (rows of one DPB slot)"""
    sends, recvs = lists
    out = []
    for peer, y0, n in sends:
        buf = comm.buffer(rk, rk.ctx.rows_bytes(n))
        rk.ctx.export_rows(slot, y0, n, comm.dev_ptr(buf))
        out.append((peer, buf))
    inc = [(peer, comm.buffer(rk, rk.ctx.rows_bytes(n), recv=True)) for peer, y0, n in recvs]
    comm.swap(rk, out, inc)
    for (peer, y0, n), (_, buf) in zip(recvs, inc):
        rk.ctx.import_rows(slot, y0, n, comm.dev_ptr(buf, staged=True))


def decode_picture(rk, comm, i):
    """one picture on one rank (ranks in other processes run the same steps at the same time)"""
    rk.ctx.launch(rk.h_recon[i])
    if rk.world > 1:
        exchange(rk, comm, rk.lf_halo(), rk.slots[i])
    rk.ctx.launch(rk.h_lf[i])
    if rk.world > 1 and rk.ref_later[i]:
        exchange(rk, comm, rk.ref_halo(), rk.slots[i])


def gather_to_root(rk, comm, slot):
    """every rank's own rows of a DPB slot into rank 0's slot (rank 0 then holds the whole picture)"""
    if rk.world == 1:
        return
    if rk.rank == 0:
        recvs = [(peer, a, b - a) for peer, (a, b) in enumerate(rk.rows) if peer]
        exchange(rk, comm, ([], recvs), slot)
    else:
        exchange(rk, comm, ([(0, rk.y0, rk.y1 - rk.y0)], []), slot)


# ------------------------------------------------------------------------------------------------
# transports
# ------------------------------------------------------------------------------------------------
class TorchComm:
    """torch.distributed point-to-point between neighbouring ranks. nccl (RCCL on ROCm): the row buffers
    are device tensors handed to batch_isend_irecv directly. gloo: host tensors, staged through a device
    buffer on each side."""

    def __init__(self, device, host_rows=False):
        """host_rows: the contexts take host pointers (the CPU tests' stand-in context): no staging"""
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.device = device
        self.gpu = dist.get_backend() == "nccl"
        self.host_rows = host_rows
        self._stage = {}

    def buffer(self, rk, nbytes, recv=False):
        t = self.torch
        return t.empty(nbytes, dtype=t.uint8, device=self.device if self.gpu else "cpu")

    def dev_ptr(self, buf, staged=False):
        if self.gpu or self.host_rows:
            return buf.data_ptr()
        # gloo: host tensor; stage through a device tensor (export writes it, import reads it)
        t = self.torch
        key = id(buf)
        d = self._stage.get(key)
        if d is None or d.numel() != buf.numel():
            d = t.empty(buf.numel(), dtype=t.uint8, device="cuda")   # the context's rows live on the GPU
            self._stage[key] = d
        if staged:
            d.copy_(buf)
            t.cuda.synchronize()
        return d.data_ptr()

    def swap(self, rk, sends, recvs):
        t, dist = self.torch, self.dist
        if not self.gpu and not self.host_rows:
            for peer, buf in sends:   # device -> host for the exported rows
                buf.copy_(self._stage[id(buf)])
        ops = [dist.P2POp(dist.isend, buf, peer) for peer, buf in sends] + [dist.P2POp(dist.irecv, buf, peer) for peer, buf in recvs]
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        if self.gpu:
            t.cuda.current_stream().synchronize()
        self._stage.clear() if len(self._stage) > 64 else None

    def max_int(self, v):
        t = self.torch
        x = t.tensor([v], dtype=t.int64, device=self.device if self.gpu else "cpu")
        self.dist.all_reduce(x, op=self.dist.ReduceOp.MAX)
        return int(x.item())


class LocalComm:
    """Ranks emulated in one process (one context each, possibly on one GPU): decode_local drives all
    ranks through a picture phase by phase, the rows passing through a mailbox of device buffers."""

    def __init__(self, device="cuda"):
        import torch
        self.torch = torch
        self.device = device
        self.box = {}

    def buffer(self, rk, nbytes, recv=False):
        return self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.device)

    def max_int(self, v):
        return v


def decode_local(ranks, comm, i):
    """picture i on every emulated rank: recon, LF-halo swap, loop filters, reference-halo swap"""
    def phase(lists_of):
        staged = []
        for rk in ranks:   # export + post
            sends, recvs = lists_of(rk)
            out = []
            for peer, y0, n in sends:
                buf = comm.buffer(rk, rk.ctx.rows_bytes(n))
                rk.ctx.export_rows(rk.slots[i], y0, n, buf.data_ptr())
                out.append((peer, buf))
            for peer, buf in out:
                comm.box[(rk.rank, peer)] = buf
            staged.append((rk, recvs))
        for rk, recvs in staged:   # collect + import
            for peer, y0, n in recvs:
                rk.ctx.import_rows(rk.slots[i], y0, n, comm.box.pop((peer, rk.rank)).data_ptr())
    for rk in ranks:
        rk.ctx.launch(rk.h_recon[i])
    phase(lambda rk: rk.lf_halo())
    for rk in ranks:
        rk.ctx.launch(rk.h_lf[i])
    if ranks[0].ref_later[i]:
        phase(lambda rk: rk.ref_halo())


def assemble(ranks, i):
    """the full picture of decode index i from every rank's own rows: [Y, Cb, Cr] numpy planes"""
    out = None
    for rk in ranks:
        planes = [rk.ctx.read_plane(N.BUF_RECO, rk.slots[i], c) for c in range(3)]
        if out is None:
            out = [np.zeros_like(pl) for pl in planes]
        out[0][rk.y0:rk.y1] = planes[0][rk.y0:rk.y1]
        for c in (1, 2):
            out[c][rk.y0 // 2:rk.y1 // 2] = planes[c][rk.y0 // 2:rk.y1 // 2]
    return out
