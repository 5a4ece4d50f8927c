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
# rows a rank's CABAC pass covers beyond its own (vvcp_set_parse_rows): the deblocking plan of the halo
# (VVCR_LF_HALO rows) and the CUs on the far side of its outermost edges
PARSE_MARGIN = LF_HALO + 8


def parse_rows(y0, y1, ctu):
    """luma rows a rank with rows [y0, y1) parses: the deblocking planner takes every edge of the CUs that
    reach VVCR_LF_HALO rows into the halo, so above it needs the CTU row over the topmost of them too"""
    return y0 - PARSE_MARGIN - ctu, y1 + PARSE_MARGIN
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


# ------------------------------------------------------------------------------------------------
# the product path: shards decoded from the bitstream
# ------------------------------------------------------------------------------------------------
def stream_shard_rows(pp, height, ctu_log2, world):
    """shard_rows from the parsed picture parameters (tile rows of vvcr_pic_params)"""
    nt = int(pp.num_tile_rows)
    bd = [int(pp.tile_row_bd[k]) for k in range(nt + 1)] if nt > 0 else None
    p = {"hdr": {"ctu_log2": ctu_log2, "height": height}}
    if bd:
        p["tile_row_bd"] = bd
    return shard_rows(p, world)


class StreamShardRank(ShardGeom):
    """One rank of a spatially sharded decode FROM THE BITSTREAM (BASELINE config 4 end to end): every
    rank runs the host parser (vvcp: headers, CABAC, motion derivation) and reconstructs and filters its
    own tile rows only (vvcp_plan_picture_rows -> vvcr_pic_params::shard_y0 / shard_y1).

    Per picture, in decoding order (DecApp::decode, DecApp.cpp:118-200):
      1. the CABAC pass of the tiles around its rows only (vvcp_set_parse_rows: the tile rows that hold
         its shard and PARSE_MARGIN rows around it; each tile's substreams on a thread of their own,
         DecSlice.cpp:106-114). HMVP resets per tile row (DecSlice.cpp:186-191), spatial candidates stay
         inside the tile and temporal ones inside the CTU row, so the motion of those rows is exact;
      2. the refined motion of its pending references: each rank's GPU refined the DMVR sub-blocks of its
         own rows; the lists are all-gathered and each rank takes its parsed PUs' run of them (the tile
         rows are whole and in decoding order: the upper neighbour's last rows, its own, the lower
         neighbour's first, vvcp_dmvr_split), so every rank records the exact refined motion field
         (CS::setRefinedMotionField, UnitTools.cpp:68) of its rows and the rows around them;
      3. motion derivation, planning of the shard, upload;
      4. the reference halo: the motion reach of the picture's MC jobs beyond the shard (max over the
         ranks, all-reduced per picture) in each reference picture, exchanged point to point with the
         neighbours when that reference has not yet been exchanged as deep (VTM 7.3 has no tile MC clamp);
      5. reconstruction stages, the loop-filter halo swap, the loop-filter stages.
    """

    def __init__(self, ctx, data, rank, world, dpb_slots, rows=None, parse_threads=4):
        import ctypes as C
        from . import bitstream as B
        from . import parser as PZ
        self.ps = PZ.Stream(data)
        self.n = n = len(self.ps)
        inf0 = self.ps.info(0)
        self.W, self.H = inf0["width"], inf0["height"]
        self.sp = N.SeqParams(self.W, self.H, 1, inf0["bit_depth"], inf0["ctu_log2"], dpb_slots, 0)
        rows = rows or stream_shard_rows(self.ps.pic_params(0), self.H, inf0["ctu_log2"], world)
        super().__init__(ctx, rank, rows)
        self.partial = world > 1
        if self.partial:
            self.ps.set_parse_rows(*parse_rows(self.y0, self.y1, 1 << inf0["ctu_log2"]))
        L = B._bind(N.lib())
        L.vvcp_plan_picture_rows.argtypes = [C.c_void_p, C.c_int32, C.POINTER(N.SeqParams), C.c_int32, C.c_void_p,
                                             C.c_uint32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
        self.L, self.C = L, C
        slots = (C.c_int32 * n)()
        if L.vvcp_decode_plan(self.ps.h, 0, dpb_slots, slots, None) < 0:
            raise RuntimeError("vvcp_decode_plan: %s" % L.vvcp_last_error().decode())
        self.slots = list(slots)
        plan = B.Plan(self.ps, dpb_slots)
        self.info = plan.info
        # decode index of every reference (the latest earlier picture of that POC in the same CVS)
        self.refs = []
        for i in range(n):
            r = []
            for l in range(2):
                for poc in plan.refs[i][l]:
                    j = next(k for k in range(i - 1, -1, -1) if self.info[k]["poc"] == poc and plan.cvs[k] == plan.cvs[i])
                    if j not in r:
                        r.append(j)
            self.refs.append(r)
        later = [False] * n
        for i in range(n):
            for j in self.refs[i]:
                later[j] = True
        self.ref_later = later
        self.handle = [None] * n
        self.ndmvr = [0] * n
        self.refined = [False] * n
        self.depth = {}        # DPB slot -> reference-halo rows exchanged for its current picture
        self.reach = 0         # largest reach seen (diagnostics)
        # the CABAC passes run ahead on parser threads (a picture's pass depends on no other picture;
        # ctypes releases the GIL inside the library)
        import concurrent.futures as cf
        self.pool = cf.ThreadPoolExecutor(max(1, parse_threads))
        self.parsed = [self.pool.submit(self.ps.parse, i) for i in range(n)]

    # ---- phases of picture i (a driver runs them on every rank: decode_stream_picture)
    def parse(self, i):
        self.parsed[i].result()

    def pending(self, i):
        """references of i whose motion is not refined yet (their deltas must be all-gathered first)"""
        return [j for j in self.refs[i] if not self.refined[j]]

    def local_deltas(self, j):
        return self.ctx.picture_dmvr_deltas(self.handle[j], self.ndmvr[j])

    def refine(self, j, parts):
        """parts: every rank's delta list of picture j (rows of its own shard), in rank order"""
        parts = [np.asarray(p, np.int32).reshape(-1, 2) for p in parts]
        if self.partial:
            # the parsed PUs above the shard are the last `a` of the ranks above (whole tile rows, decoding
            # order), those below the first `b` of the ranks below
            a, o, b = self.ps.dmvr_split(j, self.y0, self.y1)
            r = self.rank
            up = np.concatenate(parts[:r]) if r else np.zeros((0, 2), np.int32)
            down = np.concatenate(parts[r + 1:]) if r + 1 < len(parts) else np.zeros((0, 2), np.int32)
            if len(parts[r]) != o or len(up) < a or len(down) < b:
                raise RuntimeError("picture %d: DMVR delta lists do not match the parsed rows" % j)
            parts = [up[len(up) - a:], parts[r], down[:b]]
        d = np.concatenate(parts) if parts else np.zeros((0, 2), np.int32)
        self.ps.refine(j, d)
        self.refined[j] = True

    def plan(self, i):
        """derive and plan the shard of picture i; returns its reach (rows read beyond the shard)"""
        C = self.C
        self.ps.derive(i)
        pp = self.ps.pic_params(i)
        rs = (C.c_int32 * (2 * 16))()
        for l in range(2):
            for r in range(pp.num_ref[l]):
                poc = int(pp.ref_poc[l][r])
                j = next(k for k in self.refs[i] if self.info[k]["poc"] == poc)
                rs[l * 16 + r] = self.slots[j]
        h = C.c_void_p()
        rc = self.L.vvcp_plan_picture_rows(self.ps.h, i, C.byref(self.sp), self.slots[i], rs, N.STAGE_ALL, self.y0, self.y1,
                                           C.byref(h))
        if rc != 0:
            raise RuntimeError("picture %d plan: %s" % (i, self.L.vvcp_last_error().decode()))
        pic = N.Picture.wrap(h)
        c = pic.work_counts()
        self.ndmvr[i] = c["dmvr"]
        reach = max(0, self.y0 - c["ref_y0"], c["ref_y1"] - self.y1) if c["ref_y1"] > c["ref_y0"] else 0
        if self.handle[i] is not None:
            self.ctx.release(self.handle[i])
        self.handle[i] = self.ctx.prepare_planned(pic)
        pic.close()
        self.reach = max(self.reach, reach)
        return reach

    def ref_lists(self, i, M):
        """(slot, (sends, recvs)) reference-halo exchanges picture i needs at reach M (rows rounded to 8)"""
        M = int(-(-M // 8) * 8)
        out = []
        if self.world == 1 or M <= 0:
            return out
        for j in self.refs[i]:
            s = self.slots[j]
            if self.depth.get(s, 0) >= M:
                continue
            self.depth[s] = M
            self.M = M
            out.append((s, self.ref_halo()))
        return out

    def launch_recon(self, i):
        self.depth[self.slots[i]] = 0   # the slot's new picture: no rows exchanged yet
        self.ctx.launch_stages(self.handle[i], STAGES_RECON)

    def launch_lf(self, i):
        self.ctx.launch_stages(self.handle[i], STAGES_LF)
        if not self.ref_later[i]:
            self.refined[i] = True   # nobody reads its motion
        # handles of pictures well behind whose deltas were consumed (a release waits for the picture)
        for k in range(i - 8):
            if self.handle[k] is not None and self.refined[k]:
                self.ctx.release(self.handle[k])
                self.handle[k] = None

    def release(self):
        for f in self.parsed:
            f.cancel()
        self.pool.shutdown(wait=True)
        for k in range(self.n):
            if self.handle[k] is not None:
                self.ctx.release(self.handle[k])
                self.handle[k] = None
        self.ps.close()


def decode_stream_picture(rk, comm, i):
    """picture i on one rank of a torch.distributed job (the other ranks run the same calls)"""
    rk.parse(i)
    for j in rk.pending(i):
        mine = rk.local_deltas(j)
        rk.refine(j, comm.all_gather_rows(mine) if rk.world > 1 else [mine])
    reach = rk.plan(i)
    M = comm.max_int(reach) if rk.world > 1 else 0
    for slot, lists in rk.ref_lists(i, M):
        exchange(rk, comm, lists, slot)
    rk.launch_recon(i)
    if rk.world > 1:
        exchange(rk, comm, rk.lf_halo(), rk.slots[i])
    rk.launch_lf(i)


def decode_stream_local(ranks, comm, i):
    """picture i on every rank emulated in one process (LocalComm): the same phases, all ranks at a time"""
    for rk in ranks:
        rk.parse(i)
    for j in ranks[0].pending(i):
        parts = [rk.local_deltas(j) for rk in ranks]
        for rk in ranks:
            rk.refine(j, parts)
    M = max(rk.plan(i) for rk in ranks)

    def phase(lists_of, slot_of):
        staged = []
        st = comm.stream_handle() if comm.ordered else None
        for rk in ranks:
            for slot, (sends, recvs) in lists_of(rk):
                for peer, y0, n in sends:
                    buf = comm.buffer(rk, rk.ctx.rows_bytes(n))
                    if st is not None:
                        rk.ctx.export_rows_async(slot, y0, n, buf.data_ptr(), st)
                    else:
                        rk.ctx.export_rows(slot, y0, n, buf.data_ptr())
                    comm.box[(rk.rank, peer, slot)] = buf
                staged.append((rk, slot, recvs))
        for rk, slot, recvs in staged:
            for peer, y0, n in recvs:
                buf = comm.box.pop((peer, rk.rank, slot))
                if st is not None:
                    rk.ctx.import_rows_async(slot, y0, n, buf.data_ptr(), st)
                else:
                    rk.ctx.import_rows(slot, y0, n, buf.data_ptr())
    if len(ranks) > 1:
        phase(lambda rk: rk.ref_lists(i, M), None)
    for rk in ranks:
        rk.launch_recon(i)
    if len(ranks) > 1:
        phase(lambda rk: [(rk.slots[i], rk.lf_halo())], None)
    for rk in ranks:
        rk.launch_lf(i)


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
    if getattr(comm, "ordered", False):
        # RCCL: exports, the point-to-point swap and the imports all on the comm's stream, ordered on the
        # device by events against the library's lanes (vvcr_*_rows_async): no host synchronisation
        st = comm.stream_handle()
        out = []
        for peer, y0, n in sends:
            buf = comm.buffer(rk, rk.ctx.rows_bytes(n))
            rk.ctx.export_rows_async(slot, y0, n, buf.data_ptr(), st)
            out.append((peer, buf))
        inc = [(peer, comm.buffer(rk, rk.ctx.rows_bytes(n), recv=True)) for peer, y0, n in recvs]
        comm.swap(rk, out, inc)
        for (peer, y0, n), (_, buf) in zip(recvs, inc):
            rk.ctx.import_rows_async(slot, y0, n, buf.data_ptr(), st)
        return
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
        # nccl: the halo buffers, the library's row copies and the collectives share one stream of ours
        # (exchange: stream-ordered, no host synchronisation)
        self.ordered = self.gpu and not host_rows
        self.stream = torch.cuda.Stream(device=device) if self.ordered else None

    def stream_handle(self):
        return self.stream.cuda_stream

    def buffer(self, rk, nbytes, recv=False):
        t = self.torch
        if self.ordered:
            with t.cuda.stream(self.stream):   # allocated for (and reused in order on) the exchange stream
                return t.empty(nbytes, dtype=t.uint8, device=self.device)
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
        if self.ordered:
            # the work's wait() makes the current stream (ours) wait for RCCL's: the imports that follow on
            # it see the received rows; the host goes on
            with t.cuda.stream(self.stream):
                if ops:
                    for r in dist.batch_isend_irecv(ops):
                        r.wait()
            return
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

    def all_gather_rows(self, a):
        """every rank's int32 array (rows of 2), in rank order: counts first, then one padded all-gather"""
        t, dist = self.torch, self.dist
        dev = self.device if self.gpu else "cpu"
        a = np.ascontiguousarray(a, np.int32).reshape(-1)
        world = dist.get_world_size()
        n = t.tensor([a.size], dtype=t.int64, device=dev)
        ns = [t.zeros(1, dtype=t.int64, device=dev) for _ in range(world)]
        dist.all_gather(ns, n)
        ns = [int(x.item()) for x in ns]
        m = max(max(ns), 1)
        x = t.zeros(m, dtype=t.int32, device=dev)
        if a.size:
            x[:a.size] = t.from_numpy(a).to(dev)
        outs = [t.zeros(m, dtype=t.int32, device=dev) for _ in range(world)]
        dist.all_gather(outs, x)
        return [o[:k].cpu().numpy().reshape(-1, 2) for o, k in zip(outs, ns)]


class LocalComm:
    """Ranks emulated in one process (one context each, possibly on one GPU): decode_local drives all
    ranks through a picture phase by phase, the rows passing through a mailbox of device buffers."""

    def __init__(self, device="cuda", ordered=False):
        """ordered: the row copies go on one stream of ours without host synchronisation, as TorchComm's
        RCCL path does (vvcr_export_rows_async / vvcr_import_rows_async)"""
        import torch
        self.torch = torch
        self.device = device
        self.box = {}
        self.ordered = ordered
        self.stream = torch.cuda.Stream(device=device) if ordered else None

    def stream_handle(self):
        return self.stream.cuda_stream

    def buffer(self, rk, nbytes, recv=False):
        if self.ordered:
            with self.torch.cuda.stream(self.stream):
                return self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.device)
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
