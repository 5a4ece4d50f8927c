"""Bitstream-to-pictures driver: the decode loop of DecoderApp (DecApp::decode, DecApp.cpp:118-200 ->
DecLib::decode / executeLoopFilters, DecLib.cpp) on the MI355X path, from an Annex-B VVC bitstream.

Per picture, in decoding order:
  1. CABAC parse (vvcp_parse_picture) — independent of every other picture, so all pictures are parsed
     ahead on a thread pool (the library releases the GIL);
  2. motion derivation (vvcp_derive_motion) — needs the refined motion of the collocated picture, i.e.
     that picture's DMVR deltas from the GPU (vvcr_picture_dmvr_deltas waits for its inter stage only);
  3. native planning from the parser's state (vvcp_plan_picture -> vvcr_picture_*), upload
     (vvcr_prepare_planned) and launch on the context's execution lanes.
The DPB (slots) and output order follow DecLib: a picture keeps its slot until its last use as a
reference and its output; output is POC order within a coded video sequence (IDR starts a new one).
"""
import ctypes as C
import concurrent.futures as cf
import threading
import time

import numpy as np

from . import native as N
from . import parser as P

_bound = False


def _bind(L):
    global _bound
    if not _bound:
        L.vvcp_plan_picture.argtypes = [C.c_void_p, C.c_int32, C.POINTER(N.SeqParams), C.c_int32, C.c_void_p, C.c_uint32,
                                        C.POINTER(C.c_void_p)]
        _bound = True
    return L


class Plan:
    """Decode plan of a bitstream: picture order, reference structure, DPB slots and output order."""

    def __init__(self, s, nslots, base=0):
        n = len(s)
        self.info = [s.info(i) for i in range(n)]
        self.refs = []
        for i in range(n):
            pp = s.pic_params(i)
            self.refs.append([[int(pp.ref_poc[l][r]) for r in range(pp.num_ref[l])] for l in range(2)])
        # coded video sequences: an IDR (NAL types 7, 8) starts a new one
        cvs, k = [], -1
        for inf in self.info:
            if inf["nal_type"] in (7, 8) or k < 0:
                k += 1
            cvs.append(k)
        self.cvs = cvs
        key = [(cvs[i], self.info[i]["poc"]) for i in range(n)]
        self.out_order = sorted((i for i in range(n) if self.info[i]["output"]), key=lambda i: key[i])
        # a picture can be output once every picture before it in output order is decoded
        ready, m = {}, -1
        for i in self.out_order:
            m = max(m, i)
            ready[i] = m
        self.out_ready = ready
        # last decode index that needs picture i: references by later pictures of its CVS, its output
        last = list(range(n))
        self.referenced = [False] * n
        for j in range(n):
            for l in range(2):
                for poc in self.refs[j][l]:
                    src = self._find(j, poc)
                    last[src] = max(last[src], j)
                    self.referenced[src] = True
        for i, r in ready.items():
            last[i] = max(last[i], r)
        self.last_use = last
        # slots
        free = list(range(base, base + nslots))
        held = {}
        self.slot = [0] * n
        for i in range(n):
            for q, s_ in list(held.items()):
                if last[q] < i:
                    free.append(s_)
                    del held[q]
            if not free:
                raise RuntimeError("DPB of %d slots exhausted at picture %d" % (nslots, i))
            self.slot[i] = free.pop(0)
            held[i] = self.slot[i]

    def _find(self, j, poc):
        """decode index of the reference picture with this POC for picture j (the latest before j in its CVS)"""
        for i in range(j - 1, -1, -1):
            if self.info[i]["poc"] == poc and self.cvs[i] == self.cvs[j]:
                return i
        raise KeyError("picture %d: reference POC %d was not decoded" % (j, poc))

    def ref_slots(self, j):
        rs = np.zeros((2, N.MAX_REF), np.int32)
        for l in range(2):
            for r, poc in enumerate(self.refs[j][l]):
                rs[l, r] = self.slot[self._find(j, poc)]
        return rs


class SequenceDecode:
    """One decode of a bitstream through a Context, on DPB slots [base, base + nslots).

    run() parses ahead on `pool`, derives / plans / launches in decoding order on the calling thread and
    calls on_output(poc, slot) in output order while the slot still holds the picture (e.g. to write the
    YUV file). Launches go through `launch_lock`, so several SequenceDecodes (on disjoint slot ranges) may
    run on several threads against one Context."""

    def __init__(self, ctx, data, pool, nslots=16, base=0, stages=N.STAGE_ALL, launch_lock=None, keep=24):
        self.ctx, self.pool = ctx, pool
        self.L = _bind(N.lib())
        self.s = P.Stream(data, lib=self.L)
        self.plan = Plan(self.s, nslots, base)
        inf = self.plan.info[0]
        self.W, self.H = inf["width"], inf["height"]
        self.sp = N.SeqParams(self.W, self.H, 1, inf["bit_depth"], inf["ctu_log2"], ctx.dpb_slots, 0)
        self.stages = stages
        self.lock = launch_lock or threading.Lock()
        self.keep = keep
        # seconds this decode's thread spent per phase (waiting on the parse pool, on the GPU's DMVR
        # deltas, deriving motion, planning, uploading, launching)
        self.times = dict.fromkeys(("parse", "parse_wait", "dmvr_wait", "derive", "plan", "prepare", "launch"), 0.0)
        self._tlock = threading.Lock()

    def _parse(self, i):
        t0 = time.perf_counter()
        self.s.parse(i)
        dt = time.perf_counter() - t0
        with self._tlock:
            self.times["parse"] += dt   # on the pool's threads

    def _plan_picture(self, i):
        rs = self.plan.ref_slots(i)
        h = C.c_void_p()
        rc = self.L.vvcp_plan_picture(self.s.h, i, C.byref(self.sp), self.plan.slot[i], rs.ctypes.data, self.stages,
                                      C.byref(h))
        if rc != 0:
            raise P.ParseError("picture %d plan: %s" % (i, self.L.vvcp_last_error().decode()))
        return N.Picture.wrap(h)

    def run(self, on_output=None, keep_handles=False):
        """Decodes the stream; returns [(poc, slot)] in output order, and with keep_handles also the
        prepared-picture handles in decoding order (not released: the caller may launch them again)."""
        n = len(self.s)
        parsed = [self.pool.submit(self._parse, i) for i in range(n)]
        handles = {}          # decode index -> prepared-picture handle
        n_dmvr = {}
        refined = set()
        live = []
        out_pos = 0
        out = self.plan.out_order
        try:
            T = self.times
            clk = time.perf_counter
            for i in range(n):
                t0 = clk()
                parsed[i].result()
                t1 = clk()
                # the collocated picture is one of the references: refine those still pending
                for l in range(2):
                    for poc in self.plan.refs[i][l]:
                        j = self.plan._find(i, poc)
                        if j not in refined:
                            d = self.ctx.picture_dmvr_deltas(handles[j], n_dmvr[j])
                            self.s.refine(j, d)
                            refined.add(j)
                t2 = clk()
                self.s.derive(i)
                t3 = clk()
                pic = self._plan_picture(i)
                t4 = clk()
                try:
                    n_dmvr[i] = pic.work_counts()["dmvr"]
                    h = self.ctx.prepare_planned(pic)
                finally:
                    pic.close()
                t5 = clk()
                with self.lock:
                    self.ctx.launch(h)
                t6 = clk()
                with self._tlock:
                    T["parse_wait"] += t1 - t0
                T["dmvr_wait"] += t2 - t1
                T["derive"] += t3 - t2
                T["plan"] += t4 - t3
                T["prepare"] += t5 - t4
                T["launch"] += t6 - t5
                handles[i] = h
                live.append(i)
                if not self.plan.referenced[i]:
                    refined.add(i)
                while out_pos < len(out) and self.plan.out_ready[out[out_pos]] <= i:
                    k = out[out_pos]
                    if on_output:
                        on_output(self.plan.info[k]["poc"], self.plan.slot[k])
                    out_pos += 1
                # release handles of pictures far behind whose deltas are no longer needed
                while not keep_handles and len(live) > self.keep and live[0] in refined:
                    self.ctx.release(handles.pop(live.pop(0)))
            kept = [handles.pop(i) for i in range(n)] if keep_handles else None
        finally:
            for f in parsed:
                f.cancel()
            for i in live:
                if i in handles:
                    self.ctx.release(handles.pop(i))
        order = [(self.plan.info[k]["poc"], self.plan.slot[k]) for k in out]
        return (order, kept) if keep_handles else order


def decode_bitstream(data, ctx=None, threads=8, dpb_slots=16, device=0, on_output=None):
    """Decodes a whole bitstream; returns [(poc, slot)] in output order (the last pictures stay in
    their slots) and the Context (created here unless given)."""
    own = ctx is None
    s = P.Stream(data)
    inf = s.info(0)
    s.close()
    if own:
        ctx = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"],
                        dpb_slots=dpb_slots, device=device)
    with cf.ThreadPoolExecutor(threads) as pool:
        seq = SequenceDecode(ctx, data, pool, nslots=dpb_slots)
        order = seq.run(on_output)
    ctx.sync()
    return order, ctx
