"""Bitstream-to-pictures driver: the decode loop of DecoderApp (DecApp::decode, DecApp.cpp:118-200 ->
DecLib::decode / executeLoopFilters, DecLib.cpp) on the MI355X path, from an Annex-B VVC bitstream.

The loop runs natively (vvcp_decode, vvc_amd/csrc/vvcp_decode.cpp); per picture, in decoding order:
  1. CABAC parse (vvcp_parse_picture) — independent of every other picture, so all pictures are parsed
     ahead on parser threads;
  2. motion derivation (vvcp_derive_motion) — needs the refined motion of the collocated picture, i.e.
     that picture's DMVR deltas from the GPU (vvcr_picture_dmvr_deltas waits for its inter stage only);
  3. native planning from the parser's state (vvcp_plan_picture -> vvcr_picture_*), upload
     (vvcr_prepare_planned) and launch on the context's execution lanes.
The DPB (slots) and output order follow DecLib: a picture keeps its slot until its last use as a
reference and its output; output is POC order within a coded video sequence (IDR starts a new one).
Plan below restates that plan in Python for the tests (vvcp_decode_plan is the one decoding uses).
"""
import ctypes as C

import numpy as np

from . import native as N
from . import parser as P

_bound = False


def _bind(L):
    global _bound
    if not _bound:
        L.vvcp_plan_picture.argtypes = [C.c_void_p, C.c_int32, C.POINTER(N.SeqParams), C.c_int32, C.c_void_p, C.c_uint32,
                                        C.POINTER(C.c_void_p)]
        L.vvcp_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.vvcp_decode_plan.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.vvcp_decode_live_bound.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
        L.vvcp_decode_batches.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
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


OUTPUT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_int32)
PHASES = ("parse", "parse_wait", "dmvr_wait", "derive", "plan", "prepare", "launch", "output")


class DecodeParams(C.Structure):
    """vvcp_decode_params (include/vvcp.h)"""
    _fields_ = [("slot_base", C.c_int32), ("num_slots", C.c_int32), ("ctx_slots", C.c_int32), ("threads", C.c_int32),
                ("stage_mask", C.c_uint32), ("on_output", OUTPUT_FN), ("user", C.c_void_p),
                ("handles_out", C.POINTER(C.c_int32)), ("phase_seconds", C.POINTER(C.c_double))]


class SequenceDecode:
    """One decode of a bitstream through a Context, on DPB slots [base, base + nslots): the native
    decode loop vvcp_decode (vvc_amd/csrc/vvcp_decode.cpp) — parser threads, motion derivation with
    the GPU's DMVR feedback, planning, upload and launch all in C++, the GIL released for the whole
    decode. on_output(poc, slot) is called in output order while the slot still holds the picture.
    Several SequenceDecodes on disjoint slot ranges may run on several threads against one Context."""

    def __init__(self, ctx, data, pool=None, nslots=16, base=0, stages=N.STAGE_ALL, launch_lock=None, keep=24, threads=4):
        self.ctx = ctx
        self.L = _bind(N.lib())
        self.s = P.Stream(data, lib=self.L)
        self.nslots, self.base, self.stages, self.threads = nslots, base, stages, threads
        n = len(self.s)
        slots, order = (C.c_int32 * max(n, 1))(), (C.c_int32 * max(n, 1))()
        m = self.L.vvcp_decode_plan(self.s.h, base, nslots, slots, order)
        if m < 0:
            raise P.ParseError("decode plan: %s" % self.L.vvcp_last_error().decode())
        self.slot = list(slots)[:n]
        self.out_order = list(order)[:m]
        first = (C.c_int32 * max(n, 1))()
        if self.L.vvcp_decode_batches(self.s.h, base, nslots, first) < 0:
            raise P.ParseError("decode batches: %s" % self.L.vvcp_last_error().decode())
        self.batch = list(first)[:n]   # frame batching of vvcp_decode: k first of a group of k, 0 a later member
        self.info = [self.s.info(i) for i in range(n)]
        # seconds per phase (include/vvcp.h VVCP_PHASE_*): parse summed over the parser threads
        self.times = dict.fromkeys(PHASES, 0.0)

    def run(self, on_output=None, keep_handles=False):
        """Decodes the stream; returns [(poc, slot)] in output order, and with keep_handles also the
        prepared-picture handles in decoding order (not released: the caller may launch them again)."""
        n = len(self.s)
        err = []

        def cb(user, idx, poc, slot):
            try:
                on_output(poc, slot)
            except Exception as e:   # never unwind through the C frames: reported after the decode
                err.append(e)
        fn = OUTPUT_FN(cb) if on_output else OUTPUT_FN()
        handles = (C.c_int32 * max(n, 1))() if keep_handles else None
        phases = (C.c_double * len(PHASES))()
        prm = DecodeParams(self.base, self.nslots, self.ctx.dpb_slots, self.threads, self.stages, fn, None,
                           C.cast(handles, C.POINTER(C.c_int32)) if handles is not None else None,
                           C.cast(phases, C.POINTER(C.c_double)))
        rc = self.L.vvcp_decode(self.s.h, self.ctx.h, C.byref(prm))
        for k, name in enumerate(PHASES):
            self.times[name] += phases[k]
        if rc != 0:
            raise P.ParseError("vvcp_decode: %s" % self.L.vvcp_last_error().decode())
        if err:
            raise err[0]
        order = [(self.info[k]["poc"], self.slot[k]) for k in self.out_order]
        return (order, list(handles)[:n]) if keep_handles else order


def launch_groups(handles, batch):
    """The prepared handles of one decode (decoding order) grouped as vvcp_decode launches them: groups of
    frame-batched pictures (SequenceDecode.batch) and single pictures."""
    out, i = [], 0
    while i < len(handles):
        k = max(1, min(batch[i], len(handles) - i))
        out.append(handles[i:i + k])
        i += k
    return out


def launch_group(ctx, group):
    if len(group) > 1:
        ctx.launch_batch(group)
    else:
        ctx.launch(group[0])


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
    seq = SequenceDecode(ctx, data, nslots=dpb_slots, threads=threads)
    order = seq.run(on_output)
    ctx.sync()
    return order, ctx
