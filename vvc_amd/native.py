"""ctypes binding of libvvcr's C-ABI (include/vvcr.h). The product path: if the HIP library is not
built or cannot be loaded this module raises — there is no CPU fallback."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VVCR_LIB") or os.path.join(_HERE, "libvvcr.so")   # VVCR_LIB: diagnostics builds

MAX_REF = 16
MAX_TILE_LINES = 64
STAGE_RESID, STAGE_INTER, STAGE_INTRA, STAGE_LMCS_INV = 0x01, 0x02, 0x04, 0x08
STAGE_DBK, STAGE_SAO, STAGE_ALF, STAGE_ALL = 0x10, 0x20, 0x40, 0x7F
BUF_RECO, BUF_PRED, BUF_RESI = 0, 1, 2

I32 = C.c_int32


class OutputParams(C.Structure):
    """vvcr_output_params: DecoderApp -d, the conformance window (luma samples), --ClipOutputVideoToRec709Range"""
    _fields_ = [(n, I32) for n in ("file_bit_depth", "conf_left", "conf_right", "conf_top", "conf_bottom", "clip_rec709")]


class SeqParams(C.Structure):
    _fields_ = [(n, I32) for n in ("width", "height", "chroma_format", "bit_depth", "ctu_log2", "dpb_slots", "device")]


class PicParams(C.Structure):
    _fields_ = [
        ("poc", I32), ("slot", I32), ("slice_type", I32), ("slice_qp", I32),
        ("num_ref", I32 * 2),
        ("ref_slot", (I32 * MAX_REF) * 2), ("ref_poc", (I32 * MAX_REF) * 2), ("ref_lt", (I32 * MAX_REF) * 2),
        ("dual_tree", I32), ("dep_quant", I32), ("sign_hiding", I32), ("joint_cbcr", I32),
        ("bdof_enabled", I32), ("dmvr_enabled", I32), ("prof_enabled", I32), ("lfnst_enabled", I32),
        ("mts_intra", I32), ("mts_inter", I32), ("sbt", I32),
        ("wp_p", I32), ("wp_b", I32),
        ("wp", (((I32 * 7) * 3) * MAX_REF) * 2),
        ("dbk_disable", I32), ("dbk_beta_offset_div2", I32), ("dbk_tc_offset_div2", I32),
        ("lf_across_slices", I32), ("lf_across_tiles", I32),
        ("chroma_qp_off", I32 * 3),
        ("chroma_qp_map", (I32 * 128) * 3),
        ("sao_luma", I32), ("sao_chroma", I32),
        ("alf_en", I32 * 3), ("ccalf_en", I32 * 2), ("alf_vb_luma", I32), ("alf_vb_chroma", I32),
        ("lmcs_enabled", I32), ("lmcs_chroma_scale", I32), ("lmcs_min_bin", I32), ("lmcs_max_bin", I32),
        ("lmcs_fwd", C.c_int16 * 1024), ("lmcs_inv", C.c_int16 * 1024), ("lmcs_pivot", C.c_int16 * 17),
        ("lmcs_cadj", I32 * 16),
        ("max_tb_log2", I32), ("log2_max_ts", I32),
        ("use_mts", I32), ("implicit_mts", I32), ("joint_cbcr_sign", I32),
        ("num_tile_cols", I32), ("num_tile_rows", I32),
        ("tile_col_bd", I32 * (MAX_TILE_LINES + 1)), ("tile_row_bd", I32 * (MAX_TILE_LINES + 1)),
        ("entropy_sync", I32),
        ("shard_y0", I32), ("shard_y1", I32),
        ("vb_disabled", I32), ("num_vb_ver", I32), ("vb_ver", I32 * 3), ("num_vb_hor", I32), ("vb_hor", I32 * 3),
        ("ladf_num", I32), ("ladf_qp_offset", I32 * 5), ("ladf_lower_bound", I32 * 5),
    ]


class Alf(C.Structure):
    _fields_ = [("num_luma_sets", I32),
                ("luma_coef", C.c_void_p), ("luma_clip", C.c_void_p),
                ("chroma_coef", C.c_void_p), ("chroma_clip", C.c_void_p), ("cc_coef", C.c_void_p),
                ("ctb_en", C.c_void_p), ("ctb_alt", C.c_void_p), ("ctb_filter_set", C.c_void_p), ("cc_ctl", C.c_void_p)]


class VvcrError(RuntimeError):
    pass


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise VvcrError("libvvcr.so is not built (run __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.vvcr_create.argtypes = [C.POINTER(SeqParams), C.POINTER(P)]
        L.vvcr_destroy.argtypes = [P]
        L.vvcr_last_error.argtypes = [P]
        L.vvcr_last_error.restype = C.c_char_p
        L.vvcr_begin_picture.argtypes = [P, C.POINTER(PicParams)]
        L.vvcr_submit.argtypes = [P, P, I32, P, I32, P, I32, P, C.c_int64, P, P, I32]
        L.vvcr_set_loop_filter_params.argtypes = [P, P, C.POINTER(Alf)]
        L.vvcr_end_picture.argtypes = [P]
        L.vvcr_end_picture_stages.argtypes = [P, C.c_uint32]
        L.vvcr_sync.argtypes = [P]
        L.vvcr_read_plane.argtypes = [P, I32, I32, I32, P, I32]
        L.vvcr_write_plane.argtypes = [P, I32, I32, I32, P, I32]
        L.vvcr_last_stage_times.argtypes = [P, C.POINTER(C.c_float), I32]
        L.vvcr_get_dmvr_deltas.argtypes = [P, P, C.c_int64]
        L.vvcr_picture_dmvr_deltas.argtypes = [P, I32, P, C.c_int64]
        L.vvcr_prepare_picture.argtypes = [P, C.c_uint32, C.POINTER(I32)]
        L.vvcr_launch_picture.argtypes = [P, I32]
        L.vvcr_launch_picture_stages.argtypes = [P, I32, C.c_uint32]
        L.vvcr_launch_pictures.argtypes = [P, C.POINTER(I32), I32]
        L.vvcr_release_picture.argtypes = [P, I32]
        L.vvcr_kernel_stats.argtypes = [P, I32, C.POINTER(KernelStat), I32]
        L.vvcr_stream.argtypes = [P]
        L.vvcr_stream.restype = P
        L.vvcr_set_timing.argtypes = [P, I32]
        L.vvcr_rd_plan.argtypes = [P, P, I32, C.POINTER(I32)]
        L.vvcr_rd_run.argtypes = [P, I32, P, P, P, P]
        L.vvcr_fwd_plan.argtypes = [P, P, I32, I32, C.POINTER(I32)]
        L.vvcr_fwd_run.argtypes = [P, I32, P, P]
        L.vvcr_rdo_release.argtypes = [P, I32]
        L.vvcr_rd_dist.argtypes = [P, P, I32, P, C.c_int64, P, C.c_int64, P, P]
        L.vvcr_fwd_transform.argtypes = [P, P, I32, I32, P, C.c_int64, P, C.c_int64]
        L.vvcr_picture_create.argtypes = [C.POINTER(SeqParams), C.POINTER(PicParams), C.POINTER(P)]
        L.vvcr_picture_submit.argtypes = [P, P, I32, P, I32, P, I32, P, C.c_int64, P, P, I32]
        L.vvcr_picture_set_loop_filter_params.argtypes = [P, P, C.POINTER(Alf)]
        L.vvcr_picture_plan.argtypes = [P, C.c_uint32]
        L.vvcr_picture_work_counts.argtypes = [P, C.POINTER(C.c_int64), I32]
        L.vvcr_picture_last_error.argtypes = [P]
        L.vvcr_picture_last_error.restype = C.c_char_p
        L.vvcr_picture_destroy.argtypes = [P]
        L.vvcr_prepare_planned.argtypes = [P, P, C.POINTER(I32)]
        L.vvcr_output_bytes.argtypes = [P, C.POINTER(OutputParams)]
        L.vvcr_output_bytes.restype = C.c_int64
        L.vvcr_write_output.argtypes = [P, I32, C.POINTER(OutputParams), P, I32]
        L.vvcr_rows_bytes.argtypes = [P, I32]
        L.vvcr_rows_bytes.restype = C.c_int64
        L.vvcr_export_rows.argtypes = [P, I32, I32, I32, P]
        L.vvcr_import_rows.argtypes = [P, I32, I32, I32, P]
        L.vvcr_export_rows_async.argtypes = [P, I32, I32, I32, P, P]
        L.vvcr_import_rows_async.argtypes = [P, I32, I32, I32, P, P]
        _lib = L
    return _lib


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 16), ("launches", C.c_int32), ("ms", C.c_float), ("alg_bytes", C.c_double),
                ("pictures", C.c_int32), ("pad", C.c_int32)]


EXPORTS = ["vvcr_prepare_picture", "vvcr_launch_picture", "vvcr_launch_picture_stages", "vvcr_launch_pictures", "vvcr_release_picture", "vvcr_kernel_stats", "vvcr_create", "vvcr_destroy", "vvcr_last_error", "vvcr_begin_picture", "vvcr_submit",
           "vvcr_set_loop_filter_params", "vvcr_end_picture", "vvcr_end_picture_stages", "vvcr_sync",
           "vvcr_read_plane", "vvcr_write_plane", "vvcr_read_picture", "vvcr_get_dmvr_deltas", "vvcr_picture_dmvr_deltas",
           "vvcr_last_stage_times", "vvcr_stream", "vvcr_rd_plan", "vvcr_rd_run", "vvcr_fwd_plan", "vvcr_fwd_run",
           "vvcr_rdo_release", "vvcr_rd_dist", "vvcr_fwd_transform", "vvcr_set_timing",
           "vvcr_picture_create", "vvcr_picture_submit", "vvcr_picture_set_loop_filter_params", "vvcr_picture_plan",
           "vvcr_picture_work_counts", "vvcr_picture_last_error", "vvcr_picture_destroy", "vvcr_prepare_planned",
           "vvcr_rows_bytes", "vvcr_export_rows", "vvcr_import_rows", "vvcr_export_rows_async", "vvcr_import_rows_async",
           "vvcr_output_bytes", "vvcr_write_output"]

# encoder RDO block descriptors (include/vvcr.h vvcr_rd_block / vvcr_fwd_block) as numpy record types
RD_BLOCK = [("org_off", "<i8"), ("cur_off", "<i8"), ("org_stride", "<i4"), ("cur_stride", "<i4"), ("width", "<i4"),
            ("height", "<i4")]
FWD_BLOCK = [("src_off", "<i8"), ("dst_off", "<i8"), ("src_stride", "<i4"), ("width", "<i4"), ("height", "<i4"),
             ("tr_hor", "<i4"), ("tr_ver", "<i4"), ("lfnst", "<i4")]


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


class Picture:
    """Host-only picture builder (vvcr_picture_*): validate and plan one picture without a context or a
    device. Several Pictures may be planned on several threads at once (ctypes drops the GIL in the
    library calls); Context.prepare_planned uploads a planned one."""

    def __init__(self, width, height, pp, bit_depth=10, ctu_log2=7, dpb_slots=32):
        self.L = lib()
        sp = SeqParams(width, height, 1, bit_depth, ctu_log2, dpb_slots, 0)
        h = C.c_void_p()
        r = self.L.vvcr_picture_create(C.byref(sp), C.byref(pp), C.byref(h))
        if r != 0:
            raise VvcrError("vvcr_picture_create failed (%d): %s" % (r, self.L.vvcr_picture_last_error(None).decode()))
        self.h = h
        self._keep = []

    @classmethod
    def wrap(cls, handle):
        """a Picture for a vvcr_picture made elsewhere (e.g. vvcp_plan_picture); takes ownership"""
        pic = cls.__new__(cls)
        pic.L, pic.h, pic._keep = lib(), handle, []
        return pic

    def _chk(self, r, what):
        if r != 0:
            raise VvcrError("%s failed (%d): %s" % (what, r, self.L.vvcr_picture_last_error(self.h).decode()))

    def submit(self, cu, pu, tu, coef, motion, geo):
        arrs = [np.ascontiguousarray(a, np.int32) for a in (cu, pu, tu, coef, motion, geo)]
        cu, pu, tu, coef, motion, geo = arrs
        self._chk(self.L.vvcr_picture_submit(self.h, _ptr(cu), len(cu), _ptr(pu), len(pu), _ptr(tu), len(tu),
                                             _ptr(coef), coef.size, _ptr(motion), _ptr(geo), len(geo)),
                  "vvcr_picture_submit")

    def set_loop_filter_params(self, sao, alf_struct, keep):
        self._keep = keep
        self._chk(self.L.vvcr_picture_set_loop_filter_params(self.h, _ptr(sao), C.byref(alf_struct) if alf_struct else None),
                  "vvcr_picture_set_loop_filter_params")

    def plan(self, stages=STAGE_ALL):
        self._chk(self.L.vvcr_picture_plan(self.h, stages), "vvcr_picture_plan")

    def work_counts(self):
        c = (C.c_int64 * 10)()
        n = self.L.vvcr_picture_work_counts(self.h, c, 10)
        if n < 0:
            self._chk(n, "vvcr_picture_work_counts")
        return dict(zip(("tb", "mc", "mc_bidir", "affine", "recon_tiles", "intra_steps", "dbk_segments", "dmvr",
                         "ref_y0", "ref_y1"), list(c)))

    def close(self):
        if self.h:
            self.L.vvcr_picture_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One libvvcr context = one device-resident DPB and stream."""

    def __init__(self, width, height, bit_depth=10, ctu_log2=7, dpb_slots=16, device=0):
        self.L = lib()
        sp = SeqParams(width, height, 1, bit_depth, ctu_log2, dpb_slots, device)
        h = C.c_void_p()
        r = self.L.vvcr_create(C.byref(sp), C.byref(h))
        if r != 0:
            raise VvcrError("vvcr_create failed (%d): %s" % (r, self.L.vvcr_last_error(None).decode()))
        self.h = h
        self.width, self.height = width, height
        self.dpb_slots = dpb_slots
        self._keep = []

    def _chk(self, r, what):
        if r != 0:
            raise VvcrError("%s failed (%d): %s" % (what, r, self.L.vvcr_last_error(self.h).decode()))

    def close(self):
        if self.h:
            self.L.vvcr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def begin_picture(self, pp: PicParams):
        self._chk(self.L.vvcr_begin_picture(self.h, C.byref(pp)), "vvcr_begin_picture")

    def submit(self, cu, pu, tu, coef, motion, geo):
        arrs = [np.ascontiguousarray(a, np.int32) for a in (cu, pu, tu, coef, motion, geo)]
        cu, pu, tu, coef, motion, geo = arrs
        self._chk(self.L.vvcr_submit(self.h, _ptr(cu), len(cu), _ptr(pu), len(pu), _ptr(tu), len(tu),
                                     _ptr(coef), coef.size, _ptr(motion), _ptr(geo), len(geo)),
                  "vvcr_submit")

    def set_loop_filter_params(self, sao, alf_struct, keep):
        self._keep = keep
        self._chk(self.L.vvcr_set_loop_filter_params(self.h, _ptr(sao), C.byref(alf_struct) if alf_struct else None),
                  "vvcr_set_loop_filter_params")

    def end_picture(self, stages=STAGE_ALL):
        self._chk(self.L.vvcr_end_picture_stages(self.h, stages), "vvcr_end_picture_stages")

    def sync(self):
        self._chk(self.L.vvcr_sync(self.h), "vvcr_sync")

    def read_plane(self, buf, slot, comp):
        w, h = (self.width, self.height) if comp == 0 else (self.width // 2, self.height // 2)
        out = np.empty((h, w), np.int16)
        self._chk(self.L.vvcr_read_plane(self.h, buf, slot, comp, _ptr(out), w), "vvcr_read_plane")
        return out

    def write_plane(self, buf, slot, comp, data):
        data = np.ascontiguousarray(data, np.int16)
        self._chk(self.L.vvcr_write_plane(self.h, buf, slot, comp, _ptr(data), data.shape[1]), "vvcr_write_plane")

    def prepare(self, stages=STAGE_ALL):
        """vvcr_prepare_picture: plan + upload the current picture; returns a handle."""
        h = C.c_int32(0)
        self._chk(self.L.vvcr_prepare_picture(self.h, stages, C.byref(h)), "vvcr_prepare_picture")
        return h.value

    def prepare_planned(self, pic):
        """vvcr_prepare_planned: upload a planned Picture; returns a handle (thread-safe per picture)."""
        h = C.c_int32(0)
        self._chk(self.L.vvcr_prepare_planned(self.h, pic.h, C.byref(h)), "vvcr_prepare_planned")
        return h.value

    def output_bytes(self, op):
        return self.L.vvcr_output_bytes(self.h, C.byref(op))

    def write_output(self, slot, op, dev_ptr=None):
        """the slot's frame as DecoderApp writes it to its -o file (bytes); dev_ptr: write into device
        memory instead and return None"""
        if dev_ptr is not None:
            self._chk(self.L.vvcr_write_output(self.h, slot, C.byref(op), dev_ptr, 1), "vvcr_write_output")
            return None
        buf = np.empty(self.output_bytes(op), np.uint8)
        self._chk(self.L.vvcr_write_output(self.h, slot, C.byref(op), buf.ctypes.data, 0), "vvcr_write_output")
        return buf

    def rows_bytes(self, n):
        return self.L.vvcr_rows_bytes(self.h, n)

    def export_rows(self, slot, y0, n, dev_ptr):
        """luma rows [y0, y0+n) + co-located chroma rows of a DPB slot -> packed device buffer"""
        self._chk(self.L.vvcr_export_rows(self.h, slot, y0, n, dev_ptr), "vvcr_export_rows")

    def import_rows(self, slot, y0, n, dev_ptr):
        self._chk(self.L.vvcr_import_rows(self.h, slot, y0, n, dev_ptr), "vvcr_import_rows")

    def export_rows_async(self, slot, y0, n, dev_ptr, stream):
        """export_rows enqueued on a caller's HIP stream (a torch stream's cuda_stream), no host sync"""
        self._chk(self.L.vvcr_export_rows_async(self.h, slot, y0, n, dev_ptr, stream), "vvcr_export_rows_async")

    def import_rows_async(self, slot, y0, n, dev_ptr, stream):
        self._chk(self.L.vvcr_import_rows_async(self.h, slot, y0, n, dev_ptr, stream), "vvcr_import_rows_async")

    def launch(self, handle):
        self._chk(self.L.vvcr_launch_picture(self.h, handle), "vvcr_launch_picture")

    def launch_batch(self, handles):
        """frame-batched launch of independent inter pictures (vvcr_launch_pictures): one plain-MC launch"""
        arr = (C.c_int32 * len(handles))(*handles)
        self._chk(self.L.vvcr_launch_pictures(self.h, arr, len(handles)), "vvcr_launch_pictures")

    def launch_stages(self, handle, stages):
        """the stages of `stages` the picture was prepared with (vvcr_launch_picture_stages)"""
        self._chk(self.L.vvcr_launch_picture_stages(self.h, handle, stages), "vvcr_launch_picture_stages")

    def release(self, handle):
        self._chk(self.L.vvcr_release_picture(self.h, handle), "vvcr_release_picture")

    def set_timing(self, on):
        self._chk(self.L.vvcr_set_timing(self.h, 1 if on else 0), "vvcr_set_timing")

    # ---- encoder RDO inner loop (vvcr_rd_* / vvcr_fwd_*)
    def rd_dist(self, blocks, org, cur):
        """SAD and Hadamard SATD per block (RdCost xGetSAD / xGetHADs); host arrays in and out."""
        blocks = np.ascontiguousarray(blocks)
        org, cur = np.ascontiguousarray(org, np.int16), np.ascontiguousarray(cur, np.int16)
        n = len(blocks)
        sad, satd = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        self._chk(self.L.vvcr_rd_dist(self.h, blocks.ctypes.data, n, org.ctypes.data, org.size, cur.ctypes.data, cur.size,
                                      sad.ctypes.data, satd.ctypes.data), "vvcr_rd_dist")
        return sad, satd

    def fwd_transform(self, blocks, resi, ncoef, bit_depth=10):
        """Forward transforms (TrQuant::xT) of the blocks; returns the int32 coefficient pool."""
        blocks = np.ascontiguousarray(blocks)
        resi = np.ascontiguousarray(resi, np.int16)
        coef = np.zeros(ncoef, np.int32)
        self._chk(self.L.vvcr_fwd_transform(self.h, blocks.ctypes.data, len(blocks), bit_depth, resi.ctypes.data, resi.size,
                                            coef.ctypes.data, coef.size), "vvcr_fwd_transform")
        return coef

    def rd_plan(self, blocks):
        blocks = np.ascontiguousarray(blocks)
        h = C.c_int32(0)
        self._chk(self.L.vvcr_rd_plan(self.h, blocks.ctypes.data, len(blocks), C.byref(h)), "vvcr_rd_plan")
        return h.value

    def rd_run(self, plan, org_ptr, cur_ptr, sad_ptr, satd_ptr):
        """device pointers (e.g. torch tensor data_ptr()); asynchronous on the context stream"""
        self._chk(self.L.vvcr_rd_run(self.h, plan, org_ptr, cur_ptr, sad_ptr, satd_ptr), "vvcr_rd_run")

    def fwd_plan(self, blocks, bit_depth=10):
        blocks = np.ascontiguousarray(blocks)
        h = C.c_int32(0)
        self._chk(self.L.vvcr_fwd_plan(self.h, blocks.ctypes.data, len(blocks), bit_depth, C.byref(h)), "vvcr_fwd_plan")
        return h.value

    def fwd_run(self, plan, resi_ptr, coef_ptr):
        self._chk(self.L.vvcr_fwd_run(self.h, plan, resi_ptr, coef_ptr), "vvcr_fwd_run")

    def rdo_release(self, plan):
        self._chk(self.L.vvcr_rdo_release(self.h, plan), "vvcr_rdo_release")

    def kernel_stats(self, handle=0):
        """[(name, launches, ms, alg_bytes, pictures)] of the last launch of a prepared picture (0 = last launched);
        pictures: the pictures the group's launches carried (a frame-batched k_mc: 2 on the first, 0 on the other)."""
        arr = (KernelStat * 16)()
        n = self.L.vvcr_kernel_stats(self.h, handle, arr, 16)
        if n < 0:
            self._chk(n, "vvcr_kernel_stats")
        return [(arr[i].name.decode(), arr[i].launches, arr[i].ms, arr[i].alg_bytes, arr[i].pictures) for i in range(n)]

    def dmvr_deltas(self):
        """DMVR refinement deltas of the last picture, [n][2] (vvcr_get_dmvr_deltas)."""
        n = self.L.vvcr_get_dmvr_deltas(self.h, None, 0)
        if n < 0:
            self._chk(n, "vvcr_get_dmvr_deltas")
        out = np.zeros((n, 2), np.int32)
        if n:
            self._chk(min(0, self.L.vvcr_get_dmvr_deltas(self.h, out.ctypes.data, n)), "vvcr_get_dmvr_deltas")
        return out

    def picture_dmvr_deltas(self, handle, cap):
        """DMVR deltas of a launched prepared picture (vvcr_picture_dmvr_deltas); cap = expected count"""
        out = np.zeros((max(cap, 1), 2), np.int32)
        n = self.L.vvcr_picture_dmvr_deltas(self.h, handle, out.ctypes.data, cap)
        if n < 0:
            self._chk(n, "vvcr_picture_dmvr_deltas")
        if n > cap:
            raise VvcrError("DMVR delta count %d > %d" % (n, cap))
        return out[:n]

    def stage_ms(self):
        t = (C.c_float * 8)()
        self._chk(self.L.vvcr_last_stage_times(self.h, t, 8), "vvcr_last_stage_times")
        return list(t)
