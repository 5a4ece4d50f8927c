"""Host driver of the reconstruction path: replays parsed pictures (descriptor captures) through
libvvcr in decode order, manages DPB slots, and mirrors DecApp/DecLib's per-picture sequencing
(DecApp::decode DecApp.cpp:118-200: decode NALs -> DecLib::executeLoopFilters -> finishPicture).
"""
import glob
import hashlib
import json
import os

import numpy as np

from . import capfile
from . import native as N


def load_sequence(path, max_pics=0):
    files = sorted(glob.glob(os.path.join(path, "pic_*.xz"))) or sorted(glob.glob(os.path.join(path, "pic_*.cap")))
    if max_pics:
        files = files[:max_pics]
    return [capfile.load_any(f) for f in files]


def load_meta(path):
    with open(os.path.join(path, "md5.json")) as f:
        return json.load(f)


def plane_md5(plane):
    return hashlib.md5(np.ascontiguousarray(plane).astype("<u2").tobytes()).hexdigest()


class SlotAllocator:
    """Assigns DPB slots so that a picture keeps its slot until its last use as a reference."""

    def __init__(self, pics, nslots, base=0):
        self.last_use = {}
        for i, p in enumerate(pics):
            self.last_use.setdefault(p["hdr"]["poc"], i)
            for l in range(2):
                for r in range(p["hdr"]["num_ref_l%d" % l]):
                    self.last_use[int(p["ref_poc"][l][r])] = i
        self.nslots = nslots
        self.slot_of = {}
        self.free = list(range(base, base + nslots))   # base: a disjoint slot range per segment copy (bench.py)

    def assign(self, i, poc):
        # release pictures no longer referenced at or after decode index i
        for q, s in list(self.slot_of.items()):
            if self.last_use.get(q, -1) < i and q != poc:
                del self.slot_of[q]
                self.free.append(s)
        if not self.free:
            raise RuntimeError("DPB exhausted")
        s = self.free.pop(0)
        self.slot_of[poc] = s
        return s


def pic_params(p, slot, slot_of, missing_ref_slot=None):
    """Picture parameters with the DPB slots of the references. A reference POC missing from slot_of is
    an error, unless the caller runs only stages that read no reference picture (residual / loop-filter
    stage tests) and names a placeholder slot explicitly (missing_ref_slot)."""
    h = p["hdr"]
    pp = N.PicParams()
    pp.poc, pp.slot, pp.slice_type, pp.slice_qp = h["poc"], slot, h["slice_type"], h["slice_qp"]
    for l in range(2):
        n = h["num_ref_l%d" % l]
        pp.num_ref[l] = n
        for r in range(n):
            poc = int(p["ref_poc"][l][r])
            pp.ref_poc[l][r] = poc
            if poc in slot_of:
                pp.ref_slot[l][r] = slot_of[poc]
            elif missing_ref_slot is not None:
                pp.ref_slot[l][r] = missing_ref_slot
            else:   # a reference the DPB does not hold: never substitute another picture silently
                raise KeyError("POC %d: reference POC %d is not in the DPB" % (h["poc"], poc))
            pp.ref_lt[l][r] = int(p["ref_lt"][l][r])
    for k in ("dual_tree", "dep_quant", "sign_hiding", "joint_cbcr", "bdof_enabled", "dmvr_enabled", "prof_enabled",
              "lfnst_enabled", "mts_intra", "mts_inter", "sbt", "wp_p", "wp_b", "dbk_disable", "dbk_beta_offset_div2",
              "dbk_tc_offset_div2", "lf_across_slices", "lf_across_tiles", "sao_luma", "sao_chroma", "alf_vb_luma",
              "alf_vb_chroma", "lmcs_chroma_scale", "lmcs_min_bin", "lmcs_max_bin", "log2_max_ts"):
        setattr(pp, k, h[k])
    pp.lmcs_enabled = h["lmcs_enabled"] and h["lmcs_slice_flag"]
    pp.use_mts, pp.implicit_mts, pp.joint_cbcr_sign = h["use_mts"], h["implicit_mts"], h["joint_cbcr_sign"]
    pp.max_tb_log2 = int(h["max_tb_size"]).bit_length() - 1
    pp.chroma_qp_off[1], pp.chroma_qp_off[2] = h["chroma_qp_off_cb"], h["chroma_qp_off_cr"]
    pp.chroma_qp_off[0] = h["chroma_qp_off_jc"]
    wp = np.ascontiguousarray(p["wp"], np.int32)
    np.copyto(np.ctypeslib.as_array(pp.wp).reshape(wp.shape), wp)
    cqm = np.array(p["chroma_qp_map"], np.int32)
    cqm[0] = p["chroma_qp_map_jc"]          # row 0 carries the joint Cb-Cr table (vvcr.h)
    np.copyto(np.ctypeslib.as_array(pp.chroma_qp_map).reshape(cqm.shape), cqm)
    for c in range(3):
        pp.alf_en[c] = h["alf_slice_en%d" % c]
    pp.ccalf_en[0], pp.ccalf_en[1] = h["ccalf_en_cb"], h["ccalf_en_cr"]
    for name, n in (("lmcs_fwd", 1024), ("lmcs_inv", 1024), ("lmcs_pivot", 17)):
        src = np.asarray(p[name], np.int16)[:n]
        np.copyto(np.ctypeslib.as_array(getattr(pp, name))[:len(src)], src)
    cadj = np.asarray(p["lmcs_cadj"], np.int32)[:16]
    np.copyto(np.ctypeslib.as_array(pp.lmcs_cadj)[:len(cadj)], cadj)
    if "tile_col_bd" in p:   # captures without these fields hold one tile
        cb, rb = np.asarray(p["tile_col_bd"], np.int32), np.asarray(p["tile_row_bd"], np.int32)
        pp.num_tile_cols, pp.num_tile_rows = len(cb) - 1, len(rb) - 1
        np.copyto(np.ctypeslib.as_array(pp.tile_col_bd)[:len(cb)], cb)
        np.copyto(np.ctypeslib.as_array(pp.tile_row_bd)[:len(rb)], rb)
    pp.entropy_sync = h.get("entropy_sync", 0)
    if h.get("vb_disabled", 0):   # captures without these fields have no virtual boundaries
        pp.num_vb_ver, pp.num_vb_hor = h["num_vb_ver"], h["num_vb_hor"]
        pp.vb_disabled = int(pp.num_vb_ver + pp.num_vb_hor > 0)
        for i in range(3):
            pp.vb_ver[i], pp.vb_hor[i] = h["vb_ver%d" % i], h["vb_hor%d" % i]
    if h.get("ladf_num", 0):   # luma-adaptive deblocking (captures without the field: off)
        pp.ladf_num = h["ladf_num"]
        for k in range(5):
            pp.ladf_qp_offset[k], pp.ladf_lower_bound[k] = h["ladf_qp_offset%d" % k], h["ladf_lower_bound%d" % k]
    return pp


def plan_picture(p, slot, slot_of, dpb_slots=32, stages=N.STAGE_ALL):
    """Host-only planning of one parsed picture (vvcr_picture_*): returns a planned N.Picture. Runs
    without a device; safe to call for several pictures on several threads."""
    return plan_picture_pp(p, pic_params(p, slot, slot_of), dpb_slots, stages)


def plan_picture_pp(p, pp, dpb_slots=32, stages=N.STAGE_ALL):
    """plan_picture with explicit picture parameters (e.g. a spatial shard's rows)"""
    h = p["hdr"]
    pic = N.Picture(h["width"], h["height"], pp, bit_depth=h["bitdepth_y"],
                    ctu_log2=h["ctu_log2"], dpb_slots=dpb_slots)
    submit(pic, p)
    set_loop_filter_params(pic, p)
    pic.plan(stages)
    return pic


def submit(ctx, p):
    geo = p["geo"] if p["geo"].size else np.zeros((0, 13), np.int32)
    ctx.submit(p["cu"], p["pu"], p["tu"], p["coef"], p["motion"].reshape(-1, 10), geo)


def set_loop_filter_params(ctx, p):
    """SAO / ALF parameters of the picture (as reconstructed by the reference's parameter-set
    handling: SampleAdaptiveOffset::reconstructBlkSAOParams, AdaptiveLoopFilter::reconstructCoeffAPSs)."""
    h = p["hdr"]
    sao = np.ascontiguousarray(p["sao"], np.int32) if "sao" in p else None
    alf = None
    keep = [sao]
    if "alf_ctb_en" in p and h["alf_enabled"]:
        n = len(p["alf_aps_ids"])
        coef = np.ascontiguousarray(np.concatenate([p["alf_fixed"], p["alf_coef_aps"][:n]]), np.int16)
        clip = np.ascontiguousarray(np.concatenate([np.broadcast_to(p["alf_clip_default"], p["alf_fixed"].shape),
                                                    p["alf_clip_aps"][:n]]), np.int16)
        cc_ctl = np.array(p["ccalf_ctl"], np.uint8)
        cc_ctl[0] *= np.uint8(h["ccalf_en_cb"] != 0)     # control words of a disabled component are not coded
        cc_ctl[1] *= np.uint8(h["ccalf_en_cr"] != 0)
        alt = np.array(p["alf_ctb_alt"], np.uint8)
        alt[0] = 0
        arrs = [coef, clip] + [np.ascontiguousarray(p[k], t) for k, t in (
            ("alf_chroma_coef", np.int16), ("alf_chroma_clip", np.int16), ("ccalf_coef", np.int16),
            ("alf_ctb_en", np.uint8))] + [np.ascontiguousarray(alt), np.ascontiguousarray(p["alf_ctb_fidx"], np.int16),
                                         np.ascontiguousarray(cc_ctl)]
        keep += arrs
        alf = N.Alf(16 + n, *(a.ctypes.data for a in arrs))
    ctx.set_loop_filter_params(sao, alf, keep)
