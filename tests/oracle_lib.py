"""Loader for the C oracle (oracle/_build/liboracle.so) — the CPU checker. Tables are the reference's
own constants (tests/golden/tables.cap, dumped from the running reference by oracle/capture)."""
import ctypes as C
import os

import numpy as np

from vvc_amd import capfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = None
_keep = []


class OrTables(C.Structure):
    _fields_ = [("dct2", C.c_void_p * 7), ("dst7", C.c_void_p * 6), ("dct8", C.c_void_p * 6),
                ("lfnst8x8", C.c_void_p), ("lfnst4x4", C.c_void_p), ("lfnst_lut", C.c_void_p),
                ("inv_quant_scales", C.c_void_p)]


class OrPic(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("width", "height", "bit_depth", "dep_quant", "joint_cbcr_sign", "use_mts",
                                       "implicit_mts", "mts_intra", "mts_inter", "lfnst_enabled", "dual_tree")]


def tables():
    return capfile.load(os.path.join(ROOT, "tests", "golden", "tables.cap"))


def lib():
    global _lib
    if _lib is None:
        from vvc_amd import build
        path = build.build_oracle()
        L = C.CDLL(path)
        t = tables()
        ot = OrTables()

        def keep(a):
            a = np.ascontiguousarray(a, np.int16)
            _keep.append(a)
            return a.ctypes.data

        for l in range(1, 7):
            ot.dct2[l] = keep(t["dct2_%d" % (1 << l)])
        for l in range(2, 6):
            ot.dst7[l] = keep(t["dst7_%d" % (1 << l)])
            ot.dct8[l] = keep(t["dct8_%d" % (1 << l)])
        ot.lfnst8x8 = keep(t["lfnst8x8"])
        ot.lfnst4x4 = keep(t["lfnst4x4"])
        ot.lfnst_lut = keep(t["lfnst_lut"])
        ot.inv_quant_scales = keep(t["inv_quant_scales"])
        _keep.append(ot)
        L.or_set_tables(C.byref(ot))
        _lib = L
    return _lib


def pic_struct(p):
    h = p["hdr"]
    return OrPic(h["width"], h["height"], h["bitdepth_y"], h["dep_quant"], h.get("joint_cbcr_sign", 0), h.get("use_mts", 1),
                 h.get("implicit_mts", 0), h["mts_intra"], h["mts_inter"], h["lfnst_enabled"], h["dual_tree"])


def residual_picture(p):
    L = lib()
    h = p["hdr"]
    W, H = h["width"], h["height"]
    planes = [np.zeros((H, W), np.int16), np.zeros((H // 2, W // 2), np.int16), np.zeros((H // 2, W // 2), np.int16)]
    cu, pu, tu, coef = (np.ascontiguousarray(p[k], np.int32) for k in ("cu", "pu", "tu", "coef"))
    ps = pic_struct(p)
    P = C.c_void_p
    r = L.or_residual_picture(C.byref(ps), P(cu.ctypes.data), len(cu), P(pu.ctypes.data), len(pu), P(tu.ctypes.data), len(tu),
                              P(coef.ctypes.data), C.c_int64(coef.size), *(P(x.ctypes.data) for x in planes))
    assert r == 0, r
    return planes


def _p(a):
    return C.c_void_p(a.ctypes.data)


def alf_luma_sets(p):
    """luma filter sets of the picture: 16 fixed sets then the slice's APS sets (reconstructCoeffAPSs)."""
    n = len(p["alf_aps_ids"])
    coef = np.concatenate([p["alf_fixed"], p["alf_coef_aps"][:n]]).astype(np.int16)
    clip = np.concatenate([np.broadcast_to(p["alf_clip_default"], p["alf_fixed"].shape), p["alf_clip_aps"][:n]]).astype(np.int16)
    return np.ascontiguousarray(coef), np.ascontiguousarray(clip)


def sao_picture(p, planes):
    L = lib()
    h = p["hdr"]
    out = [np.empty_like(x) for x in planes]
    src = [np.ascontiguousarray(x, np.int16) for x in planes]
    sao = np.ascontiguousarray(p["sao"], np.int32)
    L.or_sao_picture(h["width"], h["height"], h["bitdepth_y"], h["ctu_log2"], _p(sao), *(_p(x) for x in src), *(_p(x) for x in out))
    return out


def alf_picture(p, planes):
    L = lib()
    h = p["hdr"]
    out = [np.empty_like(x) for x in planes]
    src = [np.ascontiguousarray(x, np.int16) for x in planes]
    coef, clip = alf_luma_sets(p)
    cc = np.ascontiguousarray(p["alf_chroma_coef"], np.int16)
    ccl = np.ascontiguousarray(p["alf_chroma_clip"], np.int16)
    ccf = np.ascontiguousarray(p["ccalf_coef"], np.int16)
    en = np.array([h["alf_slice_en0"], h["alf_slice_en1"], h["alf_slice_en2"], h["ccalf_en_cb"], h["ccalf_en_cr"]], np.int32)
    cte = np.ascontiguousarray(p["alf_ctb_en"], np.uint8)
    cta = np.ascontiguousarray(p["alf_ctb_alt"], np.uint8)
    cts = np.ascontiguousarray(p["alf_ctb_fidx"], np.int16)
    ccc = np.ascontiguousarray(p["ccalf_ctl"], np.uint8)
    L.or_alf_picture(h["width"], h["height"], h["bitdepth_y"], h["ctu_log2"], h["alf_vb_luma"], h["alf_vb_chroma"],
                     _p(coef), _p(clip), _p(cc), _p(ccl), _p(ccf), _p(en), _p(cte), _p(cta), _p(cts), _p(ccc),
                     *(_p(x) for x in src), *(_p(x) for x in out))
    return out


class OrDbkIn(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("width", "height", "bd", "ctu_log2", "dual_tree", "slice_type", "disable",
                                       "beta_offset_div2", "tc_offset_div2")] + [
        ("chroma_qp_off", C.c_int * 3), ("chroma_qp_map", C.c_void_p), ("chroma_qp_map_jc", C.c_void_p),
        ("ref_poc", C.c_void_p), ("tc_table", C.c_void_p), ("beta_table", C.c_void_p),
        ("cu", C.c_void_p), ("ncu", C.c_int), ("pu", C.c_void_p), ("npu", C.c_int), ("tu", C.c_void_p), ("ntu", C.c_int),
        ("motion", C.c_void_p)]


def deblock_picture(p, planes):
    """LoopFilter::loopFilterPic restated (oracle_dbk.c); returns new planes."""
    L = lib()
    h = p["hdr"]
    t = tables()
    out = [np.ascontiguousarray(x, np.int16).copy() for x in planes]
    arrs = dict(cqm=np.ascontiguousarray(p["chroma_qp_map"], np.int32), jc=np.ascontiguousarray(p["chroma_qp_map_jc"], np.int32),
                ref=np.ascontiguousarray(p["ref_poc"], np.int32), tc=np.ascontiguousarray(t["dbk_tc"], np.int16),
                beta=np.ascontiguousarray(t["dbk_beta"], np.int16), cu=np.ascontiguousarray(p["cu"], np.int32),
                pu=np.ascontiguousarray(p["pu"], np.int32), tu=np.ascontiguousarray(p["tu"], np.int32),
                mf=np.ascontiguousarray(p["motion"], np.int32))
    d = OrDbkIn(h["width"], h["height"], h["bitdepth_y"], h["ctu_log2"], h["dual_tree"], h["slice_type"], h["dbk_disable"],
                h["dbk_beta_offset_div2"], h["dbk_tc_offset_div2"])
    d.chroma_qp_off[0], d.chroma_qp_off[1], d.chroma_qp_off[2] = h["chroma_qp_off_cb"], h["chroma_qp_off_cr"], h["chroma_qp_off_jc"]
    d.chroma_qp_map, d.chroma_qp_map_jc = arrs["cqm"].ctypes.data, arrs["jc"].ctypes.data
    d.ref_poc, d.tc_table, d.beta_table = arrs["ref"].ctypes.data, arrs["tc"].ctypes.data, arrs["beta"].ctypes.data
    d.cu, d.ncu = arrs["cu"].ctypes.data, len(arrs["cu"])
    d.pu, d.npu = arrs["pu"].ctypes.data, len(arrs["pu"])
    d.tu, d.ntu = arrs["tu"].ctypes.data, len(arrs["tu"])
    d.motion = arrs["mf"].ctypes.data
    r = L.or_deblock_picture(C.byref(d), *(_p(x) for x in out))
    assert r == 0, r
    return out


def write_output(planes, bd, file_bd=0, conf=(0, 0, 0, 0), clip709=0):
    """DecoderApp's output frame of one picture (oracle_output.c) as a uint8 array"""
    L = lib()
    y, u, v = (np.ascontiguousarray(x, np.int16) for x in planes)
    h, w = y.shape
    fbd = file_bd or bd
    out = np.zeros(((2 if fbd > 8 else 1) * (w * h + 2 * (w // 2) * (h // 2)),), np.uint8)
    L.or_write_output.restype = C.c_int64
    n = L.or_write_output(w, h, bd, _p(y), _p(u), _p(v), w, w // 2, file_bd, *conf, clip709, _p(out))
    assert n == out.size
    return out
