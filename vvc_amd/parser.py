"""Host bitstream parser of libvvcr (include/vvcp.h) through ctypes.

Stream(data) opens an Annex-B VVC bitstream (all NAL units and headers are read at once); parse(i)
runs the CABAC pass of picture i (decoding order) and rows(i) returns its descriptor rows as numpy
arrays shaped like the capture records (vvc_amd/capfile.py): cu (N, 40), pu (N, 48), tu (N, 33) int32,
coef, sao (n_ctb, 3, 35) and the ALF CTB arrays. derive(i) then resolves the motion of picture i
(decoding order; every earlier picture refined first) and refine(i, deltas) records its motion after
DMVR for later pictures' temporal candidates; rows(i) then also holds motion (h/4, w/4, 10) and geo.
"""
import ctypes as C

import numpy as np

from . import native as N

ROWS_CU, ROWS_PU, ROWS_TU, ROWS_COEF, ROWS_SAO = 0, 1, 2, 3, 4
ROWS_ALF_EN0, ROWS_ALF_ALT0, ROWS_ALF_FSET, ROWS_CCALF0 = 5, 8, 11, 12
ROWS_MOTION, ROWS_GEO = 14, 15

_P, _I32, _I64 = C.c_void_p, C.c_int32, C.c_int64


def _bind(lib):
    if getattr(lib, "_vvcp_bound", False):
        return lib
    lib.vvcp_open.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(_P)]
    lib.vvcp_open.restype = C.c_int
    lib.vvcp_close.argtypes = [_P]
    lib.vvcp_last_error.restype = C.c_char_p
    lib.vvcp_num_pictures.argtypes = [_P]
    lib.vvcp_picture_info.argtypes = [_P, _I32, C.POINTER(_I32), _I32]
    lib.vvcp_parse_picture.argtypes = [_P, _I32]
    lib.vvcp_picture_rows.argtypes = [_P, _I32, _I32, _P, _I64]
    lib.vvcp_picture_rows.restype = _I64
    lib.vvcp_picture_params.argtypes = [_P, _I32, _P]
    lib.vvcp_alf_filters.argtypes = [_P, _I32, _P, _P, _I32, _P, _P, _P]
    lib.vvcp_derive_motion.argtypes = [_P, _I32]
    lib.vvcp_refine_motion.argtypes = [_P, _I32, _P, _I64]
    lib.vvcp_set_parse_rows.argtypes = [_P, _I32, _I32]
    lib.vvcp_dmvr_split.argtypes = [_P, _I32, _I32, _I32, C.POINTER(_I64)]
    lib._vvcp_bound = True
    return lib


class ParseError(RuntimeError):
    pass


class Stream:
    def __init__(self, data, lib=None):
        self.lib = _bind(lib or N.lib())
        self._data = bytes(data)
        h = _P()
        rc = self.lib.vvcp_open(self._data, len(self._data), C.byref(h))
        if rc != 0:
            raise ParseError("vvcp_open: %s" % self.lib.vvcp_last_error().decode())
        self.h = h

    def close(self):
        if self.h:
            self.lib.vvcp_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.lib.vvcp_num_pictures(self.h)

    def info(self, i):
        v = (_I32 * 16)()
        self.lib.vvcp_picture_info(self.h, i, v, 16)
        keys = ("poc", "slice_type", "width", "height", "ctu_log2", "bit_depth", "num_slices", "tid", "nal_type", "slice_qp",
                "conf_left", "conf_right", "conf_top", "conf_bottom", "output", "non_ref")
        return dict(zip(keys, list(v)))

    def parse(self, i):
        rc = self.lib.vvcp_parse_picture(self.h, i)
        if rc != 0:
            raise ParseError("picture %d: %s" % (i, self.lib.vvcp_last_error().decode()))

    def set_parse_rows(self, y0, y1):
        """later CABAC passes cover only the tiles holding luma rows [y0, y1) (vvcp_set_parse_rows)"""
        if self.lib.vvcp_set_parse_rows(self.h, int(y0), int(y1)) != 0:
            raise ParseError("vvcp_set_parse_rows")

    def dmvr_split(self, i, y0, y1):
        """(above, inside, below): delta rows of picture i's parsed DMVR PUs around luma rows [y0, y1)"""
        v = (_I64 * 3)()
        rc = self.lib.vvcp_dmvr_split(self.h, i, int(y0), int(y1), v)
        if rc != 0:
            raise ParseError("picture %d dmvr_split: %d" % (i, rc))
        return int(v[0]), int(v[1]), int(v[2])

    def derive(self, i):
        rc = self.lib.vvcp_derive_motion(self.h, i)
        if rc != 0:
            raise ParseError("picture %d motion: %s" % (i, self.lib.vvcp_last_error().decode()))

    def refine(self, i, deltas=None):
        d = None if deltas is None or len(deltas) == 0 else np.ascontiguousarray(deltas, np.int32).reshape(-1, 2)
        rc = self.lib.vvcp_refine_motion(self.h, i, None if d is None else d.ctypes.data, 0 if d is None else len(d))
        if rc != 0:
            raise ParseError("picture %d refine: %s" % (i, self.lib.vvcp_last_error().decode()))

    def pic_params(self, i):
        """vvcr_pic_params of picture i (N.PicParams) without the DPB slots"""
        pp = N.PicParams()
        rc = self.lib.vvcp_picture_params(self.h, i, C.addressof(pp))
        if rc != 0:
            raise ParseError("picture %d params: %s" % (i, self.lib.vvcp_last_error().decode()))
        return pp

    def alf_filters(self, i):
        """ALF / CC-ALF filters of picture i: luma_coef / luma_clip (sets, 25, 13), chroma_coef /
        chroma_clip (8, 7), cc_coef (2, 4, 8)"""
        n = self.lib.vvcp_alf_filters(self.h, i, None, None, 0, None, None, None)
        if n < 0:
            raise ParseError("picture %d ALF: %s" % (i, self.lib.vvcp_last_error().decode()))
        out = {"luma_coef": np.zeros((n, 25, 13), np.int16), "luma_clip": np.zeros((n, 25, 13), np.int16),
               "chroma_coef": np.zeros((8, 7), np.int16), "chroma_clip": np.zeros((8, 7), np.int16),
               "cc_coef": np.zeros((2, 4, 8), np.int16)}
        self.lib.vvcp_alf_filters(self.h, i, *(out[k].ctypes.data for k in ("luma_coef", "luma_clip")), n,
                                  *(out[k].ctypes.data for k in ("chroma_coef", "chroma_clip", "cc_coef")))
        return out

    def _rows(self, i, what, dtype, shape_tail):
        n = self.lib.vvcp_picture_rows(self.h, i, what, None, 0)
        if n < 0:
            raise ParseError("rows: %d" % n)
        esz = int(np.prod(shape_tail)) if shape_tail else 1
        out = np.zeros((n * esz,), dtype)
        if n:
            self.lib.vvcp_picture_rows(self.h, i, what, out.ctypes.data, n)
        return out.reshape((n,) + tuple(shape_tail)) if shape_tail else out

    def rows(self, i):
        r = {
            "cu": self._rows(i, ROWS_CU, np.int32, (40,)),
            "pu": self._rows(i, ROWS_PU, np.int32, (48,)),
            "tu": self._rows(i, ROWS_TU, np.int32, (33,)),
            "coef": self._rows(i, ROWS_COEF, np.int32, ()),
            "sao": self._rows(i, ROWS_SAO, np.int32, (35,)),
            "alf_ctb_fidx": self._rows(i, ROWS_ALF_FSET, np.int16, ()),
        }
        r["sao"] = r["sao"].reshape(-1, 3, 35)
        r["alf_ctb_en"] = np.stack([self._rows(i, ROWS_ALF_EN0 + c, np.uint8, ()) for c in range(3)])
        r["alf_ctb_alt"] = np.stack([self._rows(i, ROWS_ALF_ALT0 + c, np.uint8, ()) for c in range(3)])
        r["ccalf_ctl"] = np.stack([self._rows(i, ROWS_CCALF0 + c, np.uint8, ()) for c in range(2)])
        if self.lib.vvcp_picture_rows(self.h, i, ROWS_MOTION, None, 0) >= 0:
            inf = self.info(i)
            r["motion"] = self._rows(i, ROWS_MOTION, np.int32, (10,)).reshape((inf["height"] + 3) // 4, (inf["width"] + 3) // 4, 10)
            r["geo"] = self._rows(i, ROWS_GEO, np.int32, (13,))
        return r
