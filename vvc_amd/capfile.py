"""Reader for the per-picture capture files written by oracle/capture/vtm_capture.cpp.

A capture holds the descriptors a host parser hands to the reconstruction path (CU/PU/TU tables,
coefficient levels, motion field, SAO/ALF/LMCS/WP parameters) and, for tests, golden planes of the
reference decoder (prediction, residual, pre-loop-filter / deblocked / SAO / ALF pictures).
Chunk format: 'VVCRCAP1', then repeated {name[24], u32 dtype, u32 ndim, u64 dims[ndim], u64 nbytes, data}.
"""
import numpy as np
import zlib

_DT = {ord('b'): np.int8, ord('B'): np.uint8, ord('h'): np.int16, ord('H'): np.uint16,
       ord('i'): np.int32, ord('q'): np.int64}

# column layouts (must match vtm_capture.cpp enums)
CU_FIELDS = ("x y w h cx cy cw ch chtype predmode qp treetype modetype skip mmvdskip affine affinetype geo "
             "bdpcm bdpcmc imv rootcbf sbtinfo mtsflag lfnst bcw mip isp smvd act cqpadj depth qtdepth firstpu "
             "npu firsttu ntu slice yvalid cvalid").split()
PU_FIELDS = ("cu x y w h cx cy cw ch chtype idir_l idir_c fidir_l fidir_c mipt mrl merge regmerge mergeidx geodir "
             "geoi0 geoi1 mmvd interdir mv0x mv0y mv1x mv1y ref0 ref1 mrgtype mvrefine ciip "
             + " ".join("aff%d" % i for i in range(12)) + " dmvr_off bdof dmvr").split()
TU_FIELDS = ("cu chtype depth noresi jccr cadj " + " ".join(
    "%s%d" % (f, c) for c in range(3) for f in ("x", "y", "w", "h", "cbf", "mts", "coef", "qp", "qpts"))).split()
CU = {n: i for i, n in enumerate(CU_FIELDS)}
PU = {n: i for i, n in enumerate(PU_FIELDS)}
TU = {n: i for i, n in enumerate(TU_FIELDS)}

MODE_INTER, MODE_INTRA, MODE_IBC, MODE_PLT = 0, 1, 2, 3


def parse(buf: bytes) -> dict:
    if buf[:8] != b"VVCRCAP1":
        raise ValueError("not a VVCR capture")
    out, off = {}, 8
    while off < len(buf):
        name = buf[off:off + 24].split(b"\0", 1)[0].decode()
        dt, nd = np.frombuffer(buf, np.uint32, 2, off + 24)
        dims = tuple(int(d) for d in np.frombuffer(buf, np.uint64, nd, off + 32))
        p = off + 32 + 8 * int(nd)
        nb = int(np.frombuffer(buf, np.uint64, 1, p)[0])
        p += 8
        out[name] = np.frombuffer(buf, _DT[int(dt)], nb // np.dtype(_DT[int(dt)]).itemsize, p).reshape(dims).copy()
        off = p + nb
    keys = bytes(out.pop("hdr_keys")).decode().split(",")
    out["hdr"] = dict(zip(keys, (int(v) for v in out.pop("hdr_vals"))))
    return out


def load(path: str) -> dict:
    with open(path, "rb") as f:
        buf = f.read()
    if path.endswith(".z"):
        buf = zlib.decompress(buf)
    return parse(buf)
