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
    if "hdr_keys" in out:
        keys = bytes(out.pop("hdr_keys")).decode().split(",")
        out["hdr"] = dict(zip(keys, (int(v) for v in out.pop("hdr_vals"))))
    return out


def load(path: str) -> dict:
    with open(path, "rb") as f:
        buf = f.read()
    if path.endswith(".z"):
        buf = zlib.decompress(buf)
    return parse(buf)


# ------------------------------------------------------------------------------------------------
# compact fixture form (committed under tests/golden/): golden planes are delta-coded along the
# decode pipeline (pred -> residual -> pre-LF recon -> DBK -> SAO -> ALF) and the whole picture is
# an lzma-compressed .npz (loaded with allow_pickle=False).
# ------------------------------------------------------------------------------------------------
import io
import lzma

_CHAIN = [("pmc", "pfin"), ("dbkin", "prelf"), ("dbk", "dbkin"), ("sao", "dbk"), ("alf", "sao")]


def _recon_guess(pic, c, bd=10):
    pf = pic["pfin_" + c].astype(np.int32)
    pf = np.where(pf == -32768, 0, pf)
    return np.clip(pf + pic["resi_" + c], 0, (1 << bd) - 1)


def pack(pic: dict) -> bytes:
    arrs = {}
    for k, v in pic.items():
        if k == "hdr":
            continue
        arrs[k] = v
    for c in "yuv":
        if "prelf_" + c in pic:
            arrs["prelf_" + c] = (pic["prelf_" + c].astype(np.int32) - _recon_guess(pic, c)).astype(np.int16)
        for dst, src in _CHAIN:
            if dst + "_" + c in pic and src + "_" + c in pic:
                arrs[dst + "_" + c] = (pic[dst + "_" + c].astype(np.int32) - pic[src + "_" + c]).astype(np.int16)
    arrs["hdr_keys"] = np.frombuffer(",".join(pic["hdr"].keys()).encode(), np.uint8)
    arrs["hdr_vals"] = np.array(list(pic["hdr"].values()), np.int64)
    bio = io.BytesIO()
    np.savez(bio, **arrs)
    return lzma.compress(bio.getvalue(), preset=9)


def unpack(blob: bytes) -> dict:
    z = np.load(io.BytesIO(lzma.decompress(blob)), allow_pickle=False)
    pic = {k: z[k] for k in z.files}
    keys = bytes(pic.pop("hdr_keys")).decode().split(",")
    pic["hdr"] = dict(zip(keys, (int(v) for v in pic.pop("hdr_vals"))))
    for c in "yuv":
        if "prelf_" + c in pic:
            pic["prelf_" + c] = (pic["prelf_" + c].astype(np.int32) + _recon_guess(pic, c)).astype(np.int16)
        for dst, src in _CHAIN:
            if dst + "_" + c in pic and src + "_" + c in pic:
                pic[dst + "_" + c] = (pic[dst + "_" + c].astype(np.int32) + pic[src + "_" + c]).astype(np.int16)
    return pic


def load_any(path: str) -> dict:
    if path.endswith(".xz"):
        with open(path, "rb") as f:
            return unpack(f.read())
    return load(path)
