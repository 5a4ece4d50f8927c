"""Spatial sharding on the GPU: the tile-row streams decoded by 2..9 emulated ranks (one libvvcr context
each, in this process; rows pass between them through device buffers exactly as the RCCL path hands
them to send / recv), every rank reconstructing and filtering only its own rows. The pictures
assembled from the ranks' own rows must match the reference decoder's MD5s bit for bit."""
import os

import pytest

from vvc_amd import decode as D
from vvc_amd import native as N
from vvc_amd import shard as SH
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,world", [("ratile416_q32", 2), ("ratile1080_q32", 2), ("ratile1080_q32", 4), ("ratile1080_q32", 9),
                                        ("ra4320t_q32", 8)])
def test_sharded_decode_matches_reference_md5(golden_dir, name, world):
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    h0 = pics[0]["hdr"]
    slots = 8
    ctxs = [N.Context(h0["width"], h0["height"], bit_depth=h0["bitdepth_y"], ctu_log2=h0["ctu_log2"], dpb_slots=slots)
            for _ in range(world)]
    try:
        ranks = [SH.ShardRank(ctxs[r], pics, r, world, slots) for r in range(world)]
        M = SH.plan_and_reach(ranks)
        comm = SH.LocalComm()
        for i, p in enumerate(pics):
            SH.decode_local(ranks, comm, i)
            got = D.plane_md5s(SH.assemble(ranks, i))
            assert got == meta["poc_plane_md5"][str(p["hdr"]["poc"])], "POC %d (world %d, reach %d)" % (p["hdr"]["poc"], world, M)
        for rk in ranks:
            rk.release()
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("name,world,ordered", [("ratile416_q32", 2, False), ("ratile1080_q32", 3, False), ("ratile1080_q32", 9, False),
                                                ("ra4320t_q32", 8, False), ("ratile1080_q32", 3, True), ("ra4320t_q32", 4, True)])
def test_sharded_decode_from_bitstream_matches_reference_md5(golden_dir, name, world, ordered):
    """The product path of BASELINE config 4: every emulated rank parses the tiles around its rows of the
    .bin itself (vvcp), all-gathers the DMVR deltas of each reference, derives, plans and reconstructs its
    own tile rows only; the assembled pictures match the reference decoder's MD5s. ordered: the halo rows
    move through stream-ordered copies without host synchronisation (the RCCL path's exchange)."""
    meta = S.load_meta(os.path.join(golden_dir, name))
    data = open(os.path.join(golden_dir, "streams", name + ".bin"), "rb").read()
    from vvc_amd import parser as PZ
    ps = PZ.Stream(data)
    inf = ps.info(0)
    ps.close()
    slots = 8
    ctxs = [N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=slots)
            for _ in range(world)]
    try:
        ranks = [SH.StreamShardRank(ctxs[r], data, r, world, slots) for r in range(world)]
        comm = SH.LocalComm(ordered=ordered)
        for i in range(ranks[0].n):
            SH.decode_stream_local(ranks, comm, i)
            got = D.plane_md5s(SH.assemble(ranks, i))
            poc = ranks[0].info[i]["poc"]
            assert got == meta["poc_plane_md5"][str(poc)], "POC %d (world %d, reach %d)" % (poc, world, max(r.reach for r in ranks))
        for rk in ranks:
            rk.release()
    finally:
        for c in ctxs:
            c.close()
