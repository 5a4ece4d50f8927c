"""Spatial sharding across processes: a tile-row stream decoded by 2 or 3 ranks, one process each, over
torch.distributed (gloo: the rows go through host tensors, staged to and from the GPU by TorchComm; with
nccl = RCCL the same calls take device tensors), all on the box's one GPU. Every rank reconstructs and
filters only its own rows (vvcr_pic_params::shard_y0/shard_y1), swaps the loop-filter halo and the
reference halo with its neighbours (vvc_amd/shard.py decode_picture) and sends its rows to rank 0, which
holds the assembled picture: its plane MD5s must equal the reference decoder's for every picture."""
import datetime
import json
import os

import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rank_main(rank, world, port, name, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vvc_amd import decode as D
    from vvc_amd import native as N
    from vvc_amd import shard as SH
    from vvc_amd import stream as S
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        pics = S.load_sequence(os.path.join(GOLD, name))
        h0 = pics[0]["hdr"]
        slots = 8
        ctx = N.Context(h0["width"], h0["height"], bit_depth=h0["bitdepth_y"], ctu_log2=h0["ctu_log2"], dpb_slots=slots)
        try:
            rk = SH.ShardRank(ctx, pics, rank, world, slots)
            comm = SH.TorchComm("cpu")
            M = SH.plan_and_reach([rk], comm)
            md5 = {}
            for i, p in enumerate(pics):
                SH.decode_picture(rk, comm, i)
                SH.gather_to_root(rk, comm, rk.slots[i])
                if rank == 0:
                    md5[str(p["hdr"]["poc"])] = D.plane_md5s([ctx.read_plane(N.BUF_RECO, rk.slots[i], c) for c in range(3)])
            rk.release()
        finally:
            ctx.close()
        if rank == 0:
            with open(out, "w") as f:
                json.dump({"reach": M, "rows": rk.rows, "md5": md5}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("ratile416_q32", 2), ("ratile1080_q32", 3)])
def test_multiprocess_sharded_decode_matches_reference(tmp_path, name, world):
    import torch.multiprocessing as mp
    from vvc_amd import stream as S
    out = str(tmp_path / "md5.json")
    port = 29600 + (os.getpid() * 7 + world) % 2000
    mp.start_processes(_rank_main, args=(world, port, name, out), nprocs=world, start_method="spawn")
    got = json.load(open(out))
    meta = S.load_meta(os.path.join(GOLD, name))
    assert len(got["rows"]) == world
    assert got["md5"] == meta["poc_plane_md5"]


def _stream_rank_main(rank, world, port, name, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vvc_amd import decode as D
    from vvc_amd import native as N
    from vvc_amd import parser as PZ
    from vvc_amd import shard as SH
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        data = open(os.path.join(GOLD, "streams", name + ".bin"), "rb").read()
        ps = PZ.Stream(data)
        inf = ps.info(0)
        ps.close()
        slots = 8
        ctx = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=slots)
        try:
            rk = SH.StreamShardRank(ctx, data, rank, world, slots)
            comm = SH.TorchComm("cpu")
            md5 = {}
            for i in range(rk.n):
                SH.decode_stream_picture(rk, comm, i)
                SH.gather_to_root(rk, comm, rk.slots[i])
                if rank == 0:
                    md5[str(rk.info[i]["poc"])] = D.plane_md5s([ctx.read_plane(N.BUF_RECO, rk.slots[i], c) for c in range(3)])
            reach = rk.reach
            rk.release()
        finally:
            ctx.close()
        if rank == 0:
            with open(out, "w") as f:
                json.dump({"reach": reach, "rows": rk.rows, "md5": md5}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("ratile416_q32", 2), ("ratile1080_q32", 3)])
def test_multiprocess_sharded_decode_from_bitstream(tmp_path, name, world):
    """BASELINE config 4 from the .bin: one process per rank over torch.distributed (gloo), each parsing
    the stream itself and reconstructing its own tile rows; rank 0's assembled pictures match DecoderApp."""
    import torch.multiprocessing as mp
    from vvc_amd import stream as S
    out = str(tmp_path / "md5.json")
    port = 29700 + (os.getpid() * 11 + world) % 2000
    mp.start_processes(_stream_rank_main, args=(world, port, name, out), nprocs=world, start_method="spawn")
    got = json.load(open(out))
    meta = S.load_meta(os.path.join(GOLD, name))
    assert len(got["rows"]) == world
    assert got["md5"] == meta["poc_plane_md5"]
