"""Spatial sharding (vvc_amd/shard.py), host side: shard rows on tile rows, the halo exchange lists,
and the point-to-point exchange itself over torch.distributed gloo with two ranks on the CPU (a
stand-in context holds the DPB planes in host memory; the GPU path is tests/test_shard_gpu.py)."""
import ctypes
import os

import numpy as np
import pytest

from vvc_amd import shard as SH
from vvc_amd import stream as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_shard_rows_are_whole_tile_rows():
    p = S.load_sequence(os.path.join(GOLD, "ratile1080_q32"), max_pics=1)[0]
    ctu = 1 << p["hdr"]["ctu_log2"]
    bd = set(int(v) * ctu for v in p["tile_row_bd"]) | {p["hdr"]["height"]}
    for world in (1, 2, 3, 4, 8, 9):
        rows = SH.shard_rows(p, world)
        assert rows[0][0] == 0 and rows[-1][1] == p["hdr"]["height"]
        assert all(rows[k][1] == rows[k + 1][0] for k in range(world - 1))
        assert all(a in bd and b in bd and b > a for a, b in rows)
    with pytest.raises(ValueError):
        SH.shard_rows(p, 10)


def test_exchange_lists_pair_up():
    rows = [(0, 256), (256, 384), (384, 1080)]
    g = [SH.ShardGeom(None, r, rows, M=64) for r in range(3)]
    for halo in ("lf_halo", "ref_halo"):
        for r in range(3):
            sends, _ = getattr(g[r], halo)()
            for peer, y0, n in sends:
                _, recvs = getattr(g[peer], halo)()
                assert (r, y0, n) in recvs   # what r sends is what the peer expects, row for row
                assert rows[r][0] <= y0 and y0 + n <= rows[r][1]   # only own rows leave a rank
    # a reach beyond the shortest shard: every rank sends its rows to every other one
    g = [SH.ShardGeom(None, r, rows, M=200) for r in range(3)]
    sends, recvs = g[1].ref_halo()
    assert sorted(p for p, _, _ in sends) == [0, 2] and (0, 0, 256) in recvs and (2, 384, 696) in recvs


class HostCtx:
    """stand-in for N.Context over host memory: a DPB slot of three int16 planes"""

    def __init__(self, W, H, slots=2):
        self.W, self.H = W, H
        self.planes = [[np.zeros((H >> (c > 0), W >> (c > 0)), np.int16) for c in range(3)] for _ in range(slots)]

    def rows_bytes(self, n):
        return n * self.W * 2 + 2 * (n // 2) * (self.W // 2) * 2

    def _rows(self, slot, y0, n):
        return [self.planes[slot][c][(y0 >> (c > 0)):((y0 + n) >> (c > 0))] for c in range(3)]

    def export_rows(self, slot, y0, n, ptr):
        data = np.concatenate([r.ravel() for r in self._rows(slot, y0, n)]).astype(np.int16)
        ctypes.memmove(ptr, data.ctypes.data, data.nbytes)

    def import_rows(self, slot, y0, n, ptr):
        rows = self._rows(slot, y0, n)
        tot = sum(r.size for r in rows)
        data = np.frombuffer(ctypes.string_at(ptr, tot * 2), np.int16)
        o = 0
        for r in rows:
            r[...] = data[o:o + r.size].reshape(r.shape)
            o += r.size


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = [(0, 64), (64, 160)]
        W, H = 96, 160
        ctx = HostCtx(W, H)
        y0, y1 = rows[rank]
        val = 100 * (rank + 1)
        for c in range(3):   # own rows: rank-specific, row-dependent values; the rest: -1
            pl = ctx.planes[0][c]
            pl[:] = -1
            s = c > 0
            for y in range(y0 >> s, y1 >> s):
                pl[y] = val + y + 10 * c
        rk = SH.ShardGeom(ctx, rank, rows, M=32)
        comm = SH.TorchComm("cpu", host_rows=True)
        SH.exchange(rk, comm, rk.lf_halo(), 0)
        lf = [ctx.planes[0][c].copy() for c in range(3)]
        SH.exchange(rk, comm, rk.ref_halo(), 0)
        np.save(out % rank, np.concatenate([p.ravel() for p in lf] + [p.ravel() for p in ctx.planes[0]]))
    finally:
        dist.destroy_process_group()


def test_halo_exchange_over_gloo(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "r%d.npy")
    mp.start_processes(_worker, args=(2, 29500 + os.getpid() % 1000, out), nprocs=2, start_method="spawn")
    W, H = 96, 160
    sizes = [H * W, (H // 2) * (W // 2), (H // 2) * (W // 2)]
    for rank, (y0, y1), peer_val, (h0, h1) in ((0, (0, 64), 200, (64, 88)), (1, (64, 160), 100, (40, 64))):
        d = np.load(out % rank)
        lf = np.split(d[:sum(sizes)], np.cumsum(sizes)[:-1])
        ref = np.split(d[sum(sizes):], np.cumsum(sizes)[:-1])
        for c in range(3):
            s = 1 if c else 0
            pl = lf[c].reshape(H >> s, W >> s)
            for y in range(h0 >> s, h1 >> s):       # the 24 pre-filter halo rows came from the neighbour
                assert (pl[y] == peer_val + y + 10 * c).all(), (rank, c, y)
            rp = ref[c].reshape(H >> s, W >> s)
            m0, m1 = ((64, 96) if rank == 0 else (32, 64))
            for y in range(m0 >> s, m1 >> s):        # the 32 reference rows (reach) likewise
                assert (rp[y] == peer_val + y + 10 * c).all(), (rank, c, y)
            for y in range(y0 >> s, y1 >> s):        # own rows untouched
                assert (rp[y] == 100 * (rank + 1) + y + 10 * c).all()


def _gather_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = SH.TorchComm("cpu", host_rows=True)
        mine = np.arange(2 * (3 * rank), dtype=np.int32).reshape(-1, 2) + 1000 * rank   # rank 0 holds none
        parts = comm.all_gather_rows(mine)
        np.save(out % rank, np.concatenate(parts) if parts else np.zeros((0, 2), np.int32))
        np.save((out % rank) + ".n.npy", np.array([len(p) for p in parts]))
    finally:
        dist.destroy_process_group()


def test_dmvr_delta_all_gather_over_gloo(tmp_path):
    """The bitstream-driven shard ranks all-gather their DMVR deltas (rank order = the picture's PU order):
    variable counts, including a rank with none, arrive whole and in order on every rank."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "g%d.npy")
    mp.start_processes(_gather_worker, args=(3, 29900 + os.getpid() % 1000, out), nprocs=3, start_method="spawn")
    exp = np.concatenate([np.arange(2 * (3 * r), dtype=np.int32).reshape(-1, 2) + 1000 * r for r in range(3)])
    for r in range(3):
        assert np.array_equal(np.load(out % r), exp)
        assert list(np.load((out % r) + ".n.npy")) == [0, 3, 6]


def test_stream_shard_rows_follow_the_tile_rows():
    """StreamShardRank takes its rows from the parsed tile rows of the .bin (vvcp_picture_params)."""
    from vvc_amd import parser as PZ
    data = open(os.path.join(GOLD, "streams", "ra4320t_q32.bin"), "rb").read()
    ps = PZ.Stream(data)
    inf = ps.info(0)
    pp = ps.pic_params(0)
    ps.close()
    p = S.load_sequence(os.path.join(GOLD, "ra4320t_q32"), max_pics=1)[0]
    for world in (1, 2, 4, 8):
        assert SH.stream_shard_rows(pp, inf["height"], inf["ctu_log2"], world) == SH.shard_rows(p, world)
