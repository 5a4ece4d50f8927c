"""Frame-batched plain MC (vvcr_launch_pictures): the decode loop launches adjacent
independent inter pictures of decoding order together, so ONE k_mc launch carries both pictures' plain MC.

CPU: the grouping rule (vvcp_decode_batches) on the committed streams: no member of a group references an
earlier one (so its derivation never waits for the group's DMVR deltas), all are inter pictures of one
coded video sequence in slots of their own, and the GOP-16 hierarchy groups POC 1/3/6, 5/7/12, 9/11/14, 13/15.
GPU: resident pictures replayed in their launch groups stay MD5-exact; the batched record reports every
picture of its group (pictures = k) and the others none; a batch whose pictures depend on each other is
refused without touching the device (VVCR_E_ARG)."""
import os

import pytest

from vvc_amd import bitstream as B
from vvc_amd import decode as D
from vvc_amd import native as N
from vvc_amd import parser
from vvc_amd import stream as S

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bin(name):
    return open(os.path.join(ROOT, "streams", name + ".bin"), "rb").read()


def _batches(name, nslots=16):
    import ctypes as C
    s = parser.Stream(_bin(name))
    L = B._bind(N.lib())
    n = len(s)
    first = (C.c_int32 * n)()
    pairs = L.vvcp_decode_batches(s.h, 0, nslots, first)
    plan = B.Plan(s, nslots)
    s.close()
    return pairs, list(first), plan


@pytest.mark.parametrize("name", ["ra416_q32", "ra1080l_q32", "ra2160l_q32", "ralm416_q32", "ai416_q37", "ra4320t_q32"])
def test_pairs_are_independent_inter_pictures(name):
    pairs, first, plan = _batches(name)
    assert pairs == sum(1 for f in first if f > 1)
    pocs = [inf["poc"] for inf in plan.info]
    i = 0
    while i < len(first):
        k = first[i]
        assert 1 <= k <= 4
        g = list(range(i, i + k))
        for j in g[1:]:
            assert first[j] == 0
            assert plan.cvs[j] == plan.cvs[i]
            assert plan.slot[j] not in [plan.slot[m] for m in g if m < j], "two members share a slot"
            for m in g:
                if m < j:
                    assert pocs[m] not in plan.refs[j][0] + plan.refs[j][1], "a member references an earlier one"
        if k > 1:
            assert all(plan.info[m]["slice_type"] != 2 for m in g), "intra picture in a batch"
        i += k
    if name.startswith("ai"):
        assert pairs == 0


def test_gop16_top_layer_pairs():
    pairs, first, plan = _batches("ra2160l_q32")
    pocs = [inf["poc"] for inf in plan.info]
    got = [tuple(pocs[i:i + f]) for i, f in enumerate(first) if f > 1]
    assert got == [(1, 3, 6), (5, 7, 12), (9, 11, 14), (13, 15)], got


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ra416_q32", "ra1080_q32"])
def test_batched_groups_replayed_stay_bitexact(name, golden_dir):
    data = _bin(name)
    meta = S.load_meta(os.path.join(golden_dir, name))
    s = parser.Stream(data)
    inf = s.info(0)
    s.close()
    ctx = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=16)
    try:
        seq = B.SequenceDecode(ctx, data, nslots=16, threads=4)
        _, handles = seq.run(keep_handles=True)
        ctx.sync()
        groups = B.launch_groups(handles, seq.batch)
        assert any(len(g) > 1 for g in groups), "no frame-batched group on %s" % name
        owner = {seq.slot[i]: seq.info[i]["poc"] for i in range(len(handles))}
        for rnd in range(2):   # replayed twice: the second round overwrites every slot again
            for g in groups:
                B.launch_group(ctx, g)
            ctx.sync()
            for slot, poc in owner.items():   # (owner: the last picture of decoding order in each slot)
                assert D.plane_md5s([ctx.read_plane(N.BUF_RECO, slot, c) for c in range(3)]) == meta["poc_plane_md5"][str(poc)], \
                    "POC %d after replay %d" % (poc, rnd)
        for g in groups:
            if len(g) > 1:
                st = [dict((x[0], x) for x in ctx.kernel_stats(h)) for h in g]
                assert st[0]["mc"][4] == len(g) and st[0]["mc"][1] <= 1, st[0]["mc"]
                assert all(x["mc"][4] == 0 and x["mc"][1] == 0 for x in st[1:]), [x["mc"] for x in st]
        for h in handles:
            ctx.release(h)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_dependent_batch_is_refused(golden_dir):
    name = "ra416_q32"
    data = _bin(name)
    s = parser.Stream(data)
    inf = s.info(0)
    s.close()
    ctx = N.Context(inf["width"], inf["height"], bit_depth=inf["bit_depth"], ctu_log2=inf["ctu_log2"], dpb_slots=16)
    try:
        seq = B.SequenceDecode(ctx, data, nslots=16, threads=4)
        _, handles = seq.run(keep_handles=True)
        ctx.sync()
        plan = B.Plan(parser.Stream(data), 16)
        pocs = [i["poc"] for i in plan.info]
        # a picture and a later one that references it
        pair = next((i, j) for j in range(1, len(pocs)) for i in range(j)
                    if pocs[i] in plan.refs[j][0] + plan.refs[j][1] and plan.info[i]["slice_type"] != 2)
        with pytest.raises(N.VvcrError, match="references another picture"):
            ctx.launch_batch([handles[pair[0]], handles[pair[1]]])
        with pytest.raises(N.VvcrError):
            ctx.launch_batch([handles[pair[0]], handles[pair[0]]])
        for h in handles:
            ctx.release(h)
    finally:
        ctx.close()
