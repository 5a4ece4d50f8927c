"""End-to-end parity: every picture of each stream reconstructed by libvvcr from its descriptors alone
(references are libvvcr's own output in its device DPB) matches the reference decoder's output
picture MD5s (= the stream's decoded-picture-hash SEI) and the MD5 of DecoderApp's YUV file."""
import os

import pytest

from vvc_amd import decode as D
from vvc_amd import stream as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32", "ra1080_q32", "ailm416_q37", "ralm416_q32", "rawp416_q32", "ratile416_q32", "ratile1080_q32",
                                  "ra2160_q27", "ra2160_q32", "ra1080l_q32",
                                  "rageo480_q32", "radq0416_q32", "aibdpcm416_q32", "rawp1080_q32", "ralmgeo416_q32",
                                  "rawpp416_q32", "ratilenf416_q32"])
def test_decode_matches_reference_md5(golden_dir, name):
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    md5, yuv = D.decode_and_hash(pics)
    for poc, exp in meta["poc_plane_md5"].items():
        assert md5[int(poc)] == exp, "POC %s: plane MD5 %s != reference %s" % (poc, md5[int(poc)], exp)
    assert yuv == meta["yuv_md5"]


@pytest.mark.parametrize("lanes", ["4", "7"])
@pytest.mark.parametrize("name", ["ra416_q32", "ra1080_q32"])
def test_concurrent_segments_match_reference_md5(golden_dir, name, lanes, monkeypatch):
    """Two copies of the stream on disjoint DPB slots, every picture launched back to back with no host
    synchronisation in between: the execution lanes run pictures concurrently, ordered only by their
    slot dependencies (vvcr_api.cpp launch), and every picture of both copies must still be bit-exact."""
    from vvc_amd import native as N
    monkeypatch.setenv("VVCR_LANES", lanes)   # read by vvcr_create
    d = os.path.join(golden_dir, name)
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    n = len(pics)
    per = min(n, 16)                                   # 2 copies within the 32 DPB slots
    dec = D.Decoder(pics, dpb_slots=2 * per)
    ctx = dec.ctx
    try:
        copies = []
        for c in range(2):
            alloc = S.SlotAllocator(pics, per, base=per * c)
            hs = []
            for i, p in enumerate(pics):
                slot = alloc.assign(i, p["hdr"]["poc"])
                ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
                S.submit(ctx, p)
                S.set_loop_filter_params(ctx, p)
                hs.append((ctx.prepare(N.STAGE_ALL), p["hdr"]["poc"], slot))
            copies.append(hs)
        for rnd in range(2):
            for i in range(n):                      # interleaved: copy 0 picture i, copy 1 picture i
                for hs in copies:
                    ctx.launch(hs[i][0])
            ctx.sync()
            for hs in copies:
                owner = {slot: poc for _, poc, slot in hs}   # the last picture written to each slot
                for slot, poc in owner.items():
                    exp = meta["poc_plane_md5"][str(poc)]
                    assert D.plane_md5s(dec.read(slot)) == exp, "round %d POC %d differs" % (rnd, poc)
        for hs in copies:
            for h, _, _ in hs:
                ctx.release(h)
    finally:
        dec.close()


def test_many_launches_without_sync_keep_reference_ordering(golden_dir):
    """Dependency markers are per DPB slot (vvcr_api.cpp launch): 300 launches with no host sync, one
    reference slot kept alive across all of them and rewritten in the middle (write after read of ~100
    readers on several lanes) — every slot ends with the right picture."""
    from vvc_amd import native as N
    d = os.path.join(golden_dir, "ra416_q32")
    pics = S.load_sequence(d, max_pics=2)         # POC 0 (I) and POC 16 (B, references POC 0 only)
    meta = S.load_meta(d)
    I, B = pics
    assert {int(v) for l in range(2) for v in B["ref_poc"][l][:B["hdr"]["num_ref_l%d" % l]]} == {0}
    dec = D.Decoder(pics, dpb_slots=6)
    ctx = dec.ctx
    try:
        def prep(p, slot):
            ctx.begin_picture(S.pic_params(p, slot, {0: 0}))
            S.submit(ctx, p)
            S.set_loop_filter_params(ctx, p)
            return ctx.prepare(N.STAGE_ALL)
        hi = prep(I, 0)
        hb = [prep(B, s) for s in range(1, 6)]
        ctx.launch(hi)
        for k in range(300):
            ctx.launch(hb[k % 5])
            if k == 150:
                ctx.launch(hi)                        # rewrites the reference slot while its readers run
        ctx.sync()
        assert D.plane_md5s(dec.read(0)) == meta["poc_plane_md5"]["0"]
        for s in range(1, 6):
            assert D.plane_md5s(dec.read(s)) == meta["poc_plane_md5"]["16"], "slot %d" % s
        for h in [hi] + hb:
            ctx.release(h)
    finally:
        dec.close()


def test_bench_configuration_in_flight_matches_reference_md5(golden_dir, tmp_path):
    """bench.py's timed configuration: 4 segment copies in flight, 7 lanes (3 intra) on 8 hardware queues
    (set before the HIP runtime starts, hence a fresh process), no host sync between pictures."""
    import subprocess
    import sys
    script = tmp_path / "inflight.py"
    script.write_text(r'''
import os, sys
sys.path.insert(0, %r)
from vvc_amd import native as N, stream as S, decode as D
d = os.path.join(%r, "ra1080_q32")
pics, meta = S.load_sequence(d), S.load_meta(d)
per = 8
dec = D.Decoder(pics, dpb_slots=4 * per)
ctx = dec.ctx
copies = []
for c in range(4):
    alloc = S.SlotAllocator(pics, per, base=per * c)
    hs = []
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of)); S.submit(ctx, p); S.set_loop_filter_params(ctx, p)
        hs.append((ctx.prepare(N.STAGE_ALL), p["hdr"]["poc"], slot))
    copies.append(hs)
ctx.set_timing(False)
for rnd in range(3):
    for hs in copies:
        for h, _, _ in hs:
            ctx.launch(h)
ctx.sync()
bad = 0
for hs in copies:
    owner = {slot: poc for _, poc, slot in hs}
    for slot, poc in owner.items():
        bad += D.plane_md5s(dec.read(slot)) != meta["poc_plane_md5"][str(poc)]
print("MISMATCHES", bad)
''' % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), golden_dir))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", VVCR_LANES="7", VVCR_INTRA_LANES="3")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "MISMATCHES 0" in r.stdout, r.stdout[-2000:]


def test_stage_by_stage_launches_stay_on_one_lane(golden_dir, monkeypatch):
    """vvcr_launch_picture_stages: a picture launched one stage group at a time (residual, inter, intra,
    loop filters), two segment copies interleaved call by call so the lane choice of every call would
    differ — the later stages must run on the lane whose residual / prediction planes the earlier ones
    wrote, and every picture stays bit-exact."""
    from vvc_amd import native as N
    monkeypatch.setenv("VVCR_LANES", "5")
    monkeypatch.setenv("VVCR_INTRA_LANES", "3")   # the least recently used intra lane changes call by call
    d = os.path.join(golden_dir, "ra416_q32")
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    per = min(len(pics), 16)
    dec = D.Decoder(pics, dpb_slots=2 * per)
    ctx = dec.ctx
    groups = (N.STAGE_RESID, N.STAGE_INTER, N.STAGE_INTRA | N.STAGE_LMCS_INV, N.STAGE_DBK | N.STAGE_SAO | N.STAGE_ALF)
    try:
        copies = []
        for c in range(2):
            alloc = S.SlotAllocator(pics, per, base=per * c)
            hs = []
            for i, p in enumerate(pics):
                slot = alloc.assign(i, p["hdr"]["poc"])
                ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
                S.submit(ctx, p)
                S.set_loop_filter_params(ctx, p)
                hs.append((ctx.prepare(N.STAGE_ALL), p["hdr"]["poc"], slot))
            copies.append(hs)
        for i in range(len(pics)):
            for g in groups:
                for hs in copies:
                    ctx.launch_stages(hs[i][0], g)
        ctx.sync()
        for hs in copies:
            owner = {slot: poc for _, poc, slot in hs}
            for slot, poc in owner.items():
                assert D.plane_md5s(dec.read(slot)) == meta["poc_plane_md5"][str(poc)], "POC %d differs" % poc
            for h, _, _ in hs:
                ctx.release(h)
    finally:
        dec.close()


def test_stage_by_stage_with_every_lane_held_fails_cleanly(golden_dir, monkeypatch):
    """Three segment copies interleaved stage by stage over two B lanes (VVCR_LANES=5, VVCR_INTRA_LANES=3):
    the third copy's B picture finds both B lanes holding a picture whose later stages are pending. The
    launch must fail with VVCR_E_STATE (never overwrite a held lane's planes); after the held pictures'
    stages complete, the refused picture launches whole and every picture of the copies stays bit-exact."""
    from vvc_amd import native as N
    monkeypatch.setenv("VVCR_LANES", "5")
    monkeypatch.setenv("VVCR_INTRA_LANES", "3")
    d = os.path.join(golden_dir, "ra416_q32")
    pics = S.load_sequence(d)
    meta = S.load_meta(d)
    per = min(len(pics), 16)
    dec = D.Decoder(pics, dpb_slots=3 * per)
    ctx = dec.ctx
    groups = (N.STAGE_RESID, N.STAGE_INTER, N.STAGE_INTRA | N.STAGE_LMCS_INV, N.STAGE_DBK | N.STAGE_SAO | N.STAGE_ALF)
    try:
        copies = []
        for c in range(3):
            alloc = S.SlotAllocator(pics, per, base=per * c)
            hs = []
            for i, p in enumerate(pics):
                slot = alloc.assign(i, p["hdr"]["poc"])
                ctx.begin_picture(S.pic_params(p, slot, alloc.slot_of))
                S.submit(ctx, p)
                S.set_loop_filter_params(ctx, p)
                hs.append((ctx.prepare(N.STAGE_ALL), p["hdr"]["poc"], slot))
            copies.append(hs)
        refused = 0
        for i in range(len(pics)):
            pending = []   # copies whose picture i was refused: launched whole once the others' stages are done
            for g in groups:
                for c, hs in enumerate(copies):
                    if c in pending:
                        continue
                    try:
                        ctx.launch_stages(hs[i][0], g)
                    except N.VvcrError as e:
                        assert "pending" in str(e), str(e)
                        assert g == N.STAGE_RESID, "only a picture's first stage call can be refused"
                        pending.append(c)
            for c in pending:
                refused += 1
                ctx.launch(copies[c][i][0])
        assert refused > 0, "the interleave never found every B lane held"
        ctx.sync()
        for hs in copies:
            owner = {slot: poc for _, poc, slot in hs}
            for slot, poc in owner.items():
                assert D.plane_md5s(dec.read(slot)) == meta["poc_plane_md5"][str(poc)], "POC %d differs" % poc
            for h, _, _ in hs:
                ctx.release(h)
    finally:
        dec.close()
