"""Host logic of the replay driver (no GPU): DPB slot allocation per segment copy (vvc_amd/stream.py
SlotAllocator) — disjoint slot ranges, no slot reused while a later picture still references it, and the
minimum slot counts bench.py relies on (4 segment copies in 32 slots)."""
import os

import pytest

from vvc_amd import stream as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _refs(p):
    h = p["hdr"]
    return {int(p["ref_poc"][l][r]) for l in range(2) for r in range(h["num_ref_l%d" % l])}


@pytest.mark.parametrize("name", ["ra416_q32", "ra1080_q32", "ra2160_q32"])
def test_slot_allocator_keeps_references_resident(name):
    pics = S.load_sequence(os.path.join(GOLD, name))
    per = 32 // 4
    for c in range(4):
        a = S.SlotAllocator(pics, per, base=per * c)
        for i, p in enumerate(pics):
            poc = p["hdr"]["poc"]
            refs = _refs(p)
            slot = a.assign(i, poc)
            assert per * c <= slot < per * (c + 1)
            # every reference of this picture is still resident, in its own slot, and not this picture's slot
            for r in refs:
                assert r in a.slot_of and a.slot_of[r] != slot, (name, poc, r)


def test_slot_allocator_reports_exhaustion():
    pics = S.load_sequence(os.path.join(GOLD, "ra1080_q32"))
    with pytest.raises(RuntimeError):
        a = S.SlotAllocator(pics, 2)
        for i, p in enumerate(pics):
            a.assign(i, p["hdr"]["poc"])


# ---- host-only picture builder (vvcr_picture_*): validation and planning without a device

def _first_pic(name, idx=0):
    pics = S.load_sequence(os.path.join(GOLD, name), max_pics=idx + 1)
    alloc = S.SlotAllocator(pics, 16)
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
    return p, slot, dict(alloc.slot_of)


def _picture(p, slot, slot_of):
    from vvc_amd import native as N
    h = p["hdr"]
    return N.Picture(h["width"], h["height"], S.pic_params(p, slot, slot_of), bit_depth=h["bitdepth_y"],
                     ctu_log2=h["ctu_log2"], dpb_slots=16)


def test_builder_rejects_tu_crossing_the_bottom_edge():
    import numpy as np
    from vvc_amd import native as N
    p, slot, slot_of = _first_pic("ai416_q37")
    H = p["hdr"]["height"]
    tu = np.array(p["tu"], np.int32)
    k = int(np.nonzero(tu[:, 6 + 2] > 0)[0][-1])     # a TU with a luma block (b[0][2] = width > 0)
    tu[k, 6 + 1] = H - tu[k, 6 + 3] + 4               # b[0][1] = y: 4 rows past the bottom edge
    pic = _picture(p, slot, slot_of)
    geo = np.zeros((0, 13), np.int32)
    with pytest.raises(N.VvcrError) as e:
        pic.submit(p["cu"], p["pu"], tu, p["coef"], p["motion"].reshape(-1, 10), geo)
    assert "(-1)" in str(e.value) and "area" in str(e.value)      # VVCR_E_ARG
    pic.close()


def test_builder_rejects_cu_outside_the_picture():
    import numpy as np
    from vvc_amd import native as N
    p, slot, slot_of = _first_pic("ra416_q32", 1)
    cu = np.array(p["cu"], np.int32)
    cu[0, 0] = p["hdr"]["width"] - cu[0, 2] + 8         # x: past the right edge
    pic = _picture(p, slot, slot_of)
    with pytest.raises(N.VvcrError):
        pic.submit(cu, p["pu"], p["tu"], p["coef"], p["motion"].reshape(-1, 10), np.zeros((0, 13), np.int32))
    pic.close()


@pytest.mark.parametrize("field,value", [("num_vb_ver", 4), ("vb_ver", 100), ("vb_hor", 0), ("ladf_num", 1),
                                         ("ladf_lower_bound", 0)])
def test_builder_rejects_bad_filter_parameters(field, value):
    """virtual boundaries (count <= 3, multiples of 8 inside the picture) and LADF intervals (2..5, bounds
    increasing from 0) are checked when a picture is created; the streams' own parameters pass"""
    from vvc_amd import native as N
    for name in ("ravb416_q32", "raladf416_q32"):
        p, slot, slot_of = _first_pic(name)
        _picture(p, slot, slot_of).close()
    p, slot, slot_of = _first_pic("ravb416_q32" if "vb" in field else "raladf416_q32")
    h = p["hdr"]
    pp = S.pic_params(p, slot, slot_of)
    if field in ("vb_ver", "vb_hor"):
        getattr(pp, field)[0] = value
    elif field == "ladf_lower_bound":
        pp.ladf_lower_bound[2] = pp.ladf_lower_bound[1]   # not increasing
    else:
        setattr(pp, field, value)
    with pytest.raises(N.VvcrError):
        N.Picture(h["width"], h["height"], pp, bit_depth=h["bitdepth_y"], ctu_log2=h["ctu_log2"], dpb_slots=16).close()


def test_pic_params_refuses_missing_reference():
    p, slot, slot_of = _first_pic("ra416_q32", 1)
    with pytest.raises(KeyError):
        S.pic_params(p, slot, {})


@pytest.mark.parametrize("name", ["ai416_q37", "ra416_q32", "ralm416_q32", "rawp416_q32", "ratile416_q32"])
def test_builder_plans_every_picture(name):
    pics = S.load_sequence(os.path.join(GOLD, name))
    alloc = S.SlotAllocator(pics, 16)
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        pic = S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16)
        c = pic.work_counts()
        if p["hdr"]["slice_type"] == 2:
            assert c["intra_steps"] > 0 and c["mc"] == 0
        pic.close()


def test_threaded_planning_is_deterministic():
    """Several pictures planned at once on several threads (the library drops the GIL) give the same
    work lists as one at a time."""
    import concurrent.futures as cf
    pics = S.load_sequence(os.path.join(GOLD, "ra416_q32"))
    alloc = S.SlotAllocator(pics, 16)
    jobs = []
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        jobs.append((p, slot, dict(alloc.slot_of)))

    def counts(j):
        pic = S.plan_picture(*j, dpb_slots=16)
        c = pic.work_counts()
        pic.close()
        return c
    serial = [counts(j) for j in jobs]
    with cf.ThreadPoolExecutor(6) as ex:
        par = list(ex.map(counts, jobs))
    assert par == serial


_DBK_LISTS = r'''
import ctypes as C, hashlib, os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from vvc_amd import native as N, stream as S
L = N.lib()
L.vvcr_debug_dbk_segments.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
h = hashlib.md5()
for name in sys.argv[2:]:
    pics = S.load_sequence(os.path.join(sys.argv[1], "tests", "golden", name))
    alloc = S.SlotAllocator(pics, 16)
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        pic = S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16)
        n = L.vvcr_debug_dbk_segments(pic.h, None, 0)
        a = np.zeros(2 * n, np.uint32)
        L.vvcr_debug_dbk_segments(pic.h, a.ctypes.data, n)
        h.update(a.tobytes())
        pic.close()
print(h.hexdigest())
'''


def test_deblocking_plan_independent_of_worker_count(tmp_path):
    """The deblocking planner splits the CTUs over VVCR_DBK_THREADS workers: the segment lists (and their
    order) must be those of a single pass, for any worker count."""
    import subprocess
    import sys
    script = tmp_path / "dbk.py"
    script.write_text(_DBK_LISTS)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = []
    for t in ("1", "3", "8"):
        env = dict(os.environ, VVCR_DBK_THREADS=t, VVCR_DBK_GPU="0")
        r = subprocess.run([sys.executable, str(script), root, "ra1080_q32", "ralm416_q32"], env=env, capture_output=True,
                           text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        out.append(r.stdout.strip())
    assert out[0] == out[1] == out[2]


_PLAN_HASHES = r'''
import os, sys
sys.path.insert(0, sys.argv[1])
from vvc_amd import stream as S
for name in sys.argv[2:]:
    pics = S.load_sequence(os.path.join(sys.argv[1], "tests", "golden", name))
    alloc = S.SlotAllocator(pics, 16)
    for i, p in enumerate(pics):
        slot = alloc.assign(i, p["hdr"]["poc"])
        S.plan_picture(p, slot, alloc.slot_of, dpb_slots=16).close()
'''


def test_intra_plan_fast_paths_keep_the_plan(tmp_path):
    """The intra planner's dense-picture path (unit records preset, no CU-map indirection) must leave the
    plan unchanged: the whole plan's hash per picture (VVCR_PLAN_HASH) with the dense path off
    (VVCR_PLAN_DENSE=0) equals the default's, with one planner thread and with four (a tiled picture's
    regions are planned on threads, which orders its steps region by region: compared at equal counts)."""
    import subprocess
    import sys
    script = tmp_path / "plan.py"
    script.write_text(_PLAN_HASHES)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = []
    for dense, threads in (("0", "1"), ("1", "1"), ("0", "4"), ("1", "4")):
        env = dict(os.environ, VVCR_PLAN_HASH="1", VVCR_PLAN_DENSE=dense, VVCR_PLAN_THREADS=threads)
        r = subprocess.run([sys.executable, str(script), root, "ai416_q37", "ra416_q32", "ratilenf416_q32"], env=env,
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [l for l in r.stderr.splitlines() if l.startswith("intra plan hash")]
        assert lines
        out.append(lines)
    assert out[0] == out[1] and out[2] == out[3]
