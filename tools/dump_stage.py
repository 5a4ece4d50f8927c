"""Diagnostics: run one libvvcr stage over a fixture sequence on the GPU and dump the output planes
(npz under gpurun_out/) for offline comparison with the golden planes.

  python tools/dump_stage.py ra416_q32 inter
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import native as N  # noqa: E402
from vvc_amd import stream as S  # noqa: E402


def main():
    name, stage = sys.argv[1], sys.argv[2]
    maxp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    pics = S.load_sequence(os.path.join(ROOT, "tests", "golden", name), maxp)
    by_poc = {p["hdr"]["poc"]: p for p in pics}
    h0 = pics[0]["hdr"]
    ctx = N.Context(h0["width"], h0["height"], dpb_slots=20)
    out = {}
    for p in pics:
        poc = p["hdr"]["poc"]
        slot_of = {}
        for l in range(2):
            for r in range(p["hdr"]["num_ref_l%d" % l]):
                q = int(p["ref_poc"][l][r])
                if q not in slot_of:
                    slot_of[q] = len(slot_of) + 1
                    for c, pl in enumerate("yuv"):
                        ctx.write_plane(N.BUF_RECO, slot_of[q], c, by_poc[q]["alf_" + pl])
        ctx.begin_picture(S.pic_params(p, 0, slot_of))
        S.submit(ctx, p)
        if stage == "inter":
            if p["hdr"]["slice_type"] == 2:
                continue
            ctx.end_picture(N.STAGE_INTER)
            for c, pl in enumerate("yuv"):
                out["%d_%s" % (poc, pl)] = ctx.read_plane(N.BUF_PRED, 0, c)
            out["%d_dmvr" % poc] = ctx.dmvr_deltas()
        elif stage == "resid":
            ctx.end_picture(N.STAGE_RESID)
            for c, pl in enumerate("yuv"):
                out["%d_%s" % (poc, pl)] = ctx.read_plane(N.BUF_RESI, 0, c)
        elif stage == "recon":
            ctx.end_picture(N.STAGE_RESID | N.STAGE_INTER | N.STAGE_INTRA)
            for c, pl in enumerate("yuv"):
                out["%d_%s" % (poc, pl)] = ctx.read_plane(N.BUF_RECO, 0, c)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "dump_%s_%s.npz" % (name, stage)), **out)
    ctx.close()


if __name__ == "__main__":
    main()
