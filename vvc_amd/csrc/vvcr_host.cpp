// vvcr_host.cpp — host producer logic: turns the picture's CU/PU/TU descriptors into GPU work lists.
// The decisions mirror the reference's dispatch in InterPrediction::motionCompensation
// (InterPrediction.cpp:1517-1660) so that every PU reaches the kernel that reproduces its prediction.
#include "vvcr_host.h"
#include <string>

namespace {

constexpr int MODE_INTER = 0;
constexpr int IMV_HPEL = 3;      // TypeDef.h:924
constexpr int MRG_TYPE_DEFAULT_N = 0, MRG_TYPE_SUBPU_ATMVP = 1;
constexpr int B_SLICE = 0;       // SliceType (TypeDef.h): B_SLICE=0, P_SLICE=1, I_SLICE=2

void fail(const std::string &m) { throw VvcrError(VVCR_E_ARG, m); }

// InterPrediction::xCheckIdenticalMotion (InterPrediction.cpp:248): bi-prediction from the same
// picture with the same MV is predicted as uni-prediction from list 0.
bool identical_motion(const vvcr_pic_params &pp, int interDir, int r0, int r1, int mv0x, int mv0y, int mv1x, int mv1y) {
  if (pp.slice_type != B_SLICE || pp.wp_b) return false;
  if (interDir != 3 || r0 < 0 || r1 < 0) return false;
  return pp.ref_poc[0][r0] == pp.ref_poc[1][r1] && mv0x == mv1x && mv0y == mv1y;
}

void push_tiles(std::vector<McJob> &out, int x0, int y0, int w, int h, McJob proto) {
  for (int y = 0; y < h; y += 16)
    for (int x = 0; x < w; x += 16) {
      McJob j = proto;
      j.x = (int16_t)(x0 + x);
      j.y = (int16_t)(y0 + y);
      j.w = (uint8_t)std::min(16, w - x);
      j.h = (uint8_t)std::min(16, h - y);
      out.push_back(j);
    }
}

McJob make_job(const vvcr_pic_params &pp, int interDir, int r0, int r1, int mv0x, int mv0y, int mv1x, int mv1y,
               int bcw, bool altHpel) {
  McJob j{};
  j.flags = MC_LUMA | MC_CHROMA;
  if (identical_motion(pp, interDir, r0, r1, mv0x, mv0y, mv1x, mv1y)) interDir = 1;
  if (interDir & 1) { j.flags |= MC_L0; j.slot[0] = (int8_t)pp.ref_slot[0][r0]; j.mv[0][0] = (int16_t)mv0x; j.mv[0][1] = (int16_t)mv0y; }
  if (interDir & 2) { j.flags |= MC_L1; j.slot[1] = (int8_t)pp.ref_slot[1][r1]; j.mv[1][0] = (int16_t)mv1x; j.mv[1][1] = (int16_t)mv1y; }
  if (altHpel) j.flags |= MC_ALT_HPEL;
  j.bcw = (int8_t)bcw;
  return j;
}

}  // namespace

void validate_descriptors(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d) {
  const int ncu = (int)d.cu.size(), npu = (int)d.pu.size(), ntu = (int)d.tu.size();
  for (int i = 0; i < ncu; i++) {
    const vvcr_cu &c = d.cu[i];
    if (c.yvalid && (c.x < 0 || c.y < 0 || c.w <= 0 || c.h <= 0 || c.w > 128 || c.h > 128)) fail("CU " + std::to_string(i) + " has a bad luma area");
    if (c.cvalid && (c.cx < 0 || c.cy < 0 || c.cw <= 0 || c.ch <= 0 || c.cw > 64 || c.ch > 64)) fail("CU " + std::to_string(i) + " has a bad chroma area");
    if (!c.yvalid && !c.cvalid) fail("CU " + std::to_string(i) + " has no component");
    if (c.npu > 0 && (c.firstpu < 0 || c.firstpu + c.npu > npu)) fail("CU " + std::to_string(i) + " PU range");
    if (c.ntu > 0 && (c.firsttu < 0 || c.firsttu + c.ntu > ntu)) fail("CU " + std::to_string(i) + " TU range");
  }
  for (int i = 0; i < npu; i++) {
    const vvcr_pu &p = d.pu[i];
    if (p.cu < 0 || p.cu >= ncu) fail("PU " + std::to_string(i) + " CU index");
    const vvcr_cu &c = d.cu[p.cu];
    if (c.predmode == MODE_INTER) {
      if ((p.interdir & 1) && (p.ref0 < 0 || p.ref0 >= pp.num_ref[0])) fail("PU " + std::to_string(i) + " ref0");
      if ((p.interdir & 2) && (p.ref1 < 0 || p.ref1 >= pp.num_ref[1])) fail("PU " + std::to_string(i) + " ref1");
    }
  }
  for (int i = 0; i < ntu; i++) {
    const vvcr_tu &t = d.tu[i];
    if (t.cu < 0 || t.cu >= ncu) fail("TU " + std::to_string(i) + " CU index");
    for (int c = 0; c < 3; c++) {
      const int32_t *b = t.b[c];
      if (b[2] <= 0) continue;
      const int pw = c ? sp.width / 2 : sp.width, ph = c ? sp.height / 2 : sp.height;
      const int maxs = b[6] >= 0 ? 64 : 128;   // coded TBs are <= 64 (maxTbSize); residual-free TUs span the CU
      if (b[0] < 0 || b[1] < 0 || b[0] + b[2] > pw + 128 || b[1] + b[3] > ph + 128 || b[2] > maxs || b[3] > maxs) fail("TU " + std::to_string(i) + " area");
      if (b[6] >= 0 && (int64_t)b[6] + (int64_t)b[2] * b[3] > (int64_t)d.coef.size()) fail("TU " + std::to_string(i) + " coefficient range");
    }
  }
  if (!d.motion.empty() && d.motion.size() != (size_t)(sp.width / 4) * (sp.height / 4)) fail("motion field size");
}

void build_work_lists(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, WorkLists &wl) {
  wl.clear();
  const int W4 = sp.width / 4;
  for (const vvcr_cu &c : d.cu) {
    if (c.predmode != MODE_INTER || !c.yvalid) continue;
    if (c.geo || c.affine) { wl.n_unsupported_inter++; continue; }
    for (int k = 0; k < c.npu; k++) {
      const vvcr_pu &p = d.pu[c.firstpu + k];
      const bool alt = c.imv == IMV_HPEL;
      const int bcw = p.ciip ? 2 : c.bcw;   // BCW is not applied to CIIP (InterPrediction.cpp:1397)
      if (p.mrgtype == MRG_TYPE_SUBPU_ATMVP) {
        // xSubPuMC (InterPrediction.cpp:289): 8x8 sub-blocks with their own motion, no BDOF / DMVR
        for (int y = 0; y < p.h; y += 8)
          for (int x = 0; x < p.w; x += 8) {
            const vvcr_motion &m = d.motion[(size_t)((p.y + y) >> 2) * W4 + ((p.x + x) >> 2)];
            McJob j = make_job(pp, m.inter_dir, m.ref0, m.ref1, m.mv0x, m.mv0y, m.mv1x, m.mv1y, m.bcw, alt);
            push_tiles(wl.mc_basic, p.x + x, p.y + y, std::min(8, p.w - x), std::min(8, p.h - y), j);
          }
        continue;
      }
      if (p.dmvr || p.bdof) { wl.n_unsupported_inter++; continue; }
      McJob j = make_job(pp, p.interdir, p.ref0, p.ref1, p.mv0x, p.mv0y, p.mv1x, p.mv1y, bcw, alt);
      push_tiles(wl.mc_basic, p.x, p.y, p.w, p.h, j);
    }
  }
}
