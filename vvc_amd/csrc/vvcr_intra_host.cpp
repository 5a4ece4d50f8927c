// vvcr_intra_host.cpp — reconstruction planning: decoding order, availability order maps and
// dependency levels for the intra / CIIP steps (see vvcr_intra.h).
//
// Decoding order follows DecCu::decompressCtu (DecCu.cpp:102-155): CTUs in raster order; inside a CTU
// the CUs in coding order (separate luma / chroma passes for a dual tree); an intra CU reconstructs all
// its luma transform blocks, then Cb and Cr per transform unit (xReconIntraQT / xIntraRecQT :489-612);
// ISP sub-partitions in order, with the prediction regions of CU::isPredRegDiffFromTB (UnitTools.cpp:3692);
// an inter CU is one step (xReconInter :664-772, setDecomp of the whole CU), CIIP predicting its planar
// part from the reconstructed neighbours first (IntraPrediction::geneIntrainterPred :735).
#include "vvcr_intra.h"
#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <memory>
#include <queue>
#include <thread>
#include <exception>
#include <string>
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace {

// IntraPrediction::initPredIntraParams (IntraPrediction.cpp:1030-1100) for one step: the wide-angle mode
// (getWideAngle :184), intraPredAngle / invAngle (g_intraPredAngle-style tables :72-76), PDPC and its
// angular scale, the reference smoothing and the interpolation-filter choice (m_ipaParam), the same
// derivation k_intra made per step before. Block sizes: the region (ISP: predSize by the CU).
constexpr int kPlanar = 0, kDC = 1, kHor = 18, kDia = 34, kVer = 50, kVdia = 66;
constexpr int16_t kAngTable[32] = {0, 1, 2, 3, 4, 6, 8, 10, 12, 14, 16, 18, 20, 23, 26, 29, 32, 35, 39, 45, 51, 57, 64, 73, 86, 102, 128, 171, 256, 341, 512, 1024};
constexpr int16_t kInvAngTable[32] = {0, 16384, 8192, 5461, 4096, 2731, 2048, 1638, 1365, 1170, 1024, 910, 819, 712, 630, 565,
                                      512, 468, 420, 364, 321, 287, 256, 224, 191, 161, 128, 96, 64, 48, 32, 16};
constexpr uint8_t kIntraFilter[8] = {24, 24, 24, 14, 2, 0, 0, 0};
int ilog2i(int v) { int r = -1; while (v > 0) { v >>= 1; r++; } return r; }
int wide_angle_h(int w, int h, int mode) {
  if (mode > kDC && mode <= kVdia) {
    const int modeShift[6] = {0, 6, 10, 12, 14, 15};
    const int d = std::abs(ilog2i(w) - ilog2i(h));
    if (w > h && mode < 2 + modeShift[d]) mode += kVdia - 1;
    else if (h > w && mode > kVdia - modeShift[d]) mode -= kVdia - 1;
  }
  return mode;
}
void set_pred_params(IntraJob &J) {
  const bool ciip = J.flags & IJ_CIIP, isp = J.flags & (IJ_ISP_HOR | IJ_ISP_VER), mip = J.flags & IJ_MIP;
  const bool bdpcm = J.flags & IJ_BDPCM, lmMode = J.comp > 0 && J.mode >= 67;
  const int w = J.w, h = J.h, mrl = J.comp ? 0 : J.mrl;
  const int dirMode = ciip ? kPlanar : (int)J.mode;
  const int bw = isp ? J.cw : w, bh = isp ? J.ch : h;
  const int predMode = (lmMode || mip || bdpcm) ? dirMode : wide_angle_h(bw, bh, dirMode);
  const bool isModeVer = predMode >= kDia;
  bool applyPDPC = w >= 4 && h >= 4 && mrl == 0;
  const int angMode = isModeVer ? predMode - kVer : -(predMode - kHor);
  int absAng = 0, invAngle = 0, angle = 0, angScale = 0;
  if (!lmMode && !mip && !bdpcm && dirMode > kDC && dirMode < 67) {
    const int a = std::abs(angMode);
    absAng = kAngTable[a];
    invAngle = kInvAngTable[a];
    angle = angMode < 0 ? -absAng : absAng;
    if (angMode < 0) {
      applyPDPC = false;
    } else if (angMode > 0) {
      const int side = isModeVer ? h : w;
      angScale = std::min(2, ilog2i(side) - (ilog2i(3 * invAngle - 2) - 8));
      applyPDPC = applyPDPC && angScale >= 0;
    }
  }
  bool refFilter = false, interp = false;
  if (J.comp == 0 && !isp && !mip && mrl == 0 && dirMode != kDC && !bdpcm && !lmMode) {
    if (dirMode == kPlanar) {
      refFilter = w * h > 32;
    } else {
      const int diff = std::min(std::abs(predMode - kHor), std::abs(predMode - kVer));
      const int log2Size = (ilog2i(w) + ilog2i(h)) >> 1;
      if (diff > kIntraFilter[log2Size]) {
        refFilter = (absAng & 31) == 0;
        interp = !refFilter;
      }
    }
  }
  J.ang = (int16_t)angle;
  J.inv_ang = (int16_t)invAngle;
  J.pred_mode = (int8_t)predMode;
  J.pbits = (uint8_t)((applyPDPC ? PB_PDPC : 0) | (refFilter ? PB_REFFILT : 0) | (interp ? PB_INTERP : 0) |
                      (std::max(0, angScale) << 4));
}


constexpr int MODE_INTER = 0, MODE_INTRA = 1;

struct Planner {
  const vvcr_seq_params &sp;
  const vvcr_pic_params &pp;
  const PictureDescriptors &d;
  IntraPlan &out;
  int W4, H4, ctu;
  // Per 4x4 luma unit / 2x2 chroma unit: the CU covering it per channel (umap: the producer's maps when
  // it hands them over, else own_map). Only the units of CUs whose reconstruction is a step ("written":
  // intra, CIIP, chroma steps) carry their own order / level / producers in ur (one record per unit:
  // the planner's unit visits touch one cache line, not five arrays),
  // initialised when the CU is planned; the units of a plain inter CU share its cu_seq, level 0 and no
  // producer, so a B picture's inter CUs cost no per-unit work.
  // per unit of channel ch: decoding order (seq), level, and the steps (indices into jobs) that reconstruct
  // it: prod[0] luma (ch 0) or Cb, prod[1] Cr (ch 1)
  struct UnitRec { int32_t order, level, prod[2]; };
  // The per-unit / per-CU / per-CTU arrays are shared with the region planners of a tiled picture (run:
  // each plans the CTUs of one tile / slice, writes only its own CUs' and units' entries and reads no
  // other region's): the planner that owns them holds the storage (*_store), every planner the pointers.
  bigbuf::raw<UnitRec> ur_store[2];
  UnitRec *ur[2] = {nullptr, nullptr};
  static int pslot(int comp) { return comp == 2 ? 1 : 0; }
  const int32_t *umap[2] = {nullptr, nullptr};
  bigbuf::vec<int32_t> own_map[2];
  bigbuf::vec<int32_t> cu_seq_store;
  int32_t *cu_seq = nullptr;        // per CU: the seq of a plain inter CU, kInf until planned
  bigbuf::vec<uint8_t> written_store[2];
  uint8_t *written[2] = {nullptr, nullptr};   // per CU and channel: its units carry their own order / level / producers
  // A picture without inter CUs (an intra picture: most of the planner's time) has every unit record
  // preset to the "not decoded" sentinel (order kUnset > any seq): a unit's record is then read directly,
  // without the CU map and written flag in front of it (r06: I picture plan -N %)
  bool dense = false;
  static constexpr int32_t kUnset = 0x7f7f7f7f;
  static constexpr int32_t kInf = 1 << 30;
  int32_t order_of(int ch, size_t i) const {
    if (dense) return ur[ch][i].order;   // (kUnset or the unit's seq)
    const int32_t m = umap[ch][i];
    if (m < 0) return kInf;
    return written[ch][m] ? ur[ch][i].order : cu_seq[m];
  }
  // first write of CU ci's units of channel ch: their own order / level / producers from here on
  void touch(int ch, int ci) {
    if (written[ch][ci]) return;
    written[ch][ci] = 1;
    const vvcr_cu &c = d.cu[ci];
    const int s = ch ? 1 : 2;
    const int x = ch ? c.cx : c.x, y = ch ? c.cy : c.y, w = ch ? c.cw : c.w, h = ch ? c.ch : c.h;
    for (int uy = y >> s; uy < (y + h + (1 << s) - 1) >> s; uy++)
      for (int ux = x >> s; ux < (x + w + (1 << s) - 1) >> s; ux++) {
        const size_t i = (size_t)uy * W4 + ux;
        ur[ch][i] = UnitRec{kInf, 0, {-1, -1}};
      }
  }
  bigbuf::vec<std::pair<int32_t, IntraJob>> jobs;   // (level, job)
  bigbuf::vec<int32_t> dep_off{0}, dep_flat;        // per job (CSR): the steps it reads from (indices into jobs)
  bigbuf::vec<int32_t> cur;                         // dependencies of the step being planned
  bigbuf::vec<int32_t> cur_mark;                    // per job: the step count at which it last entered `cur`
  bigbuf::vec<int32_t> cclm_deps;                   // scratch of intra_chroma
  void add_dep(int32_t pr) {   // O(1) de-duplication (a CCLM block reads hundreds of luma units)
    if ((size_t)pr >= cur_mark.size()) cur_mark.resize(std::max<size_t>(2 * cur_mark.size(), (size_t)pr + 1024), -1);
    const int32_t tok = (int32_t)jobs.size();
    if (cur_mark[pr] != tok) { cur_mark[pr] = tok; cur.push_back(pr); }
  }
  int seq = 0;
  bool cscale = false;                              // LMCS chroma residual scaling active in this picture
  bool fuse = false;                                // plain inter CUs reconstructed by k_mc (fused_inter_cu)
  // Slice / tile of every CTU (getCURestricted: a neighbour is usable only inside the same slice and
  // tile, CodingStructure.cpp:1519-1537, CU::isSameSliceAndTile UnitTools.cpp:170); cur_reg is the
  // region of the CU being planned / the step being resolved.
  bigbuf::vec<int32_t> ctu_reg_store;
  const int32_t *ctu_reg = nullptr;
  int wc = 1, cur_reg = 0;
  int region_at(int lx, int ly) const { return ctu_reg[(size_t)(ly >> sp.ctu_log2) * wc + (lx >> sp.ctu_log2)]; }

  Planner(const vvcr_seq_params &s, const vvcr_pic_params &p, const PictureDescriptors &dd, IntraPlan &o)
      : sp(s), pp(p), d(dd), out(o) {
    W4 = sp.width / 4;
    H4 = sp.height / 4;
    ctu = 1 << sp.ctu_log2;
  }

  // component-sample rectangle -> unit rectangle of map ch (4x4 luma units / 2x2 chroma units); the
  // highest level among the decoded units read, whose producing steps of component comp are collected
  // in `cur` (the step's dependencies)
  int max_level(int ch, int comp, int x0, int y0, int x1, int y1) {   // inclusive sample bounds
    const int s = ch ? 1 : 2;
    const int pw = ch ? sp.width / 2 : sp.width, ph = ch ? sp.height / 2 : sp.height;
    x0 = std::max(x0, 0); y0 = std::max(y0, 0);
    x1 = std::min(x1, pw - 1); y1 = std::min(y1, ph - 1);
    int m = 0;
    if (x0 > x1 || y0 > y1) return 0;
    // a unit is 4x4 luma samples in both maps: its CTU is (u >> lg); the region is looked up per CTU
    const int lg = sp.ctu_log2 - 2;
    int lastc = -1;
    bool regok = false;
    for (int uy = y0 >> s; uy <= (y1 >> s); uy++)
      for (int ux = x0 >> s; ux <= (x1 >> s); ux++) {
        const int c = (uy >> lg) * wc + (ux >> lg);   // the region first: another region's units are not read
        if (c != lastc) { lastc = c; regok = ctu_reg[c] == cur_reg; }
        if (!regok) continue;
        const size_t i = (size_t)uy * W4 + ux;
        if (!dense) {
          const int32_t cu = umap[ch][i];
          if (cu < 0 || !written[ch][cu]) continue;
        }
        const UnitRec &r = ur[ch][i];
        if (r.order >= seq) continue;
        m = std::max(m, r.level);
        const int32_t pr = r.prod[pslot(comp)];
        if (pr >= 0) add_dep(pr);
      }
    return m;
  }
  void mark(int ci, int ch, int x, int y, int w, int h, int lev, bool set_order, int comp = -1, int job = -1) {
    touch(ch, ci);
    const int s = ch ? 1 : 2;
    for (int uy = y >> s; uy < (y + h + (1 << s) - 1) >> s; uy++)
      for (int ux = x >> s; ux < (x + w + (1 << s) - 1) >> s; ux++) {
        const size_t i = (size_t)uy * W4 + ux;
        UnitRec &r = ur[ch][i];
        r.level = lev;
        if (set_order) r.order = seq;
        if (comp >= 0) r.prod[pslot(comp)] = job;
      }
  }
  // level of a prediction from the reference lines of region (x, y, w, h) with lengths topLen/leftLen
  int ref_level(int ch, int comp, int x, int y, int topLen, int leftLen, int mrl) {
    int m = max_level(ch, comp, x - 1 - mrl, y - 1 - mrl, x + topLen - 1, y - 1);
    m = std::max(m, max_level(ch, comp, x - 1 - mrl, y - 1 - mrl, x - 1, y + leftLen - 1));
    return m;
  }

  // appends a step with the dependencies collected in `cur`; returns its index
  int push(int lev, const IntraJob &j) {
    std::sort(cur.begin(), cur.end());
    cur.erase(std::unique(cur.begin(), cur.end()), cur.end());
    jobs.emplace_back(lev, j);
    dep_flat.insert(dep_flat.end(), cur.begin(), cur.end());
    dep_off.push_back((int32_t)dep_flat.size());
    cur.clear();
    return (int)jobs.size() - 1;
  }

  IntraJob base(const vvcr_cu &c, int comp) const {
    IntraJob j{};
    j.comp = (uint8_t)comp;
    j.seq = seq;
    if (comp == 0) { j.cx = (int16_t)c.x; j.cy = (int16_t)c.y; j.cw = (uint8_t)c.w; j.ch = (uint8_t)c.h; }
    else { j.cx = (int16_t)c.cx; j.cy = (int16_t)c.cy; j.cw = (uint8_t)c.cw; j.ch = (uint8_t)c.ch; }
    return j;
  }

  // LMCS chroma residual scaling of a chroma block whose luma-equivalent top-left is (lx, ly): the CU
  // covering the top-left of its 64x64 VPDU gives the neighbour samples (Reshape::calculateChromaAdjVpduNei,
  // Reshape.cpp:107-198); the step reads them, so their producers become dependencies. Returns the level.
  int set_cscale(IntraJob &j, int lx, int ly) {
    const int n64 = std::min(64, ctu);
    const int vx0 = (lx / n64) * n64, vy0 = (ly / n64) * n64;
    const int ci = umap[0][(size_t)(vy0 >> 2) * W4 + (vx0 >> 2)];
    if (ci < 0) throw VvcrError(VVCR_E_STATE, "LMCS: no luma CU at a VPDU corner");
    const vvcr_cu &t = d.cu[ci];
    j.vx = (int16_t)t.x; j.vy = (int16_t)t.y;
    const bool left = t.x > 0 && region_at(t.x - 1, t.y) == cur_reg, above = t.y > 0 && region_at(t.x, t.y - 1) == cur_reg;
    j.vnb = CS_SCALE | (left ? CS_LEFT : 0) | (above ? CS_ABOVE : 0);
    int lev = 0;
    if (left) lev = std::max(lev, max_level(0, 0, t.x - 1, t.y, t.x - 1, t.y + n64 - 1));
    if (above) lev = std::max(lev, max_level(0, 0, t.x, t.y - 1, t.x + n64 - 1, t.y - 1));
    return lev;
  }

  void inter_cu(int ci) {
    const vvcr_cu &c = d.cu[ci];
    const vvcr_pu &p = d.pu[c.firstpu];
    seq++;
    if (p.ciip) {
      // CIIP: planar from the neighbours, blended with the inter prediction (geneWeightedPred :681)
      auto intraAt = [&](int x, int y) {
        if (x < 0 || y < 0 || x >= sp.width || y >= sp.height || region_at(x, y) != cur_reg) return false;
        const int n = umap[0][(size_t)(y >> 2) * W4 + (x >> 2)];
        return n >= 0 && n <= ci && d.cu[n].predmode == MODE_INTRA;
      };
      const bool n0 = intraAt(c.x - 1, c.y + c.h - 1), n1 = intraAt(c.x + c.w - 1, c.y - 1);
      const int wIntra = (n0 && n1) ? 3 : ((!n0 && !n1) ? 1 : 2);
      // chroma blocks 2 samples wide keep the plain inter prediction (DecCu.cpp:701, IntraPrediction.cpp:746)
      const int ncomp = c.cw > 2 ? 3 : 1;
      int id[3];
      for (int comp = 0; comp < ncomp; comp++) {
        const int ch = comp ? 1 : 0;
        IntraJob j = base(c, comp);
        j.x = j.cx; j.y = j.cy; j.w = j.cw; j.h = j.ch;
        j.flags = IJ_CIIP;
        j.mode = 0;
        j.ciip_w = (uint8_t)wIntra;
        int lev = ref_level(ch, comp, j.x, j.y, 2 * j.w, 2 * j.h, 0);
        if (comp > 0 && cscale && j.w * j.h > 4) lev = std::max(lev, set_cscale(j, c.x, c.y));
        id[comp] = push(lev + 1, j);
      }
      int lev = 0;
      for (auto it = jobs.end() - ncomp; it != jobs.end(); ++it) lev = std::max(lev, it->first);
      mark(ci, 0, c.x, c.y, c.w, c.h, lev, true, 0, id[0]);
      if (ncomp == 3) {
        mark(ci, 1, c.cx, c.cy, c.cw, c.ch, lev, true, 1, id[1]);
        mark(ci, 1, c.cx, c.cy, c.cw, c.ch, lev, false, 2, id[2]);
      } else if (c.cvalid) {
        inter_chroma(ci);
      }
      return;
    }
    // plain inter: level 0, reconstructed before the intra waves (by k_mc itself when fused: no tiles);
    // with LMCS chroma residual scaling the chroma scale depends on reconstructed luma next to the VPDU,
    // so the chroma becomes a step
    const bool chromaStep = cscale && c.cvalid;
    if (!(fuse && fused_inter_cu(pp, d, c)))
      for (int y = 0; y < c.h; y += 16)
      for (int x = 0; x < c.w; x += 16) {
        ReconTile t{};
        t.x = (int16_t)(c.x + x); t.y = (int16_t)(c.y + y);
        t.w = (uint8_t)std::min(16, c.w - x); t.h = (uint8_t)std::min(16, c.h - y);
        t.comps = (uint8_t)((c.yvalid ? 1 : 0) | (c.cvalid && !chromaStep ? 2 : 0));
        if (t.comps) out.inter_tiles.push_back(t);
      }
    cu_seq[ci] = seq;   // its units: level 0, no producer (reconstructed before the intra waves)
    if (chromaStep) inter_chroma_step(ci);
  }

  // the chroma of an inter CU on its own (a CIIP CU whose chroma is not blended)
  void inter_chroma(int ci) {
    const vvcr_cu &c = d.cu[ci];
    if (cscale) {
      inter_chroma_step(ci);
      return;
    }
    for (int y = 0; y < c.h; y += 16)
      for (int x = 0; x < c.w; x += 16) {
        ReconTile t{};
        t.x = (int16_t)(c.x + x); t.y = (int16_t)(c.y + y);
        t.w = (uint8_t)std::min(16, c.w - x); t.h = (uint8_t)std::min(16, c.h - y);
        t.comps = 2;
        out.inter_tiles.push_back(t);
      }
    cu_seq[ci] = seq;
  }

  void inter_chroma_step(int ci) {
    const vvcr_cu &c = d.cu[ci];
    int id[3] = {-1, -1, -1}, lev = 0;
    for (int comp = 1; comp < 3; comp++) {
      IntraJob j = base(c, comp);
      j.x = j.cx; j.y = j.cy; j.w = j.cw; j.h = j.ch;
      j.xkind = XK_INTER_CHROMA;
      const int l = 1 + set_cscale(j, c.x, c.y);
      id[comp] = push(l, j);
      lev = std::max(lev, l);
    }
    mark(ci, 1, c.cx, c.cy, c.cw, c.ch, lev, true, 1, id[1]);
    mark(ci, 1, c.cx, c.cy, c.cw, c.ch, lev, false, 2, id[2]);
  }

  void intra_luma(int ci) {
    const vvcr_cu &c = d.cu[ci];
    const vvcr_pu &p = d.pu[c.firstpu];
    if (c.isp) {
      const bool ver = c.isp == 2;   // ISPType: 1 HOR_INTRA_SUBPARTITIONS, 2 VER_INTRA_SUBPARTITIONS
      const bool regDiff = ver && ((c.w == 8 && c.h > 4) || c.w == 4);
      // prediction regions in order (TBs, or 4-wide regions covering several 1/2-wide TBs)
      std::vector<std::array<int, 4>> regs;
      for (int t = c.firsttu; t < c.firsttu + c.ntu; t++) {
        const int32_t *b = d.tu[t].b[0];
        if (b[2] <= 0) continue;
        if (regDiff) {
          if ((b[0] - c.x) % 4 == 0) regs.push_back({b[0], b[1], 4, b[3]});
        } else {
          regs.push_back({b[0], b[1], b[2], b[3]});
        }
      }
      // one step runs all regions in order: region k > 0 reads only the CU-level reference lines
      // and region k-1 (initIntraPatternChTypeISP), both available to the step itself
      if (regs.empty()) return;
      seq++;
      IntraJob j = base(c, 0);
      j.x = (int16_t)regs[0][0]; j.y = (int16_t)regs[0][1]; j.w = (uint8_t)regs[0][2]; j.h = (uint8_t)regs[0][3];
      j.flags = ver ? IJ_ISP_VER : IJ_ISP_HOR;
      j.mode = (uint8_t)p.fidir_l;
      j.isp_k = (uint8_t)regs.size();
      const int fTop = ver ? 2 * c.w : c.w + j.w, fLeft = ver ? c.h + j.h : 2 * c.h;
      const int lev = 1 + ref_level(0, 0, c.x, c.y, fTop, fLeft, 0);
      const int id = push(lev, j);
      mark(ci, 0, c.x, c.y, c.w, c.h, lev, true, 0, id);   // setDecomp of the whole CU (DecCu.cpp:288-291)
      seq += (int)regs.size() - 1;
      return;
    }
    for (int t = c.firsttu; t < c.firsttu + c.ntu; t++) {
      const int32_t *b = d.tu[t].b[0];
      if (b[2] <= 0) continue;
      seq++;
      IntraJob j = base(c, 0);
      j.x = (int16_t)b[0]; j.y = (int16_t)b[1]; j.w = (uint8_t)b[2]; j.h = (uint8_t)b[3];
      j.mrl = (uint8_t)p.mrl;
      if (c.bdpcm) { j.flags = IJ_BDPCM; j.mode = (uint8_t)c.bdpcm; }
      else if (c.mip) { j.flags = IJ_MIP | (p.mipt ? IJ_MIP_T : 0); j.mode = (uint8_t)p.idir_l; }
      else j.mode = (uint8_t)p.fidir_l;
      const int lev = 1 + ref_level(0, 0, j.x, j.y, 2 * j.w, 2 * j.h, j.mrl);
      const int id = push(lev, j);
      mark(ci, 0, j.x, j.y, j.w, j.h, lev, true, 0, id);
    }
  }

  void intra_chroma(int ci) {
    const vvcr_cu &c = d.cu[ci];
    const vvcr_pu &p = d.pu[c.firstpu];
    const bool dual = c.chtype == 1;
    for (int t = c.firsttu; t < c.firsttu + c.ntu; t++) {
      int cclm_lev = -1, cclm_box[4] = {0, 0, 0, 0};   // Cb's CCLM luma dependencies, reused by Cr (same block)
      cclm_deps.clear();
      for (int comp = 1; comp < 3; comp++) {
        const int32_t *b = d.tu[t].b[comp];
        if (b[2] <= 0) continue;
        seq++;
        IntraJob j = base(c, comp);
        j.x = (int16_t)b[0]; j.y = (int16_t)b[1]; j.w = (uint8_t)b[2]; j.h = (uint8_t)b[3];
        if (c.bdpcmc) { j.flags = IJ_BDPCM; j.mode = (uint8_t)c.bdpcmc; }
        else j.mode = (uint8_t)p.fidir_c;
        if (dual) j.flags |= IJ_DUAL;
        int lev = ref_level(1, comp, j.x, j.y, 2 * j.w, 2 * j.h, 0);
        if (!c.bdpcmc && p.fidir_c >= 67) {
          // CCLM (xGetLumaRecPixels IntraPrediction.cpp:1316-1650): the co-located luma block, the luma
          // rows above it (with the above-right extension, up to twice the width) and the columns left of
          // it (with the below-left extension); the strips are taken 4 samples deep
          const int lx = 2 * j.x, ly = 2 * j.y;
          if (cclm_lev >= 0 && cclm_box[0] == j.x && cclm_box[1] == j.y && cclm_box[2] == j.w && cclm_box[3] == j.h) {
            lev = std::max(lev, cclm_lev);
            for (int32_t pr : cclm_deps) add_dep(pr);
          } else {
            const size_t c0 = cur.size();   // the luma producers follow the chroma ones (disjoint sets)
            int cl = max_level(0, 0, lx, ly, lx + 2 * j.w - 1, ly + 2 * j.h - 1);
            cl = std::max(cl, max_level(0, 0, lx - 4, ly - 4, lx + 4 * j.w - 1, ly - 1));
            cl = std::max(cl, max_level(0, 0, lx - 4, ly, lx - 1, ly + 4 * j.h - 1));
            lev = std::max(lev, cl);
            cclm_lev = cl;
            cclm_box[0] = j.x; cclm_box[1] = j.y; cclm_box[2] = j.w; cclm_box[3] = j.h;
            cclm_deps.assign(cur.begin() + c0, cur.end());
          }
        }
        if (cscale && j.w * j.h > 4) lev = std::max(lev, set_cscale(j, 2 * j.x, 2 * j.y));
        lev += 1;
        const int id = push(lev, j);
        mark(ci, 1, j.x, j.y, j.w, j.h, lev, true, comp, id);
      }
    }
  }

  // ---- availability, as the reference evaluates it when the step runs (final order map: a unit is
  // decoded before step s iff order < s)
  // reg: the region of the step being resolved (low 32 bits) and, with WPP, its CTU column (high 32 bits:
  // getCURestricted returns no CU at a CTU column beyond the current one, CodingStructure.cpp:1524-1528)
  bool av(int ch, int x, int y, int sq, int64_t reg) const {
    const int pw = ch ? sp.width / 2 : sp.width, ph = ch ? sp.height / 2 : sp.height;
    if (x < 0 || y < 0 || x >= pw || y >= ph) return false;
    const int s = ch ? 1 : 2, cs = ch ? 1 : 0;
    if (((x << cs) >> sp.ctu_log2) > (int)(reg >> 32)) return false;
    return order_of(ch, (size_t)(y >> s) * W4 + (x >> s)) < sq && region_at(x << cs, y << cs) == (int)(uint32_t)reg;
  }
  // the availability key of a step at luma position (lx, ly)
  int64_t av_key(int lx, int ly) const {
    const int64_t col = pp.entropy_sync ? (lx >> sp.ctu_log2) : 0x7fffffff;
    return (int64_t)(uint32_t)region_at(lx, ly) | col << 32;
  }
  // xFillReferenceSamples unit scan (IntraPrediction.cpp:913-986, isAboveAvailable etc. :1208-1310):
  // returns the 65-bit availability mask in (lo, hi)
  struct FillShape {
    bool prefix, corner;
    int nul, nut;
  };
  void fill_mask(int ch, int sq, int64_t reg, int fx, int fy, int fw, int fh, int predSize, int predHSize, uint64_t &lo, uint32_t &hi,
                 FillShape *shape = nullptr) const {
    const int uw = ch ? 2 : 4, uh = uw;
    const int totalAbove = (predSize + uw - 1) / uw, totalLeft = (predHSize + uh - 1) / uh;
    const int numAbove = std::max(fw / uw, 1), numLeft = std::max(fh / uh, 1);
    const int numAR = totalAbove - numAbove, numBL = totalLeft - numLeft;
    bool F[2 * 64 + 1] = {};
    F[totalLeft] = av(ch, fx - 1, fy - 1, sq, reg);
    for (int i = 0; i < numAbove && av(ch, fx + i * uw, fy - 1, sq, reg); i++) F[totalLeft + 1 + i] = true;
    for (int i = 0; i < numAR && av(ch, fx + fw - 1 + uw + i * uw, fy - 1, sq, reg); i++) F[totalLeft + 1 + numAbove + i] = true;
    for (int i = 0; i < numLeft && av(ch, fx - 1, fy + i * uh, sq, reg); i++) F[totalLeft - 1 - i] = true;
    for (int i = 0; i < numBL && av(ch, fx - 1, fy + fh - 1 + uh + i * uh, sq, reg); i++) F[totalLeft - 1 - numLeft - i] = true;
    lo = 0; hi = 0;
    const int total = totalAbove + totalLeft + 1;
    if (total > 65) throw VvcrError(VVCR_E_STATE, "intra plan: more than 65 reference units");
    for (int u = 0; u < total; u++)
      if (F[u]) { if (u < 64) lo |= 1ull << u; else hi |= 1u << (u - 64); }
    if (shape) {   // corner + leading runs of each line; prefix if nothing is available after a gap
      FillShape &S = *shape;
      S.corner = F[totalLeft];
      S.nut = 0; S.nul = 0;
      while (S.nut < totalAbove && F[totalLeft + 1 + S.nut]) S.nut++;
      while (S.nul < totalLeft && F[totalLeft - 1 - S.nul]) S.nul++;
      S.prefix = true;
      for (int i = S.nut; i < totalAbove; i++) if (F[totalLeft + 1 + i]) S.prefix = false;
      for (int i = S.nul; i < totalLeft; i++) if (F[totalLeft - 1 - i]) S.prefix = false;
    }
  }
  // CCLM neighbourhood (above / left complete, above-right / below-left unit counts): 12 bits
  uint32_t nb_bits(int ch, int sq, int64_t reg, int x, int y, int w, int h, int unit) const {
    const int na = w / unit, nl = h / unit;
    int l = 0, a = 0, bl = 0, ar = 0;
    while (l < nl && av(ch, x - 1, y + l * unit, sq, reg)) l++;
    while (a < na && av(ch, x + a * unit, y - 1, sq, reg)) a++;
    const bool left = l == nl, above = a == na;
    if (left) while (bl < nl && av(ch, x - 1, y + h - 1 + unit + bl * unit, sq, reg)) bl++;
    if (above) while (ar < na && av(ch, x + w - 1 + unit + ar * unit, y - 1, sq, reg)) ar++;
    if (ar > 31 || bl > 31) throw VvcrError(VVCR_E_STATE, "intra plan: CCLM neighbourhood too large");
    return (above ? 1u : 0u) | (left ? 2u : 0u) | (uint32_t)ar << 2 | (uint32_t)bl << 7;
  }
  // (const: the steps resolve on several threads)
  void resolve_availability(IntraJob &j) const {
    const int comp = j.comp, ch = comp ? 1 : 0;
    const int64_t reg = av_key(j.cx << ch, j.cy << ch);
    const bool isp = (j.flags & (IJ_ISP_HOR | IJ_ISP_VER)) != 0, ver = (j.flags & IJ_ISP_VER) != 0;
    uint64_t lo;
    uint32_t hi;
    FillShape fs;
    int fx, fy, mrl = comp ? 0 : j.mrl;
    if (!isp) {
      fill_mask(ch, j.seq, reg, j.x, j.y, j.w, j.h, 2 * j.w, 2 * j.h, lo, hi, &fs);
      fx = j.x; fy = j.y;
    } else {
      const int fTop = ver ? 2 * j.cw : j.cw + j.w, fLeft = ver ? j.ch + j.h : 2 * j.ch;
      fill_mask(0, j.seq, reg, j.cx, j.cy, j.cw, j.ch, fTop, fLeft, lo, hi, &fs);
      fx = j.cx; fy = j.cy; mrl = 0;
    }
    if (fs.prefix && fs.nul < 256 && fs.nut < 256) {
      j.vnb |= CS_PREFIX | (fs.corner ? CS_CORNER : 0);
      j.nul = (uint8_t)fs.nul; j.nut = (uint8_t)fs.nut;
      // the available samples: top row x in [ox, ox + mrl + nut * unit], left column y in [oy, oy + mrl + nul * unit]
      const int us = ch ? 2 : 4, ox = fx - 1 - mrl, oy = fy - 1 - mrl;
      const int s = ch ? 1 : 0, t0x = (j.cx << s) >> sp.ctu_log2 << sp.ctu_log2 >> s, t0y = (j.cy << s) >> sp.ctu_log2 << sp.ctu_log2 >> s;
      const int tw = ctu >> s;
      const int xe = ox + mrl + fs.nut * us, ye = oy + mrl + fs.nul * us;
      const bool any = fs.corner || fs.nut || fs.nul;
      if (!any || (ox >= t0x && oy >= t0y && xe < t0x + tw && ye < t0y + tw)) j.vnb |= CS_INTILE;
    }
    j.av[0] = (uint32_t)lo;
    j.av[1] = (uint32_t)(lo >> 32);
    j.av[2] = hi;
    j.av[3] = 0;
    if (isp)
      for (int k = 1; k < j.isp_k && k < 4; k++) {
        const bool a = ver ? av(0, j.x + k * j.w, j.y - 1, j.seq, reg) : av(0, j.x - 1, j.y + k * j.h, j.seq, reg);
        if (a) j.av[2] |= 1u << (8 + k);
      }
    if (comp > 0 && j.mode >= 67 && !(j.flags & IJ_BDPCM)) {
      const bool dual = (j.flags & IJ_DUAL) != 0;
      const uint32_t lr = dual ? nb_bits(1, j.seq, reg, j.x, j.y, j.w, j.h, 2) : nb_bits(0, j.seq, reg, 2 * j.x, 2 * j.y, 2 * j.w, 2 * j.h, 4);
      const uint32_t lm = nb_bits(1, j.seq, reg, j.x, j.y, j.w, j.h, 2);
      j.av[2] |= lr << 16;
      j.av[3] = lm;
    }
  }

  // the CUs of CTUs ks (raster order) in decoding order per CTU (start / order: CSR over the CTUs)
  void plan_ctus(const std::vector<int> &ks, const std::vector<int> &start, const std::vector<int> &order) {
    for (int k : ks)
      for (int pass = 0; pass < (pp.dual_tree ? 2 : 1); pass++)
        for (int jx = start[k]; jx < start[k + 1]; jx++) {
          const int i = order[jx];
          const vvcr_cu &c = d.cu[i];
          if (pp.dual_tree && c.chtype != pass) continue;
          if (!in_shard(pp, c)) continue;   // another shard reconstructs it (different tile: never read here)
          cur_reg = ctu_reg[k];
          if (c.predmode == MODE_INTER) {
            inter_cu(i);
          } else if (c.predmode == MODE_INTRA) {
            if (c.yvalid) intra_luma(i);
            if (c.cvalid) intra_chroma(i);
          } else {
            throw VvcrError(VVCR_E_UNSUPPORTED, "IBC / palette CUs are not supported");
          }
        }
  }

  // Steps of every CTU with their dependencies. Nothing crosses a region (tile and slice: every neighbour
  // read is getCURestricted's), so with several regions each is planned by a planner of its own on
  // VVCR_PLAN_THREADS threads, sharing the unit / CU arrays, and their steps are appended region by region
  // (dependency indices moved by the steps before them); a CTU's steps stay contiguous, each region's are
  // in raster order of its CTUs. The steps equal the sequential plan's up to that order and the seq
  // numbers, which only order units inside one region.
  void plan_regions(const std::vector<int> &start, const std::vector<int> &order) {
    const int nctu = wc * ((sp.height + ctu - 1) / ctu);
    std::vector<std::vector<int>> groups;
    {
      std::vector<std::pair<int32_t, int>> key(nctu);
      for (int k = 0; k < nctu; k++) key[k] = {ctu_reg[k], k};
      std::stable_sort(key.begin(), key.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
      for (int q = 0; q < nctu; q++) {
        if (q == 0 || key[q].first != key[q - 1].first) groups.emplace_back();
        groups.back().push_back(key[q].second);
      }
    }
    const int ng = (int)groups.size();
    if (ng <= 1 || plan_threads() <= 1) {
      std::vector<int> all(nctu);
      for (int k = 0; k < nctu; k++) all[k] = k;
      plan_ctus(all, start, order);
      return;
    }
    std::sort(groups.begin(), groups.end(), [](const auto &a, const auto &b) { return a[0] < b[0]; });
    std::vector<std::unique_ptr<IntraPlan>> outs(ng);
    std::vector<std::unique_ptr<Planner>> subs(ng);
    for (int g = 0; g < ng; g++) {
      outs[g].reset(new IntraPlan());
      subs[g].reset(new Planner(sp, pp, d, *outs[g]));
      Planner &P = *subs[g];
      P.cscale = cscale; P.fuse = fuse; P.wc = wc; P.ctu_reg = ctu_reg; P.cu_seq = cu_seq; P.dense = dense;
      for (int k = 0; k < 2; k++) { P.umap[k] = umap[k]; P.ur[k] = ur[k]; P.written[k] = written[k]; }
    }
    std::vector<std::exception_ptr> err(ng);
    std::atomic<int> next{0};
    auto work = [&]() {
      for (int g; (g = next.fetch_add(1)) < ng;) {
        try {
          subs[g]->plan_ctus(groups[g], start, order);
        } catch (...) {
          err[g] = std::current_exception();
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min(plan_threads(), ng); t++) th.emplace_back(work);
    work();
    for (std::thread &t : th) t.join();
    for (const std::exception_ptr &e : err)
      if (e) std::rethrow_exception(e);
    for (int g = 0; g < ng; g++) {
      Planner &P = *subs[g];
      const int32_t jbase = (int32_t)jobs.size(), dbase = (int32_t)dep_flat.size();
      jobs.insert(jobs.end(), P.jobs.begin(), P.jobs.end());
      for (int32_t v : P.dep_flat) dep_flat.push_back(v + jbase);
      for (size_t i = 1; i < P.dep_off.size(); i++) dep_off.push_back(dbase + P.dep_off[i]);
      out.inter_tiles.insert(out.inter_tiles.end(), outs[g]->inter_tiles.begin(), outs[g]->inter_tiles.end());
    }
  }

  static int plan_threads() {
    static const int n = [] { const char *e = getenv("VVCR_PLAN_THREADS"); return e ? std::max(1, atoi(e)) : 4; }();
    return n;
  }

  void run() {
    static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
#define PROF_MARK(n)                                                                                             \
  if (prof) {                                                                                                    \
    auto t1 = std::chrono::steady_clock::now();                                                                  \
    fprintf(stderr, "  intra plan %-6s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t1 - t0).count()); \
    t0 = t1;                                                                                                     \
  }
    const size_t nu = (size_t)W4 * H4;
    // per-unit arrays without initialisation: only the units of written CUs are read (touch)
    // (resize would zero 7 arrays of a unit each per picture, 14 MB at 4K, for the few units a B picture plans);
    // a dense picture presets them (order kUnset: every unit read before it is decoded counts as not decoded)
    static const bool allow_dense = [] { const char *e = getenv("VVCR_PLAN_DENSE"); return !e || atoi(e) != 0; }();   // 0: off (tests)
    dense = allow_dense && std::none_of(d.cu.begin(), d.cu.end(), [](const vvcr_cu &c) { return c.predmode == MODE_INTER; });
    for (int k = 0; k < 2; k++) {
      ur_store[k].alloc(nu, false);
      ur[k] = ur_store[k].p;
      if (dense) std::memset((void *)ur[k], 0x7f, nu * sizeof(UnitRec));
    }
    cu_seq_store.assign(d.cu.size(), kInf);
    cu_seq = cu_seq_store.data();
    for (int k = 0; k < 2; k++) { written_store[k].assign(d.cu.size(), 0); written[k] = written_store[k].data(); }
    for (int k = 0; k < 2; k++) {
      if (d.cu_map[k].size() == nu) {   // the producer's CU maps (the host parser hands them over)
        umap[k] = d.cu_map[k].data();
        continue;
      }
      own_map[k].assign(nu, -1);
      for (size_t i = 0; i < d.cu.size(); i++) {
        const vvcr_cu &c = d.cu[i];
        if (k == 0 && c.yvalid)
          for (int uy = c.y >> 2; uy < (c.y + c.h) >> 2; uy++)
            for (int ux = c.x >> 2; ux < (c.x + c.w) >> 2; ux++) own_map[0][(size_t)uy * W4 + ux] = (int)i;
        if (k == 1 && c.cvalid)
          for (int uy = c.cy >> 1; uy < (c.cy + c.ch + 1) >> 1; uy++)
            for (int ux = c.cx >> 1; ux < (c.cx + c.cw + 1) >> 1; ux++) own_map[1][(size_t)uy * W4 + ux] = (int)i;
      }
      umap[k] = own_map[k].data();
    }
    wc = (sp.width + ctu - 1) / ctu;
    const int hc = (sp.height + ctu - 1) / ctu;
    const int ncu = (int)d.cu.size();
    {
      // tile of every CTU from the column / row boundaries, slice from the CUs it holds
      std::vector<int32_t> tcol(wc, 0), trow(hc, 0);
      const int ntc = std::max(1, pp.num_tile_cols), ntr = std::max(1, pp.num_tile_rows);
      if (pp.num_tile_cols > 0)
        for (int t = 0; t < ntc; t++)
          for (int x = pp.tile_col_bd[t]; x < pp.tile_col_bd[t + 1] && x < wc; x++) tcol[x] = t;
      if (pp.num_tile_rows > 0)
        for (int t = 0; t < ntr; t++)
          for (int y = pp.tile_row_bd[t]; y < pp.tile_row_bd[t + 1] && y < hc; y++) trow[y] = t;
      ctu_reg_store.assign((size_t)wc * hc, 0);
      for (int y = 0; y < hc; y++)
        for (int x = 0; x < wc; x++) ctu_reg_store[(size_t)y * wc + x] = (trow[y] * ntc + tcol[x]) << 16;
      for (const vvcr_cu &c : d.cu) {
        const int x = c.yvalid ? c.x : 2 * c.cx, y = c.yvalid ? c.y : 2 * c.cy;
        int32_t &r = ctu_reg_store[(size_t)(y >> sp.ctu_log2) * wc + (x >> sp.ctu_log2)];
        r = (r & ~0xffff) | (c.slice & 0xffff);
      }
      ctu_reg = ctu_reg_store.data();
    }
    std::vector<int> start((size_t)wc * hc + 1, 0), order(ncu), ctu_of(ncu);
    for (int i = 0; i < ncu; i++) {
      const vvcr_cu &c = d.cu[i];
      const int x = c.yvalid ? c.x : 2 * c.cx, y = c.yvalid ? c.y : 2 * c.cy;
      ctu_of[i] = (y >> sp.ctu_log2) * wc + (x >> sp.ctu_log2);
      start[ctu_of[i] + 1]++;
    }
    for (int k = 0; k < wc * hc; k++) start[k + 1] += start[k];
    {
      std::vector<int> pos(start);
      for (int i = 0; i < ncu; i++) order[pos[ctu_of[i]]++] = i;
    }
    plan_regions(start, order);
    PROF_MARK("jobs");
    // Steps grouped by CTU (raster order), inside a CTU by level: a topological order of the dependency
    // graph (every dependency is in the same CTU at a lower level, or in an earlier CTU — the left /
    // above neighbours). k_intra runs one CTU per workgroup with the CTU's samples in LDS; a dependency
    // inside the CTU is encoded as its local index (>= 0), one in another CTU as ~(global index), and
    // the producing step is flagged IJ_PUBLISH (drains its global stores and raises a global flag).
    const int nj = (int)jobs.size();
    std::vector<int32_t> ctu_of_job(nj);
    {
      std::vector<uint8_t> seen((size_t)wc * hc, 0);
      for (int i = 0; i < nj; i++) {
        const IntraJob &j = jobs[i].second;
        const int s = j.comp ? 1 : 0;
        const int lx = j.cx << s, ly = j.cy << s;   // CU position in luma samples (a CU never crosses a CTU)
        ctu_of_job[i] = (ly >> sp.ctu_log2) * wc + (lx >> sp.ctu_log2);
        if (i && ctu_of_job[i] == ctu_of_job[i - 1]) continue;
        if (seen[ctu_of_job[i]]) throw VvcrError(VVCR_E_STATE, "intra plan: a CTU's steps are not contiguous");
        seen[ctu_of_job[i]] = 1;
      }
    }
    // the steps of one CTU are contiguous in creation order: blocks [cb[k], cb[k+1])
    std::vector<int32_t> cb;
    for (int i = 0; i < nj; i++)
      if (i == 0 || ctu_of_job[i] != ctu_of_job[i - 1]) cb.push_back(i);
    cb.push_back(nj);
    auto D = [&](int i) { return std::make_pair(dep_flat.data() + dep_off[i], dep_flat.data() + dep_off[i + 1]); };
    // Take order inside a CTU: a topological order that prefers the steps with the longest chain of
    // dependent work behind them (list scheduling by bottom level). The kernel's waves take steps in this
    // order, so the critical chain is started as early as its dependencies allow. Step costs are rough
    // estimates in microseconds (measured per step kind on MI355X, tools/iprof_ctu.py).
    std::vector<double> bl(nj, 0.0), maxsucc(nj, 0.0), cost(nj, 0.0), fin(nj, 0.0);
    static const bool take_order_bl = [] { const char *e = getenv("VVCR_TAKE_ORDER"); return e && !strcmp(e, "bl"); }();
    static const double take_alpha = [] { const char *e = getenv("VVCR_TAKE_ALPHA"); return e ? atof(e) : 2.5; }();
    for (int i = nj - 1; i >= 0; i--) {   // creation order is topological (dependencies are earlier)
      const IntraJob &j = jobs[i].second;
      const bool isp = (j.flags & (IJ_ISP_HOR | IJ_ISP_VER)) != 0;
      const double c = 3.0 + 0.002 * j.w * j.h * (isp ? j.isp_k : 1) + (isp ? 1.6 * (j.isp_k - 1) : 0.0) +
                       ((j.flags & IJ_MIP) ? 2.5 : 0.0) + ((j.comp && j.mode >= 67) ? 3.0 : 0.0);
      cost[i] = c;
      bl[i] = c + maxsucc[i];
      for (auto [p, e] = D(i); p != e; ++p) maxsucc[*p] = std::max(maxsucc[*p], bl[i]);
    }
    PROF_MARK("bl");
    // Wait lists: a same-CTU dependency that another dependency of the step already reaches through
    // same-CTU dependencies is implied (that one could only finish after it: flags are raised after the
    // step's stores complete, LDS is coherent inside the CU), so the kernel need not poll it. Bitsets of
    // same-CTU ancestors per CTU block, in creation order (topological). Cross-CTU dependencies are all
    // kept: they also decide which steps publish their samples to HBM.
    std::vector<int32_t> wd_off(nj + 1, 0), wd_flat;
    wd_flat.reserve(dep_flat.size());
    // In-CTU take order (list scheduling by bottom level) in the same pass over the CTU blocks.
    std::vector<int32_t> perm;
    perm.reserve(nj);
    {
      std::vector<uint64_t> anc, implied;
      std::vector<int32_t> indeg, soff, sflat;
      for (size_t k = 0; k + 1 < cb.size(); k++) {
        const int b0 = cb[k], n = cb[k + 1] - b0, words = (n + 63) / 64;
        anc.assign((size_t)n * words, 0);
        implied.assign(words, 0);
        for (int i = b0; i < b0 + n; i++) {
          const int li = i - b0;
          uint64_t *a = anc.data() + (size_t)li * words;
          const int lw = (li >> 6) + 1;   // ancestors of step li are < li
          std::fill(implied.begin(), implied.begin() + lw, 0);
          for (auto [p, e] = D(i); p != e; ++p) {
            const int dd = *p;
            if (dd < b0) continue;
            const int ld = dd - b0;
            const uint64_t *ad = anc.data() + (size_t)ld * words;
            for (int w = 0; w <= (ld >> 6); w++) { a[w] |= ad[w]; implied[w] |= ad[w]; }
            a[ld >> 6] |= 1ull << (ld & 63);
          }
          for (auto [p, e] = D(i); p != e; ++p) {
            const int dd = *p;
            if (dd >= b0) {
              const int ld = dd - b0;
              if (implied[ld >> 6] >> (ld & 63) & 1) continue;
            }
            wd_flat.push_back(dd);
          }
          wd_off[i + 1] = (int32_t)wd_flat.size();
        }
        // successors inside the CTU (CSR over local indices) and in-degrees
        indeg.assign(n, 0);
        soff.assign(n + 1, 0);
        for (int i = b0; i < b0 + n; i++)
          for (auto [p, e] = D(i); p != e; ++p)
            if (*p >= b0) { indeg[i - b0]++; soff[*p - b0 + 1]++; }
        for (int q = 0; q < n; q++) soff[q + 1] += soff[q];
        sflat.assign(soff[n], 0);
        {
          std::vector<int32_t> pos(soff.begin(), soff.end() - 1);
          for (int i = b0; i < b0 + n; i++)
            for (auto [p, e] = D(i); p != e; ++p)
              if (*p >= b0) sflat[pos[*p - b0]++] = i - b0;
        }
        int taken = 0;
        if (take_order_bl) {
          auto cmp = [&](int32_t x, int32_t y) { return bl[b0 + x] < bl[b0 + y] || (bl[b0 + x] == bl[b0 + y] && x > y); };
          std::priority_queue<int32_t, std::vector<int32_t>, decltype(cmp)> ready(cmp);
          for (int q = 0; q < n; q++) if (indeg[q] == 0) ready.push(q);
          while (!ready.empty()) {
            const int32_t x = ready.top();
            ready.pop();
            perm.push_back(b0 + x);
            taken++;
            for (int t = soff[x]; t < soff[x + 1]; t++) if (--indeg[sflat[t]] == 0) ready.push(sflat[t]);
          }
        } else {
          // Take order from a timing simulation of the kernel: kNW waves take steps in list order, a wave
          // that takes a step waits for its dependencies, then runs it for its estimated cost. Each time a
          // wave frees up, the list gets the step (among those whose same-CTU dependencies are already in
          // the list) with the longest chain behind it, less VVCR_TAKE_ALPHA (2.5) times the idle time it
          // would cost that wave. Dependencies on other CTUs use the finish times simulated for those CTUs
          // (raster order: they come first; all CTU workgroups start together). A pure bottom-level order
          // (VVCR_TAKE_ORDER=bl, r01) lets ready steps queue behind steps that wait on another CTU; pure
          // earliest-start delays the critical chain. Measured (k_intra, median of 20): 1080p I picture
          // 5.67 (bl) -> 5.59 ms, 4K 12.25 -> 11.97 ms; earliest-start first 6.67 / 14.8 ms.
          constexpr int kNW = kIntraWaves;
          constexpr double kLocal = 0.3, kGlobal = 1.5;   // hand-off latencies (us)
          double wfree[kNW] = {};
          std::vector<double> rdy(n, 0.0);
          std::vector<int32_t> known;
          auto make_known = [&](int q) {
            double r = 0;
            for (auto [p, e] = D(b0 + q); p != e; ++p) r = std::max(r, fin[*p] + (*p >= b0 ? kLocal : kGlobal));
            rdy[q] = r;
            known.push_back(q);
          };
          for (int q = 0; q < n; q++) if (indeg[q] == 0) make_known(q);
          while (!known.empty()) {
            int w = 0;
            for (int k = 1; k < kNW; k++) if (wfree[k] < wfree[w]) w = k;
            const double t = wfree[w];
            // priority: the chain behind the step, less the wave idle time it would cost (alpha per us)
            size_t best = 0;
            double bs = std::max(t, rdy[known[0]]), bk = bl[b0 + known[0]] - take_alpha * (bs - t);
            for (size_t k = 1; k < known.size(); k++) {
              const double st = std::max(t, rdy[known[k]]);
              const int q = known[k], qb = known[best];
              const double key = bl[b0 + q] - take_alpha * (st - t);
              if (key > bk + 1e-9 || (key > bk - 1e-9 && q < qb)) {
                best = k;
                bs = st;
                bk = key;
              }
            }
            const int x = known[best];
            known[best] = known.back();
            known.pop_back();
            fin[b0 + x] = bs + cost[b0 + x];
            wfree[w] = fin[b0 + x];
            perm.push_back(b0 + x);
            taken++;
            for (int t2 = soff[x]; t2 < soff[x + 1]; t2++) if (--indeg[sflat[t2]] == 0) make_known(sflat[t2]);
          }
        }
        if (taken != n) throw VvcrError(VVCR_E_STATE, "intra plan: dependency cycle inside a CTU");
      }
    }
    PROF_MARK("wdeps");
    // CTU order of the launch: wavefront (anti-diagonals x + 2y, the lower CTU of a diagonal first: 4K
    // I picture -1 %; VVCR_CTU_ORDER=raster for the raster order). Every cross-CTU dependency (left, above-left, above, above-right) is on an earlier CTU in
    // both orders, so a workgroup only ever waits for CTUs already taken; in wavefront order the CTUs
    // taken but not finished are the few on the active diagonals, so a launch of a few dozen workgroups
    // keeps the whole wavefront busy (raster order needs about a row of CTUs per active row).
    {
      static const int order_kind = [] {   // 0 wavefront, lower CTU of a diagonal first; 1 raster; 2 upper first
        const char *e = getenv("VVCR_CTU_ORDER");
        return !e ? 0 : (!strcmp(e, "raster") ? 1 : (!strcmp(e, "wf_up") ? 2 : 0));
      }();
      const bool raster = order_kind == 1;
      const int nb = (int)cb.size() - 1;
      if (!raster && nb > 1) {
        std::vector<int32_t> bo(nb);
        for (int k = 0; k < nb; k++) bo[k] = k;
        auto key = [&](int k) {
          const int c = ctu_of_job[cb[k]], x = c % wc, y = c / wc;
          return std::make_pair(x + 2 * y, order_kind == 2 ? y : -y);
        };
        std::stable_sort(bo.begin(), bo.end(), [&](int a, int b) { return key(a) < key(b); });
        std::vector<int32_t> p2;
        p2.reserve(nj);
        for (int k : bo) p2.insert(p2.end(), perm.begin() + cb[k], perm.begin() + cb[k + 1]);
        perm.swap(p2);
      }
    }
    std::vector<int32_t> rank(nj);
    for (int i = 0; i < nj; i++) rank[perm[i]] = i;
    out.jobs.resize(nj);
    out.dep_start.assign(nj + 1, 0);
    out.deps.clear();
    out.deps.reserve(wd_flat.size());
    out.ctu_list.clear();
    out.ctu_start.clear();
    for (int i = 0; i < nj; i++) {
      const int32_t o = perm[i];
      if (out.ctu_list.empty() || out.ctu_list.back() != ctu_of_job[o]) {
        out.ctu_list.push_back(ctu_of_job[o]);
        out.ctu_start.push_back(i);
      }
      out.jobs[i] = jobs[o].second;
    }
    out.ctu_start.push_back(nj);
    for (size_t c = 0; c + 1 < out.ctu_start.size(); c++)
      if (out.ctu_start[c + 1] - out.ctu_start[c] > kIntraMaxStepsPerCtu)
        throw VvcrError(VVCR_E_UNSUPPORTED, "intra plan: more steps in one CTU than the kernel's LDS flag array holds");
    int c = 0;
    for (int i = 0; i < nj; i++) {
      while (out.ctu_start[c + 1] <= i) c++;
      const int32_t o = perm[i];
      for (auto [p, e] = D(o); p != e; ++p) {
        const int32_t rd = rank[*p];
        if (rd >= i) throw VvcrError(VVCR_E_STATE, "intra plan: dependency is not earlier in step order");
        if (rd < out.ctu_start[c]) out.jobs[rd].flags |= IJ_PUBLISH;
      }
      for (int t = wd_off[o]; t < wd_off[o + 1]; t++) {
        const int32_t rd = rank[wd_flat[t]];
        out.deps.push_back(rd >= out.ctu_start[c] ? rd - out.ctu_start[c] : ~rd);
      }
      out.dep_start[i + 1] = (int32_t)out.deps.size();
    }
    PROF_MARK("final");
    // per step, independent of the others (the final order map is read-only now): a large plan (an
    // intra picture, ~70 k steps at 4K) splits the steps over VVCR_PLAN_THREADS (4) threads
    auto resolve = [&](size_t a, size_t b) {
      for (size_t k = a; k < b; k++) {
        IntraJob &j = out.jobs[k];
        if (j.xkind == XK_INTER_CHROMA) continue;   // inter chroma steps read no reference samples
        resolve_availability(j);
        set_pred_params(j);
      }
    };
    const int nthr = plan_threads();
    const size_t njobs = out.jobs.size();
    if (njobs >= 16384 && nthr > 1) {
      std::vector<std::exception_ptr> err(nthr);
      auto part = [&](int t) {
        try {
          resolve(njobs * t / nthr, njobs * (t + 1) / nthr);
        } catch (...) {
          err[t] = std::current_exception();
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < nthr; t++) th.emplace_back(part, t);
      part(0);
      for (std::thread &t : th) t.join();
      for (const std::exception_ptr &e : err)
        if (e) std::rethrow_exception(e);
    } else {
      resolve(0, njobs);
    }
    PROF_MARK("avail");
  }
};

}  // namespace

void plan_intra(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, IntraPlan &out, bool fuse) {
  out.clear();
  auto P = std::make_unique<Planner>(sp, pp, d, out);
  P->cscale = pp.lmcs_enabled && pp.lmcs_chroma_scale;
  P->fuse = fuse;
  P->run();
  // VVCR_PLAN_HASH (diagnostics): one FNV-1a hash of the whole plan per picture on stderr, to show that a
  // planner change leaves its output unchanged
  static const bool hash = getenv("VVCR_PLAN_HASH") != nullptr;
  if (hash) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
      for (size_t k = 0; k < n; k++) h = (h ^ ((const uint8_t *)p)[k]) * 1099511628211ull;
    };
    mix(out.jobs.data(), out.jobs.size() * sizeof(IntraJob));
    mix(out.dep_start.data(), out.dep_start.size() * sizeof(int32_t));
    mix(out.deps.data(), out.deps.size() * sizeof(int32_t));
    mix(out.ctu_list.data(), out.ctu_list.size() * sizeof(int32_t));
    mix(out.ctu_start.data(), out.ctu_start.size() * sizeof(int32_t));
    mix(out.inter_tiles.data(), out.inter_tiles.size() * sizeof(ReconTile));
    fprintf(stderr, "intra plan hash %016llx steps %zu\n", (unsigned long long)h, out.jobs.size());
  }
}

// Diagnostics (host only, no device): the intra plan of one picture's descriptors. Per step
// out[k*8 + {0..7}] = x, y, comp, w, h, flags, isp_k, seq; deps in CSR form (dep_start[n+1], deps).
// Returns the number of steps (or a negative error); counts[0] = steps, counts[1] = dependencies.
extern "C" int vvcr_debug_plan_intra(const vvcr_seq_params *sp, const vvcr_pic_params *pp, const vvcr_cu *cu, int32_t ncu,
                                     const vvcr_pu *pu, int32_t npu, const vvcr_tu *tu, int32_t ntu, int32_t *out,
                                     int32_t cap, int32_t *dep_start, int32_t *deps, int32_t dcap, int32_t *counts) {
  try {
    PictureDescriptors d;
    d.cu.assign(cu, cu + ncu);
    d.pu.assign(pu, pu + npu);
    d.tu.assign(tu, tu + ntu);
    IntraPlan ip;
    plan_intra(*sp, *pp, d, ip, false);
    const int n = (int)ip.jobs.size();
    counts[0] = n;
    counts[1] = (int)ip.deps.size();
    if (n > cap || (int)ip.deps.size() > dcap) return n;
    for (int k = 0; k < n; k++) {
      const IntraJob &j = ip.jobs[k];
      const int32_t r[8] = {j.x, j.y, j.comp, j.w, j.h, j.flags, j.isp_k, j.seq};
      memcpy(out + 8 * k, r, sizeof r);
    }
    memcpy(dep_start, ip.dep_start.data(), (n + 1) * sizeof(int32_t));
    memcpy(deps, ip.deps.data(), ip.deps.size() * sizeof(int32_t));
    return n;
  } catch (const VvcrError &e) {
    return e.code;
  }
}
