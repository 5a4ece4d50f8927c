// vvcr_dbk_host.cpp — deblocking edge planning (host producer side).
//
// Derives, for every 4-sample edge segment of the picture, the parameters the deblocking decision
// needs: boundary strength per component, maximum filter lengths, and the P/Q average QPs. This is
// the control part of LoopFilter::xDeblockCU (source/Lib/CommonLib/LoopFilter.cpp:261-408):
// edge flags and TU/PU markers (xSetEdgefilterMultiple :627), filter lengths from transform sizes
// (:454) and for SbTMVP/affine sub-blocks (:550), xGetBoundaryStrengthSingle (:674), and the QP / length
// bookkeeping of xEdgeFilterLuma (:844-979) and xEdgeFilterChroma (:1087-1244). The sample decisions
// and filtering run on the GPU (vvcr_dbk.hip). Each CU writes only edge positions inside its own area,
// so the per-CTU state of the reference reduces to per-CU work over picture-wide maps.
#include "vvcr_dbk.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

namespace {

enum { VER = 0, HOR = 1 };
enum { BX = 0, BY, BW, BH, BCBF };
constexpr int MODE_INTRA = 1;
constexpr int MRG_TYPE_SUBPU_ATMVP = 1;

// Picture-wide lookup state, built once and then only read (the CTU workers share it): CU and TU index
// maps on the 4x4 luma / 2x2 chroma grid, and the chroma QPs of every TU.
struct Maps {
  bigbuf::vec<int> own_cu_map[2], tu_map[2];
  const int32_t *cu_map[2] = {nullptr, nullptr};   // the producer's CU maps when handed over, else own_cu_map
  bigbuf::vec<int8_t> cqp;                         // [TU][Cb, Cr] QpParam(tu, comp).Qp(0) - qpBdOffset
};

struct Planner {
  const vvcr_seq_params &sp;
  const vvcr_pic_params &pp;
  const PictureDescriptors &d;
  DbkLists &out;
  Maps &M;
  int W4, H4, ctu, parts;
  bigbuf::vec<int> (&own_cu_map)[2] = M.own_cu_map;
  bigbuf::vec<int> (&tu_map)[2] = M.tu_map;
  const int32_t *(&cu_map)[2] = M.cu_map;
  // per-CU scratch in CTU-relative coordinates (the reference's per-CTU arrays, LoopFilter.h:66-79)
  int ctu_x = 0, ctu_y = 0;
  uint8_t bs[2][32 * 32];
  uint8_t edge[2][32 * 32];
  // edge lengths / transform-edge flags on the edge grid of the CTU: 4x4 luma units, 2x2 chroma units
  // (edges off the grid, ISP sub-partitions 1 or 2 samples wide, are never filtered nor read)
  uint8_t lenP[3][32][32], lenQ[3][32][32], tedge[32][32];
  bool left = false, top = false, internal = false;
  const std::vector<uint8_t> &lf_nb;   // lf_ctb_neighbours, or empty

  Planner(const vvcr_seq_params &s, const vvcr_pic_params &p, const PictureDescriptors &dd, DbkLists &o, Maps &m,
          const std::vector<uint8_t> &nb)
      : sp(s), pp(p), d(dd), out(o), M(m), lf_nb(nb) {
    W4 = sp.width / 4;
    H4 = sp.height / 4;
    ctu = 1 << sp.ctu_log2;
    parts = ctu / 4;
  }

  int get_cu(int x, int y, int ch) const {
    const int s = ch ? 1 : 2;
    const int i = cu_map[ch][(size_t)(y >> s) * W4 + (x >> s)];
    if (i < 0) throw VvcrError(VVCR_E_ARG, "deblocking: no CU covers a neighbouring position");
    return i;
  }
  int get_tu(int x, int y, int ch) const {
    const int s = ch ? 1 : 2;
    int t = tu_map[ch][(size_t)(y >> s) * W4 + (x >> s)];
    if (t == -1) throw VvcrError(VVCR_E_ARG, "deblocking: no TU covers a neighbouring position");
    if (t >= 0) return t;   // (chroma maps and non-ISP luma TUs: no descriptor read, the common case)
    t = -t - 2;             // an ISP CU's area (the map holds -(first TU) - 2)
    {       // CodingStructure::getTU (CodingStructure.cpp:379): search the ISP sub-partitions
      for (int k = 0; k < 4 && t + k < (int)d.tu.size(); k++) {
        const int32_t *b = d.tu[t + k].b[0];
        if (x >= b[BX] && x < b[BX] + b[BW] && y >= b[BY] && y < b[BY] + b[BH]) return t + k;
      }
    }
    return t;
  }
  void fill(bigbuf::vec<int> &m, int x, int y, int w, int h, int s, int v) {
    for (int j = y >> s; j < (y + h + (1 << s) - 1) >> s; j++)
      for (int i = x >> s; i < (x + w + (1 << s) - 1) >> s; i++) m[(size_t)j * W4 + i] = v;
  }
  int raster(int x, int y) const { return ((x & (ctu - 1)) >> 2) + ((y & (ctu - 1)) >> 2) * parts; }

  static void cu_area(const vvcr_cu &c, int *a) {
    if (c.yvalid) { a[0] = c.x; a[1] = c.y; a[2] = c.w; a[3] = c.h; }
    else { a[0] = c.cx * 2; a[1] = c.cy * 2; a[2] = c.cw * 2; a[3] = c.ch * 2; }
  }

  void build_maps() {
    const size_t n = (size_t)W4 * H4;
    for (int k = 0; k < 2; k++) {
      tu_map[k].assign(n, -1);
      if (d.cu_map[k].size() == n) { cu_map[k] = d.cu_map[k].data(); continue; }
      own_cu_map[k].assign(n, -1);
      for (size_t i = 0; i < d.cu.size(); i++) {
        const vvcr_cu &c = d.cu[i];
        if (k == 0 && c.yvalid) fill(own_cu_map[0], c.x, c.y, c.w, c.h, 2, (int)i);
        if (k == 1 && c.cvalid) fill(own_cu_map[1], c.cx, c.cy, c.cw, c.ch, 1, (int)i);
      }
      cu_map[k] = own_cu_map[k].data();
    }
    for (size_t t = 0; t < d.tu.size(); t++) {
      const vvcr_cu &c = d.cu[d.tu[t].cu];
      const int32_t *b0 = d.tu[t].b[0], *b1 = d.tu[t].b[1];
      if (b0[BW] > 0 && b0[BH] > 0) {
        if (c.isp) {   // the first ISP TU owns the CU area in the index map (CodingStructure::addTU :624)
          if ((int)t == c.firsttu) fill(tu_map[0], c.x, c.y, c.w, c.h, 2, -(int)t - 2);   // flagged: get_tu searches
        } else {
          fill(tu_map[0], b0[BX], b0[BY], b0[BW], b0[BH], 2, (int)t);
        }
      }
      if (b1[BW] > 0 && b1[BH] > 0) fill(tu_map[1], b1[BX], b1[BY], b1[BW], b1[BH], 1, (int)t);
    }
    M.cqp.resize(2 * d.tu.size());
    for (size_t t = 0; t < d.tu.size(); t++)
      for (int comp = 1; comp <= 2; comp++) M.cqp[2 * t + comp - 1] = (int8_t)chroma_qp((int)t, comp);
  }

  void set_edges(int dir, int x, int y, int w, int h, bool val, bool edgeIdx) {
    const int add = dir == VER ? parts : 1, n = dir == VER ? h / 4 : w / 4;
    int idx = raster(x, y);
    for (int i = 0; i < n; i++, idx += add) {
      edge[dir][idx] = val;
      if (bs[dir][idx] && val) bs[dir][idx] = 3;
      else if (!edgeIdx) bs[dir][idx] = val;
    }
  }

  void len_from_tu(int dir, const vvcr_cu &cu, int t) {
    const vvcr_tu &tu = d.tu[t];
    for (int comp = 0; comp < 3; comp++) {
      const int ch = comp ? 1 : 0;
      const int32_t *b = tu.b[comp], *bch = tu.b[ch];
      if (b[BW] <= 0 || b[BH] <= 0) continue;
      const int cux = comp ? cu.cx : cu.x, cuy = comp ? cu.cy : cu.y;
      const int xo = b[BX] - (ctu_x >> ch), yo = b[BY] - (ctu_y >> ch);
      const int step = 4 >> ch;
      const bool horz = dir == HOR;
      if (!(horz ? (b[BY] == cuy ? top : internal) : (b[BX] == cux ? left : internal))) continue;
      const int n = horz ? b[BW] : b[BH];
      for (int k = 0; k < n; k += step) {
        const int qx = horz ? bch[BX] + k : bch[BX], qy = horz ? bch[BY] : bch[BY] + k;
        const int sizeQ = horz ? b[BH] : b[BW];
        const int tp = horz ? get_tu(qx, qy - 1, ch) : get_tu(qx - 1, qy, ch);
        const int sizeP = horz ? d.tu[tp].b[comp][BH] : d.tu[tp].b[comp][BW];
        const int X = horz ? xo + k : xo, Y = horz ? yo : yo + k;
        const int g = ch ? 1 : 2;   // log2 of the grid unit in component samples
        if ((X | Y) & ((1 << g) - 1)) continue;
        const int U = X >> g, V = Y >> g;
        if (comp == 0) {
          tedge[U][V] = 1;
          const bool small = sizeP <= 4 || sizeQ <= 4;
          lenQ[0][U][V] = small ? 1 : (sizeQ >= 32 ? 7 : 3);
          lenP[0][U][V] = small ? 1 : (sizeP >= 32 ? 7 : 3);
        } else {
          lenQ[comp][U][V] = lenP[comp][U][V] = (sizeQ >= 8 && sizeP >= 8) ? 3 : 1;
        }
      }
    }
  }

  void len_subblocks(int dir, const vvcr_pu &pu, int w, int h) {
    const int xo = pu.x - ctu_x, yo = pu.y - ctu_y;
    auto &Q = lenQ[0];
    auto &P = lenP[0];
    const bool horz = dir == HOR;
    const int outer = horz ? h : w, inner = horz ? w : h;
    for (int a = 0; a < outer; a += 8)
      for (int b = 0; b < inner; b += 4) {
        const int U = (horz ? xo + b : xo + a) >> 2, V = (horz ? yo + a : yo + b) >> 2;   // 4x4 units
        auto T = [&](int delta) { return horz ? tedge[U][V + (delta >> 2)] : tedge[U + (delta >> 2)][V]; };
        if (T(0)) {
          if (Q[U][V] > 5) Q[U][V] = 5;
          if (a > 0 && P[U][V] > 5) P[U][V] = 5;
        } else if (a > 0 && (T(-4) || a + 4 >= outer || T(4))) {
          Q[U][V] = P[U][V] = 1;
        } else if (a > 0 && (T(-8) || a + 8 >= outer || T(8))) {
          Q[U][V] = P[U][V] = 2;
        } else {
          Q[U][V] = P[U][V] = 3;
        }
      }
  }

  static int bs_set(int v, int comp) { return v << (comp * 2); }

  int boundary_strength(int cui, int dir, int lx, int ly) const {
    const vvcr_cu &cuQ = d.cu[cui];
    const int ch = cuQ.chtype;
    const int sh = cuQ.yvalid ? 0 : 1;
    const int qx = lx >> sh, qy = ly >> sh;
    const int px = dir == VER ? qx - 1 : qx, py = dir == VER ? qy : qy - 1;
    // an edge inside the CU (sub-block / TU edges): P is the same CU, without a map lookup
    const bool same = px >= (cuQ.yvalid ? cuQ.x : cuQ.cx) && py >= (cuQ.yvalid ? cuQ.y : cuQ.cy);
    const vvcr_cu &cuP = same ? cuQ : d.cu[get_cu(px, py, ch)];
    if (cuP.predmode == MODE_INTRA || cuQ.predmode == MODE_INTRA) {
      const int bsY = (cuP.predmode == MODE_INTRA && cuP.bdpcm) && (cuQ.predmode == MODE_INTRA && cuQ.bdpcm) ? 0 : 2;
      const int bsC = (cuP.predmode == MODE_INTRA && cuP.bdpcmc) && (cuQ.predmode == MODE_INTRA && cuQ.bdpcmc) ? 0 : 2;
      return bs_set(bsY, 0) + bs_set(bsC, 1) + bs_set(bsC, 2);
    }
    const int marker = bs[dir][raster(lx, ly)];
    const bool ciip = d.pu[cuQ.firstpu].ciip || (!same && d.pu[cuP.firstpu].ciip);
    if (marker && ciip) return bs_set(2, 0) + bs_set(2, 1) + bs_set(2, 2);
    int tmp = 0;
    if (marker) {   // transform edge: the coded-block flags of both sides (a sub-block-only edge has none)
      const int tqi = get_tu(qx, qy, ch);
      const int tpi = (same && cuQ.ntu == 1 && !cuQ.isp) ? tqi : get_tu(px, py, ch);   // one TU: both sides
      const vvcr_tu &tq = d.tu[tqi], &tp = d.tu[tpi];
      if (tq.b[0][BCBF] || tp.b[0][BCBF]) tmp += bs_set(1, 0);
      if (tq.b[1][BCBF] || tp.b[1][BCBF] || tq.jccr || tp.jccr) tmp += bs_set(1, 1);
      if (tq.b[2][BCBF] || tp.b[2][BCBF] || tq.jccr || tp.jccr) tmp += bs_set(1, 2);
    }
    if ((tmp & 3) == 1) return tmp;
    if (ciip) return 1;
    if (!cuQ.yvalid) return tmp;
    if (marker != 0 && marker != 3) return tmp;
    return motion_bs(dir, lx, ly, tmp);
  }

  // the motion part of xGetBoundaryStrengthSingle (LoopFilter.cpp:748-812) for luma position (lx, ly) of an
  // inter Q block and its P neighbour, on top of the transform part tmp
  int motion_bs(int dir, int lx, int ly, int tmp) const {
    const int lpx = dir == VER ? lx - 1 : lx, lpy = dir == VER ? ly : ly - 1;
    return motion_bs_pair(d.motion[(size_t)(lpy >> 2) * W4 + (lpx >> 2)], d.motion[(size_t)(ly >> 2) * W4 + (lx >> 2)], tmp);
  }
  int motion_bs_pair(const MotionRec &mp, const MotionRec &mq, int tmp) const {
    const int th = 8;
    // the same motion on both sides (one PU, or equal neighbours): no motion boundary
    if (*(const uint16_t *)&mp.ref0 == *(const uint16_t *)&mq.ref0 && std::memcmp(&mp.mv0x, &mq.mv0x, 16) == 0 &&
        (mp.ref0 >= 0 || pp.slice_type == 0))
      return tmp;
    if (pp.slice_type == 0) {
      // Picture identity: entries of the lists with equal POC are the same decoded picture.
      const int NONE = INT32_MIN;
      const int rP0 = mp.ref0 >= 0 ? pp.ref_poc[0][mp.ref0] : NONE, rP1 = mp.ref1 >= 0 ? pp.ref_poc[1][mp.ref1] : NONE;
      const int rQ0 = mq.ref0 >= 0 ? pp.ref_poc[0][mq.ref0] : NONE, rQ1 = mq.ref1 >= 0 ? pp.ref_poc[1][mq.ref1] : NONE;
      const int p0x = mp.ref0 >= 0 ? mp.mv0x : 0, p0y = mp.ref0 >= 0 ? mp.mv0y : 0;
      const int p1x = mp.ref1 >= 0 ? mp.mv1x : 0, p1y = mp.ref1 >= 0 ? mp.mv1y : 0;
      const int q0x = mq.ref0 >= 0 ? mq.mv0x : 0, q0y = mq.ref0 >= 0 ? mq.mv0y : 0;
      const int q1x = mq.ref1 >= 0 ? mq.mv1x : 0, q1y = mq.ref1 >= 0 ? mq.mv1y : 0;
      int b;
      if ((rP0 == rQ0 && rP1 == rQ1) || (rP0 == rQ1 && rP1 == rQ0)) {
        const bool s00 = std::abs(q0x - p0x) >= th || std::abs(q0y - p0y) >= th || std::abs(q1x - p1x) >= th || std::abs(q1y - p1y) >= th;
        const bool s01 = std::abs(q1x - p0x) >= th || std::abs(q1y - p0y) >= th || std::abs(q0x - p1x) >= th || std::abs(q0y - p1y) >= th;
        b = rP0 != rP1 ? (rP0 == rQ0 ? s00 : s01) : (s00 && s01);
      } else {
        b = 1;
      }
      return b + tmp;
    }
    if (mp.ref0 < 0 || mq.ref0 < 0) throw VvcrError(VVCR_E_ARG, "deblocking: P-slice inter block without list-0 reference");
    if (pp.ref_poc[0][mp.ref0] != pp.ref_poc[0][mq.ref0]) return tmp + 1;
    return (std::abs(mq.mv0x - mp.mv0x) >= th || std::abs(mq.mv0y - mp.mv0y) >= th) ? tmp + 1 : tmp;
  }

  int chroma_qp_cached(int t, int comp) const { return M.cqp[2 * (size_t)t + comp - 1]; }
  // QpParam(tu, comp).Qp(0) - qpBdOffset (Quant.cpp:65-138); joint Cb-Cr mode 3 uses the JOINT_CbCr tables
  int chroma_qp(int t, int comp) const {
    const int qpy = d.cu[d.tu[t].cu].qp;
    const bool jqp = d.tu[t].jccr == 3;
    const int off = jqp ? pp.chroma_qp_off[0] : pp.chroma_qp_off[comp];
    const int32_t *map = pp.chroma_qp_map[jqp ? 0 : comp];
    const int qbd = 6 * (sp.bit_depth - 8);
    int q = map[std::clamp(qpy, -qbd, 63) + 64];
    q = std::clamp(q + off, -qbd, 63) + qbd;
    q = std::clamp(q, 0, 63 + qbd);
    return q - qbd;
  }

  // an edge on a virtual boundary is not filtered (xDeriveEdgefilterParam, LoopFilter.cpp:433-452: every TU,
  // PU and sub-block edge of a CU the boundary crosses whose line is the boundary)
  bool on_vb(int dir, int px, int py) const {
    if (!pp.vb_disabled) return false;
    if (dir == VER) {
      for (int i = 0; i < pp.num_vb_ver && i < 3; i++) if (px == pp.vb_ver[i]) return true;
    } else {
      for (int i = 0; i < pp.num_vb_hor && i < 3; i++) if (py == pp.vb_hor[i]) return true;
    }
    return false;
  }

  void emit_luma(int cui, int dir, int e) {
    const vvcr_cu &cu = d.cu[cui];
    const int n = dir == VER ? cu.h / 4 : cu.w / 4;
    for (int i = 0; i < n; i++) {
      const int px = dir == VER ? cu.x + e * 4 : cu.x + i * 4;
      const int py = dir == VER ? cu.y + i * 4 : cu.y + e * 4;
      if (on_vb(dir, px, py)) continue;
      const int b = bs[dir][raster(px, py)] & 3;
      if (!b) continue;
      const vvcr_cu &cuP = d.cu[get_cu(dir == VER ? px - 1 : px, dir == VER ? py : py - 1, cu.chtype)];
      const int qp = (cuP.qp + cu.qp + 1) >> 1;
      int lp = lenP[0][(px - ctu_x) >> 2][(py - ctu_y) >> 2], lq = lenQ[0][(px - ctu_x) >> 2][(py - ctu_y) >> 2];
      bool pl = false, ql = false;
      if (lp > 3) {
        pl = true;
        if (lp > 5 && cuP.affine) lp = 5;
      }
      if (lq > 3) ql = true;
      if (dir == HOR && py % ctu == 0) pl = false;
      DbkSeg s;
      s.x4 = (uint16_t)(px >> 2);
      s.y4 = (uint16_t)(py >> 2);
      s.w = (uint32_t)b | (uint32_t)lp << 2 | (uint32_t)lq << 5 | (uint32_t)(qp & 63) << 8 | (uint32_t)pl << 14 | (uint32_t)ql << 15;
      out.luma[dir].push_back(s);
    }
  }

  void emit_chroma(int cui, int dir, int e) {
    const vvcr_cu &cu = d.cu[cui];
    int a[4];
    cu_area(cu, a);
    const int r = raster(a[0], a[1]);
    if ((dir == VER && (r % parts + e) % 4) || (dir == HOR && (r / parts + e) % 4)) return;
    const int n = dir == VER ? a[3] / 4 : a[2] / 4;
    for (int i = 0; i < n; i++) {
      const int px = dir == VER ? a[0] + e * 4 : a[0] + i * 4;
      const int py = dir == VER ? a[1] + i * 4 : a[1] + e * 4;
      if (on_vb(dir, px, py)) continue;
      const int v = bs[dir][raster(px, py)];
      const int bS[2] = {(v >> 2) & 3, (v >> 4) & 3};
      if (!bS[0] && !bS[1]) continue;
      const int nlx = dir == VER ? px - 4 : px, nly = dir == VER ? py : py - 4;
      int cpi = cu.chtype ? get_cu(nlx >> 1, nly >> 1, 1) : get_cu(nlx, nly, 0);
      if (d.cu[cpi].treetype != 0 || pp.dual_tree) cpi = get_cu(nlx >> 1, nly >> 1, 1);
      const vvcr_cu &cuP = d.cu[cpi];
      const int cx = (px - ctu_x) >> 2, cy = (py - ctu_y) >> 2;   // 2x2 chroma units
      const bool large = lenP[1][cx][cy] >= 3 && lenQ[1][cx][cy] >= 3;
      const bool ctbh = dir == HOR && py % ctu == 0;
      uint32_t w = (uint32_t)large << 4 | (uint32_t)ctbh << 19;
      bool any = false;
      for (int k = 0; k < 2; k++) {
        if (!(bS[k] == 2 || (large && bS[k] == 1))) continue;
        const int comp = k + 1;
        const int shP = cuP.yvalid ? 0 : 1, shQ = cu.yvalid ? 0 : 1;
        const int tq = get_tu(px >> shQ, py >> shQ, cu.chtype);
        const int p1x = px >> shP, p1y = py >> shP;
        const int tp = get_tu(dir == VER ? p1x - 1 : p1x, dir == VER ? p1y : p1y - 1, cuP.chtype);
        const int qp = (chroma_qp_cached(tq, comp) + chroma_qp_cached(tp, comp) + 1) >> 1;
        w |= (uint32_t)bS[k] << (2 * k) | (uint32_t)((qp + 64) & 127) << (5 + 7 * k);
        any = true;
      }
      if (!any) continue;
      DbkSeg s;
      s.x4 = (uint16_t)(px >> 2);
      s.y4 = (uint16_t)(py >> 2);
      s.w = w;
      out.chroma[dir].push_back(s);
    }
  }

  bool lf_edge_ok(const vvcr_cu &cu, bool leftEdge) const {
    if (lf_nb.empty()) return true;
    const int x = cu.yvalid ? cu.x : 2 * cu.cx, y = cu.yvalid ? cu.y : 2 * cu.cy;
    if (leftEdge ? (x & (ctu - 1)) : (y & (ctu - 1))) return true;
    const int wc = (sp.width + ctu - 1) / ctu;
    return lf_nb[(size_t)(y >> sp.ctu_log2) * wc + (x >> sp.ctu_log2)] & (leftEdge ? LFNB_L : LFNB_A);
  }

  void deblock_cu(int cui, int dir) {
    const vvcr_cu &cu = d.cu[cui];
    int a[4];
    cu_area(cu, a);
    const int ch = cu.chtype;
    const int cpx = ch ? cu.cx : cu.x, cpy = ch ? cu.cy : cu.y;
    if (pp.dbk_disable) { left = top = internal = false; }
    else {
      // xSetLoopfilterParam (LoopFilter.cpp:656-672): the left / top neighbour must be available across tiles /
      // slices not filtered across (isAvailableLeft / Above); only at a CTB edge can it lie in another tile / slice
      internal = true;
      left = cpx > 0 && lf_edge_ok(cu, true);
      top = cpy > 0 && lf_edge_ok(cu, false);
    }
    int edges[2 * 128 + 16], ne = 0;
    for (int t = cu.firsttu; t < cu.firsttu + cu.ntu; t++) {
      int ta[4];
      if (cu.yvalid) { const int32_t *b = d.tu[t].b[0]; ta[0] = b[BX]; ta[1] = b[BY]; ta[2] = b[BW]; ta[3] = b[BH]; }
      else std::memcpy(ta, a, sizeof ta);
      set_edges(dir, ta[0], ta[1], ta[2], ta[3], internal, false);   // the other direction's pass sets its own
      len_from_tu(dir, cu, t);
      const int32_t *tb = d.tu[t].b[ch];
      edges[ne++] = dir == HOR ? (tb[BY] - cpy) / 4 : (tb[BX] - cpx) / 4;
    }
    for (int pi = cu.firstpu; pi < cu.firstpu + cu.npu; pi++) {
      const vvcr_pu &pu = d.pu[pi];
      int pa[4];
      if (cu.yvalid) { pa[0] = pu.x; pa[1] = pu.y; pa[2] = pu.w; pa[3] = pu.h; }
      else std::memcpy(pa, a, sizeof pa);
      const int pux = ch ? pu.cx : pu.x, puy = ch ? pu.cy : pu.y;
      const bool xoff = pux != cpx, yoff = puy != cpy;
      if (dir == VER) set_edges(VER, pa[0], pa[1], pa[2], pa[3], xoff ? internal : left, xoff);
      else set_edges(HOR, pa[0], pa[1], pa[2], pa[3], yoff ? internal : top, yoff);
      edges[ne++] = dir == HOR ? (puy - cpy) / 4 : (pux - cpx) / 4;
      if ((pu.merge && pu.mrgtype == MRG_TYPE_SUBPU_ATMVP) || cu.affine) {
        if (dir == HOR) {
          for (int off = 8; off < pa[3]; off += 8) {
            set_edges(HOR, cu.x, cu.y + off, cu.w, 4, internal, true);
            edges[ne++] = (puy + off - cpy) / 4;
          }
        } else {
          for (int off = 8; off < pa[2]; off += 8) {
            set_edges(VER, cu.x + off, cu.y, 4, cu.h, internal, true);
            edges[ne++] = (pux + off - cpx) / 4;
          }
        }
        if (pu.w > 0) len_subblocks(dir, pu, pa[2], pa[3]);
      }
    }
    // An edge inside an inter, non-CIIP luma CU that is not a transform edge (sub-block edges of affine /
    // SbTMVP CUs: most of the edges of a B picture) has only the motion part of the boundary strength.
    const bool fast = cu.yvalid && cu.predmode != MODE_INTRA && !d.pu[cu.firstpu].ciip;
    std::sort(edges, edges + ne);
    auto bs_at = [&](int x, int y) {
      const int r = raster(a[0] + x, a[1] + y);
      if (!edge[dir][r]) return;
      if (fast && bs[dir][r] == 0 && (dir == VER ? x : y) > 0) bs[dir][r] = (uint8_t)motion_bs(dir, a[0] + x, a[1] + y, 0);
      else bs[dir][r] = (uint8_t)boundary_strength(cui, dir, a[0] + x, a[1] + y);
    };
    if (cu.yvalid) {   // edge flags are only ever set on the edge lines listed: visit those, not the whole CU
      const bool ver = dir == VER;
      const int rstep = ver ? parts : 1, n = (ver ? a[3] : a[2]) / 4;
      const ptrdiff_t qstep = ver ? W4 : 1, pofs = ver ? -1 : -(ptrdiff_t)W4;
      if (fast && ver) {   // interior vertical lines row by row: the motion records of a row are adjacent
        int lines[64], nl = 0;
        for (int k = 0; k < ne; k++)
          if ((!k || edges[k] != edges[k - 1]) && edges[k] > 0 && edges[k] * 4 < a[2]) lines[nl++] = edges[k];
        const MotionRec *row = d.motion.data() + (size_t)(a[1] >> 2) * W4 + (a[0] >> 2);
        int r0 = raster(a[0], a[1]);
        for (int i = 0; i < n; i++, row += W4, r0 += parts)
          for (int t = 0; t < nl; t++) {
            const int u = lines[t], r = r0 + u;
            if (!edge[dir][r]) continue;
            if (bs[dir][r] == 0) bs[dir][r] = (uint8_t)motion_bs_pair(row[u - 1], row[u], 0);
            else bs[dir][r] = (uint8_t)boundary_strength(cui, dir, a[0] + 4 * u, a[1] + 4 * i);
          }
      }
      for (int k = 0; k < ne; k++) {
        if (k && edges[k] == edges[k - 1]) continue;
        const int o = edges[k] * 4;
        if (o < 0 || o >= (ver ? a[2] : a[3])) continue;
        if (fast && o > 0 && ver) continue;   // done above
        if (fast && o > 0) {   // interior line of an inter CU: the motion part unless a transform edge marks it
          const int x0 = ver ? a[0] + o : a[0], y0 = ver ? a[1] : a[1] + o;
          const MotionRec *mq = d.motion.data() + (size_t)(y0 >> 2) * W4 + (x0 >> 2);
          int r = raster(x0, y0);
          for (int i = 0; i < n; i++, r += rstep, mq += qstep) {
            if (!edge[dir][r]) continue;
            if (bs[dir][r] == 0) bs[dir][r] = (uint8_t)motion_bs_pair(mq[pofs], *mq, 0);
            else bs[dir][r] = (uint8_t)boundary_strength(cui, dir, ver ? x0 : x0 + 4 * i, ver ? y0 + 4 * i : y0);
          }
        } else if (ver) {
          for (int y = 0; y < a[3]; y += 4) bs_at(o, y);
        } else {
          for (int x = 0; x < a[2]; x += 4) bs_at(x, o);
        }
      }
    } else {
      for (int y = 0; y < a[3]; y += 4)
        for (int x = 0; x < a[2]; x += 4) bs_at(x, y);
    }
    int prev = -1;
    for (int k = 0; k < ne; k++) {
      if (edges[k] == prev) continue;
      prev = edges[k];
      if (cu.yvalid) emit_luma(cui, dir, edges[k]);
      if (cu.cvalid && (!cu.isp || edges[k] == 0)) emit_chroma(cui, dir, edges[k]);
    }
  }

  void reset(int dir) {
    std::memset(bs[dir], 0, sizeof bs[dir]);
    std::memset(edge[dir], 0, sizeof edge[dir]);
    std::memset(lenP, 0, sizeof lenP);
    std::memset(lenQ, 0, sizeof lenQ);
    std::memset(tedge, 0, sizeof tedge);
  }

  // CUs grouped by CTU (raster order): start[k] .. start[k + 1] index order[] for CTU k
  void group(std::vector<int> &start, std::vector<int> &order) const {
    const int wc = (sp.width + ctu - 1) / ctu, hc = (sp.height + ctu - 1) / ctu;
    const int ncu = (int)d.cu.size();
    start.assign((size_t)wc * hc + 1, 0);
    order.resize(ncu);
    std::vector<int> ctu_of(ncu);
    for (int i = 0; i < ncu; i++) {
      int a[4];
      cu_area(d.cu[i], a);
      ctu_of[i] = (a[1] >> sp.ctu_log2) * wc + (a[0] >> sp.ctu_log2);
      start[ctu_of[i] + 1]++;
    }
    for (int k = 0; k < wc * hc; k++) start[k + 1] += start[k];
    std::vector<int> pos(start.begin(), start.end() - 1);
    for (int i = 0; i < ncu; i++) order[pos[ctu_of[i]]++] = i;
  }

  // the edges of CTUs [k0, k1) in one direction (every CTU's state is its own: LoopFilter::xDeblockCU
  // works CTU by CTU)
  void run_ctus(int dir, int k0, int k1, const std::vector<int> &start, const std::vector<int> &order) {
    const int wc = (sp.width + ctu - 1) / ctu;
    // a shard plans the edges of the CUs within VVCR_LF_HALO rows of its own rows: its loop filters
    // rebuild the deblocked samples the SAO / ALF of its rows read (see vvcr.h)
    const bool shard = pp.shard_y1 > 0;
    const int ly0 = pp.shard_y0 - VVCR_LF_HALO, ly1 = pp.shard_y1 + VVCR_LF_HALO;
    for (int k = k0; k < k1; k++) {
      ctu_x = (k % wc) * ctu;
      ctu_y = (k / wc) * ctu;
      if (shard && (ctu_y + ctu <= ly0 || ctu_y >= ly1)) continue;
      for (int pass = 0; pass < (pp.dual_tree ? 2 : 1); pass++) {
        reset(dir);
        for (int j = start[k]; j < start[k + 1]; j++) {
          const int i = order[j];
          if (pp.dual_tree && d.cu[i].chtype != pass) continue;
          if (shard && !cu_in_rows(d.cu[i], ly0, ly1)) continue;
          deblock_cu(i, dir);
        }
      }
    }
  }
};

}  // namespace

// Workers take contiguous CTU ranges and fill lists of their own, appended in CTU order afterwards: the
// lists are those of one pass over the CTUs, whatever the number of workers (VVCR_DBK_THREADS, default 4;
// the picture's other planners run beside them).
void plan_deblocking(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, const std::vector<uint8_t> &lf_nb,
                     DbkLists &out) {
  out.clear();
  if (pp.dbk_disable) return;
  if (sp.width % 8 || sp.height % 8) throw VvcrError(VVCR_E_UNSUPPORTED, "deblocking: picture size not a multiple of 8");
  static const int nthreads = [] {
    const char *e = getenv("VVCR_DBK_THREADS");
    return e ? std::max(1, std::min(32, atoi(e))) : 4;
  }();
  Maps M;
  std::vector<int> start, order;
  {
    DbkLists scratch;
    auto P = std::make_unique<Planner>(sp, pp, d, scratch, M, lf_nb);   // ~200 KB of per-CTU state: keep it off the stack
    P->build_maps();
    P->group(start, order);
  }
  const int nctu = (int)start.size() - 1;
  const int T = std::max(1, std::min(nthreads, nctu / 8));
  std::vector<DbkLists> part(T);
  std::vector<std::exception_ptr> err(T);
  auto work = [&](int t) {
    try {
      auto P = std::make_unique<Planner>(sp, pp, d, part[t], M, lf_nb);
      const int k0 = (int)((int64_t)nctu * t / T), k1 = (int)((int64_t)nctu * (t + 1) / T);
      for (int dir = 0; dir < 2; dir++) P->run_ctus(dir, k0, k1, start, order);
    } catch (...) {
      err[t] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  for (auto &e : err)
    if (e) std::rethrow_exception(e);
  for (int dir = 0; dir < 2; dir++)
    for (int t = 0; t < T; t++) {
      out.luma[dir].insert(out.luma[dir].end(), part[t].luma[dir].begin(), part[t].luma[dir].end());
      out.chroma[dir].insert(out.chroma[dir].end(), part[t].chroma[dir].begin(), part[t].chroma[dir].end());
    }
}

// Compact copies of the descriptors for the device planner (vvcr_dbk_plan.hip): one pass over the CU / PU /
// TU rows, with the chroma QP of every TU resolved here (the host planner's chroma_qp).
void pack_dbk_inputs(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, const std::vector<uint8_t> &lf_nb,
                     DbkGpuInputs &out) {
  out.clear();
  if (pp.dbk_disable) return;
  if (sp.width % 8 || sp.height % 8) throw VvcrError(VVCR_E_UNSUPPORTED, "deblocking: picture size not a multiple of 8");
  const size_t ncu = d.cu.size(), npu = d.pu.size(), ntu = d.tu.size();
  if (ncu > (size_t)DBKP_IDX_MASK || ntu > (size_t)DBKP_IDX_MASK) throw VvcrError(VVCR_E_ARG, "deblocking: too many coding units");
  out.cu.resize(ncu);
  out.pu.resize(npu);
  out.tu.resize(ntu);
  for (size_t i = 0; i < ncu; i++) {
    const vvcr_cu &c = d.cu[i];
    DbCu &o = out.cu[i];
    o.x = (int16_t)c.x; o.y = (int16_t)c.y; o.w = (int16_t)c.w; o.h = (int16_t)c.h;
    o.cx = (int16_t)c.cx; o.cy = (int16_t)c.cy; o.cw = (int16_t)c.cw; o.ch = (int16_t)c.ch;
    o.firstpu = c.firstpu; o.firsttu = c.firsttu; o.npu = (int16_t)c.npu; o.ntu = (int16_t)c.ntu;
    o.qp = (int16_t)c.qp;
    uint16_t f = 0;
    if (c.chtype) f |= DBC_CHTYPE;
    if (c.predmode == MODE_INTRA) f |= DBC_INTRA;
    if (c.bdpcm) f |= DBC_BDPCM;
    if (c.bdpcmc) f |= DBC_BDPCMC;
    if (c.affine) f |= DBC_AFFINE;
    if (c.isp) f |= DBC_ISP;
    if (c.treetype != 0) f |= DBC_TREE;
    if (c.yvalid) f |= DBC_YVALID;
    if (c.cvalid) f |= DBC_CVALID;
    if (c.firstpu >= 0 && (size_t)c.firstpu < npu && d.pu[c.firstpu].ciip) f |= DBC_CIIP;
    if (!lf_nb.empty()) {   // tile / slice edges not filtered across (the host planner's lf_edge_ok)
      const int ctu = 1 << sp.ctu_log2, wc = (sp.width + ctu - 1) / ctu;
      const int lx = c.yvalid ? c.x : 2 * c.cx, ly = c.yvalid ? c.y : 2 * c.cy;
      const uint8_t m = lf_nb[(size_t)(ly >> sp.ctu_log2) * wc + (lx >> sp.ctu_log2)];
      if ((lx & (ctu - 1)) == 0 && !(m & LFNB_L)) f |= DBC_NOLEFT;
      if ((ly & (ctu - 1)) == 0 && !(m & LFNB_A)) f |= DBC_NOTOP;
    }
    o.flags = f;
    if (c.chtype) out.chroma_pass = true;
    // the edge lines (the host planner's deblock_cu edge list, as a mask) and the CU's units on them: its
    // runs in the item lists of its pass (vvcr_dbk_plan.hip k_dbkp_maps writes them there)
    const int ch = c.chtype, cpx = ch ? c.cx : c.x, cpy = ch ? c.cy : c.y;
    const int a2 = c.yvalid ? c.w : 2 * c.cw, a3 = c.yvalid ? c.h : 2 * c.ch;
    uint64_t m[2] = {0, 0};
    auto add = [&](int dir, int v) { if (v >= 0 && v < 64) m[dir] |= 1ull << v; };
    for (int t = c.firsttu; t < c.firsttu + c.ntu; t++) {
      const int32_t *tb = d.tu[t].b[ch];
      add(0, (tb[BX] - cpx) / 4);
      add(1, (tb[BY] - cpy) / 4);
    }
    if (c.npu > 0) {
      const vvcr_pu &u = d.pu[c.firstpu];
      const int pux = ch ? u.cx : u.x, puy = ch ? u.cy : u.y;
      add(0, (pux - cpx) / 4);
      add(1, (puy - cpy) / 4);
      if ((u.merge && u.mrgtype == MRG_TYPE_SUBPU_ATMVP) || c.affine) {
        const int pw = c.yvalid ? u.w : a2, ph = c.yvalid ? u.h : a3;
        for (int off = 8; off < pw; off += 8) add(0, (pux + off - cpx) / 4);
        for (int off = 8; off < ph; off += 8) add(1, (puy + off - cpy) / 4);
      }
    }
    const int wq = a2 / 4, hq = a3 / 4;
    m[0] &= wq >= 64 ? ~0ull : (1ull << wq) - 1;   // lines inside the CU
    m[1] &= hq >= 64 ? ~0ull : (1ull << hq) - 1;
    for (int dir = 0; dir < 2; dir++) {
      o.lines[dir] = (uint32_t)m[dir];
      if (m[dir] >> 32) throw VvcrError(VVCR_E_ARG, "deblocking: CU wider than 128 samples");
      o.item0[dir] = out.nitems[2 * ch + dir];
      out.nitems[2 * ch + dir] += __builtin_popcountll(m[dir]) * (dir == 0 ? hq : wq);
    }
  }
  for (size_t i = 0; i < npu; i++) {
    const vvcr_pu &u = d.pu[i];
    DbPu &o = out.pu[i];
    o.x = (int16_t)u.x; o.y = (int16_t)u.y; o.w = (int16_t)u.w; o.h = (int16_t)u.h; o.cx = (int16_t)u.cx; o.cy = (int16_t)u.cy;
    o.sub = (u.merge && u.mrgtype == MRG_TYPE_SUBPU_ATMVP) ? 1 : 0;
    o.pad = 0;
  }
  const int qbd = 6 * (sp.bit_depth - 8);
  for (size_t t = 0; t < ntu; t++) {
    const vvcr_tu &u = d.tu[t];
    DbTu &o = out.tu[t];
    for (int c = 0; c < 3; c++)
      for (int k = 0; k < 4; k++) o.b[c][k] = (int16_t)u.b[c][k];
    o.cu = u.cu;
    o.cbf = (uint8_t)((u.b[0][BCBF] ? 1 : 0) | (u.b[1][BCBF] ? 2 : 0) | (u.b[2][BCBF] ? 4 : 0));
    o.jccr = (uint8_t)u.jccr;
    // QpParam(tu, comp).Qp(0) - qpBdOffset (Quant.cpp:65-138), as Planner::chroma_qp
    const int qpy = d.cu[u.cu].qp;
    for (int comp = 1; comp <= 2; comp++) {
      const bool jqp = u.jccr == 3;
      const int off = jqp ? pp.chroma_qp_off[0] : pp.chroma_qp_off[comp];
      const int32_t *map = pp.chroma_qp_map[jqp ? 0 : comp];
      int q = map[std::clamp(qpy, -qbd, 63) + 64];
      q = std::clamp(q + off, -qbd, 63) + qbd;
      q = std::clamp(q, 0, 63 + qbd);
      o.cqp[comp - 1] = (int8_t)(q - qbd);
    }
  }
}
