// vvcr_dbk_plan.hip — deblocking edge planning on the device (SURVEY.md K12 "metadata kernel"; r05): the
// control part of LoopFilter::xDeblockCU (LoopFilter.cpp:261-408) that vvcr_dbk_host.cpp runs on the
// host — edge flags and TU / PU / sub-block markers (xSetEdgefilterMultiple :627), filter lengths from
// transform sizes (:454) and of SbTMVP / affine sub-blocks (:550), xGetBoundaryStrengthSingle (:674), and
// the QP / length bookkeeping of xEdgeFilterLuma (:844-979) and xEdgeFilterChroma (:1087-1244) — as one
// thread per (CU, direction). It is the same algorithm as the host planner (every rule cited there), over
// picture-wide maps instead of the reference's per-CTU arrays: a CU writes and reads only the edge
// positions of its own area (its left / top boundary and its internal edges), so the CUs of a picture
// plan independently. Kernels, per picture, on the picture's lane before the deblocking filter:
//   k_dbkp_maps     CU index maps (luma 4x4 / chroma 2x2 units) and TU index maps, one thread per CU / TU
//   k_dbkp_cu<dir>  the edges of one CU in one direction, the segment words into dense maps
//   k_dbkp_compact  the dense words of both directions into the four segment lists k_dbk reads, with
//                   their lengths on the device (order: by workgroup reservation; every segment of one
//                   direction is independent, so the lists' order does not change the filtered samples)
// Inputs: compact CU / PU / TU records (DbCu / DbPu / DbTu, vvcr_dbk.h, built by pack_dbk_inputs) and the
// 4x4 motion field (MotionRec) of the picture, uploaded with its work lists.
#include "vvcr_dbk.h"

namespace {

enum { VER = 0, HOR = 1 };

__device__ __forceinline__ int cdiv(int a, int s) { return (a + (1 << s) - 1) >> s; }

struct Planner {
  const DbkPlanArgs &A;
  __device__ explicit Planner(const DbkPlanArgs &a) : A(a) {}

  __device__ int pos(int x, int y) const { return (y >> 2) * A.W4 + (x >> 2); }   // luma 4x4 unit
  __device__ int get_cu(int x, int y, int ch) const {
    const int s = ch ? 1 : 2;
    const int i = A.cu_map[ch][(y >> s) * A.W4 + (x >> s)];
    if (i < 0) { atomicOr(A.err, 2); return 0; }   // "deblocking: no CU covers a neighbouring position"
    return i;
  }
  __device__ int get_tu(int x, int y, int ch) const {
    const int s = ch ? 1 : 2;
    int t = A.tu_map[ch][(y >> s) * A.W4 + (x >> s)];
    if (t == -1) { atomicOr(A.err, 2); return 0; }
    if (t >= 0) return t;
    t = -t - 2;   // an ISP CU's area: CodingStructure::getTU (CodingStructure.cpp:379) searches its sub-partitions
    for (int k = 0; k < 4 && t + k < A.ntu; k++) {
      const int16_t *b = A.tu[t + k].b[0];
      if (x >= b[0] && x < b[0] + b[2] && y >= b[1] && y < b[1] + b[3]) return t + k;
    }
    return t;
  }
  __device__ static void cu_area(const DbCu &c, int *a) {
    if (c.flags & DBC_YVALID) { a[0] = c.x; a[1] = c.y; a[2] = c.w; a[3] = c.h; }
    else { a[0] = c.cx * 2; a[1] = c.cy * 2; a[2] = c.cw * 2; a[3] = c.ch * 2; }
  }

  // xSetEdgefilterMultiple (:627)
  __device__ void set_edges(int dir, int x, int y, int w, int h, bool val, bool edgeIdx) const {
    const int add = dir == VER ? A.W4 : 1, n = dir == VER ? h / 4 : w / 4;
    int idx = pos(x, y);
    uint8_t *bs = A.bs[dir], *edge = A.edge[dir];
    for (int i = 0; i < n; i++, idx += add) {
      edge[idx] = val;
      if (bs[idx] && val) bs[idx] = 3;
      else if (!edgeIdx) bs[idx] = val;
    }
  }

  // filter lengths from the transform sizes on both sides (:454)
  __device__ void len_from_tu(int dir, const DbCu &cu, int t, bool left, bool top, bool internal) const {
    const DbTu &tu = A.tu[t];
    for (int comp = 0; comp < 3; comp++) {
      const int ch = comp ? 1 : 0;
      const int16_t *b = tu.b[comp], *bch = tu.b[ch];
      if (b[2] <= 0 || b[3] <= 0) continue;
      const int cux = comp ? cu.cx : cu.x, cuy = comp ? cu.cy : cu.y;
      const int step = 4 >> ch;
      const bool horz = dir == HOR;
      if (!(horz ? (b[1] == cuy ? top : internal) : (b[0] == cux ? left : internal))) continue;
      const int n = horz ? b[2] : b[3];
      for (int k = 0; k < n; k += step) {
        const int qx = horz ? bch[0] + k : bch[0], qy = horz ? bch[1] : bch[1] + k;
        const int sizeQ = horz ? b[3] : b[2];
        const int tp = horz ? get_tu(qx, qy - 1, ch) : get_tu(qx - 1, qy, ch);
        const int sizeP = horz ? A.tu[tp].b[comp][3] : A.tu[tp].b[comp][2];
        const int X = horz ? b[0] + k : b[0], Y = horz ? b[1] : b[1] + k;   // component samples
        const int g = ch ? 1 : 2;
        if ((X | Y) & ((1 << g) - 1)) continue;
        const int p = (Y >> g) * A.W4 + (X >> g);   // the 4x4 luma / 2x2 chroma unit: one grid
        if (comp == 0) {
          A.tedge[dir][p] = 1;
          const bool small = sizeP <= 4 || sizeQ <= 4;
          A.lenQ[dir][0][p] = small ? 1 : (sizeQ >= 32 ? 7 : 3);
          A.lenP[dir][0][p] = small ? 1 : (sizeP >= 32 ? 7 : 3);
        } else {
          A.lenQ[dir][comp][p] = A.lenP[dir][comp][p] = (sizeQ >= 8 && sizeP >= 8) ? 3 : 1;
        }
      }
    }
  }

  // sub-block edge lengths of SbTMVP / affine PUs (:550)
  __device__ void len_subblocks(int dir, const DbPu &pu, int w, int h) const {
    uint8_t *Q = A.lenQ[dir][0], *Pp = A.lenP[dir][0];
    const uint8_t *te = A.tedge[dir];
    const bool horz = dir == HOR;
    const int outer = horz ? h : w, inner = horz ? w : h;
    for (int a = 0; a < outer; a += 8)
      for (int b = 0; b < inner; b += 4) {
        const int x = horz ? pu.x + b : pu.x + a, y = horz ? pu.y + a : pu.y + b;
        const int p = pos(x, y);
        auto T = [&](int delta) { return horz ? te[pos(x, y + delta)] : te[pos(x + delta, y)]; };
        if (T(0)) {
          if (Q[p] > 5) Q[p] = 5;
          if (a > 0 && Pp[p] > 5) Pp[p] = 5;
        } else if (a > 0 && (T(-4) || a + 4 >= outer || T(4))) {
          Q[p] = Pp[p] = 1;
        } else if (a > 0 && (T(-8) || a + 8 >= outer || T(8))) {
          Q[p] = Pp[p] = 2;
        } else {
          Q[p] = Pp[p] = 3;
        }
      }
  }

  __device__ static int bs_set(int v, int comp) { return v << (comp * 2); }

  // the motion part of xGetBoundaryStrengthSingle (:748-812)
  __device__ int motion_bs_pair(const MotionRec &mp, const MotionRec &mq, int tmp) const {
    const int th = 8;
    // the same motion on both sides (one PU, or equal neighbours): no motion boundary
    if (mp.ref0 == mq.ref0 && mp.ref1 == mq.ref1 && mp.mv0x == mq.mv0x && mp.mv0y == mq.mv0y && mp.mv1x == mq.mv1x &&
        mp.mv1y == mq.mv1y && (mp.ref0 >= 0 || A.slice_type == 0))
      return tmp;
    if (A.slice_type == 0) {
      const int NONE = INT32_MIN;
      const int rP0 = mp.ref0 >= 0 ? A.ref_poc[0][mp.ref0] : NONE, rP1 = mp.ref1 >= 0 ? A.ref_poc[1][mp.ref1] : NONE;
      const int rQ0 = mq.ref0 >= 0 ? A.ref_poc[0][mq.ref0] : NONE, rQ1 = mq.ref1 >= 0 ? A.ref_poc[1][mq.ref1] : NONE;
      const int p0x = mp.ref0 >= 0 ? mp.mv0x : 0, p0y = mp.ref0 >= 0 ? mp.mv0y : 0;
      const int p1x = mp.ref1 >= 0 ? mp.mv1x : 0, p1y = mp.ref1 >= 0 ? mp.mv1y : 0;
      const int q0x = mq.ref0 >= 0 ? mq.mv0x : 0, q0y = mq.ref0 >= 0 ? mq.mv0y : 0;
      const int q1x = mq.ref1 >= 0 ? mq.mv1x : 0, q1y = mq.ref1 >= 0 ? mq.mv1y : 0;
      int b;
      if ((rP0 == rQ0 && rP1 == rQ1) || (rP0 == rQ1 && rP1 == rQ0)) {
        const bool s00 = abs(q0x - p0x) >= th || abs(q0y - p0y) >= th || abs(q1x - p1x) >= th || abs(q1y - p1y) >= th;
        const bool s01 = abs(q1x - p0x) >= th || abs(q1y - p0y) >= th || abs(q0x - p1x) >= th || abs(q0y - p1y) >= th;
        b = rP0 != rP1 ? (rP0 == rQ0 ? s00 : s01) : (s00 && s01);
      } else {
        b = 1;
      }
      return b + tmp;
    }
    if (mp.ref0 < 0 || mq.ref0 < 0) { atomicOr(A.err, 2); return tmp; }   // P-slice inter block without list 0
    if (A.ref_poc[0][mp.ref0] != A.ref_poc[0][mq.ref0]) return tmp + 1;
    return (abs(mq.mv0x - mp.mv0x) >= th || abs(mq.mv0y - mp.mv0y) >= th) ? tmp + 1 : tmp;
  }
  __device__ int motion_bs(int dir, int lx, int ly, int tmp) const {
    const int lpx = dir == VER ? lx - 1 : lx, lpy = dir == VER ? ly : ly - 1;
    return motion_bs_pair(A.motion[(lpy >> 2) * A.W4 + (lpx >> 2)], A.motion[(ly >> 2) * A.W4 + (lx >> 2)], tmp);
  }

  // xGetBoundaryStrengthSingle (:674)
  __device__ int boundary_strength(int cui, int dir, int lx, int ly) const {
    const DbCu &cuQ = A.cu[cui];
    const int ch = cuQ.flags & DBC_CHTYPE ? 1 : 0;
    const bool yv = cuQ.flags & DBC_YVALID;
    const int sh = yv ? 0 : 1;
    const int qx = lx >> sh, qy = ly >> sh;
    const int px = dir == VER ? qx - 1 : qx, py = dir == VER ? qy : qy - 1;
    const bool same = px >= (yv ? cuQ.x : cuQ.cx) && py >= (yv ? cuQ.y : cuQ.cy);
    const DbCu &cuP = same ? cuQ : A.cu[get_cu(px, py, ch)];
    const bool iP = cuP.flags & DBC_INTRA, iQ = cuQ.flags & DBC_INTRA;
    if (iP || iQ) {
      const int bsY = (iP && (cuP.flags & DBC_BDPCM)) && (iQ && (cuQ.flags & DBC_BDPCM)) ? 0 : 2;
      const int bsC = (iP && (cuP.flags & DBC_BDPCMC)) && (iQ && (cuQ.flags & DBC_BDPCMC)) ? 0 : 2;
      return bs_set(bsY, 0) + bs_set(bsC, 1) + bs_set(bsC, 2);
    }
    const int marker = A.bs[dir][pos(lx, ly)];
    const bool ciip = (cuQ.flags & DBC_CIIP) || (!same && (cuP.flags & DBC_CIIP));
    if (marker && ciip) return bs_set(2, 0) + bs_set(2, 1) + bs_set(2, 2);
    int tmp = 0;
    if (marker) {
      const int tqi = get_tu(qx, qy, ch);
      const int tpi = (same && cuQ.ntu == 1 && !(cuQ.flags & DBC_ISP)) ? tqi : get_tu(px, py, ch);
      const DbTu &tq = A.tu[tqi], &tp = A.tu[tpi];
      if ((tq.cbf & 1) || (tp.cbf & 1)) tmp += bs_set(1, 0);
      if ((tq.cbf & 2) || (tp.cbf & 2) || tq.jccr || tp.jccr) tmp += bs_set(1, 1);
      if ((tq.cbf & 4) || (tp.cbf & 4) || tq.jccr || tp.jccr) tmp += bs_set(1, 2);
    }
    if ((tmp & 3) == 1) return tmp;
    if (ciip) return 1;
    if (!yv) return tmp;
    if (marker != 0 && marker != 3) return tmp;
    return motion_bs(dir, lx, ly, tmp);
  }

  __device__ void emit_luma(int cui, int dir, int e) const {
    const DbCu &cu = A.cu[cui];
    const int n = dir == VER ? cu.h / 4 : cu.w / 4;
    const int ctu = 1 << A.ctu_log2;
    const int ch = cu.flags & DBC_CHTYPE ? 1 : 0;
    for (int i = 0; i < n; i++) {
      const int px = dir == VER ? cu.x + e * 4 : cu.x + i * 4;
      const int py = dir == VER ? cu.y + i * 4 : cu.y + e * 4;
      const int p = pos(px, py);
      const int b = A.bs[dir][p] & 3;
      if (!b) continue;
      const DbCu &cuP = A.cu[get_cu(dir == VER ? px - 1 : px, dir == VER ? py : py - 1, ch)];
      const int qp = (cuP.qp + cu.qp + 1) >> 1;
      int lp = A.lenP[dir][0][p], lq = A.lenQ[dir][0][p];
      bool pl = false, ql = false;
      if (lp > 3) {
        pl = true;
        if (lp > 5 && (cuP.flags & DBC_AFFINE)) lp = 5;
      }
      if (lq > 3) ql = true;
      if (dir == HOR && py % ctu == 0) pl = false;
      A.segL[dir][p] = (uint32_t)b | (uint32_t)lp << 2 | (uint32_t)lq << 5 | (uint32_t)(qp & 63) << 8 | (uint32_t)pl << 14 | (uint32_t)ql << 15;
    }
  }

  __device__ void emit_chroma(int cui, int dir, int e) const {
    const DbCu &cu = A.cu[cui];
    int a[4];
    cu_area(cu, a);
    const int ctu = 1 << A.ctu_log2, parts = ctu / 4;
    const int r = ((a[0] & (ctu - 1)) >> 2) + ((a[1] & (ctu - 1)) >> 2) * parts;   // the CTU raster index of the host planner
    if ((dir == VER && (r % parts + e) % 4) || (dir == HOR && (r / parts + e) % 4)) return;
    const int n = dir == VER ? a[3] / 4 : a[2] / 4;
    const int chQ = cu.flags & DBC_CHTYPE ? 1 : 0;
    for (int i = 0; i < n; i++) {
      const int px = dir == VER ? a[0] + e * 4 : a[0] + i * 4;
      const int py = dir == VER ? a[1] + i * 4 : a[1] + e * 4;
      const int p = pos(px, py);
      const int v = A.bs[dir][p];
      const int bS[2] = {(v >> 2) & 3, (v >> 4) & 3};
      if (!bS[0] && !bS[1]) continue;
      const int nlx = dir == VER ? px - 4 : px, nly = dir == VER ? py : py - 4;
      int cpi = chQ ? get_cu(nlx >> 1, nly >> 1, 1) : get_cu(nlx, nly, 0);
      if ((A.cu[cpi].flags & DBC_TREE) || A.dual_tree) cpi = get_cu(nlx >> 1, nly >> 1, 1);
      const DbCu &cuP = A.cu[cpi];
      const bool large = A.lenP[dir][1][p] >= 3 && A.lenQ[dir][1][p] >= 3;
      const bool ctbh = dir == HOR && py % ctu == 0;
      uint32_t w = (uint32_t)large << 4 | (uint32_t)ctbh << 19;
      bool any = false;
      for (int k = 0; k < 2; k++) {
        if (!(bS[k] == 2 || (large && bS[k] == 1))) continue;
        const int comp = k + 1;
        const int shP = (cuP.flags & DBC_YVALID) ? 0 : 1, shQ = (cu.flags & DBC_YVALID) ? 0 : 1;
        const int tq = get_tu(px >> shQ, py >> shQ, chQ);
        const int p1x = px >> shP, p1y = py >> shP;
        const int tp = get_tu(dir == VER ? p1x - 1 : p1x, dir == VER ? p1y : p1y - 1, (cuP.flags & DBC_CHTYPE) ? 1 : 0);
        const int qp = (A.tu[tq].cqp[comp - 1] + A.tu[tp].cqp[comp - 1] + 1) >> 1;
        w |= (uint32_t)bS[k] << (2 * k) | (uint32_t)((qp + 64) & 127) << (5 + 7 * k);
        any = true;
      }
      if (any) A.segC[dir][p] = w;
    }
  }

  // LoopFilter::xDeblockCU for one CU and direction (the host planner's deblock_cu; edge lines of the CU as a
  // bit mask of 4-sample offsets instead of a sorted array)
  __device__ void deblock_cu(int cui, int dir) const {
    const DbCu &cu = A.cu[cui];
    int a[4];
    cu_area(cu, a);
    const bool yv = cu.flags & DBC_YVALID;
    const int ch = cu.flags & DBC_CHTYPE ? 1 : 0;
    const int cpx = ch ? cu.cx : cu.x, cpy = ch ? cu.cy : cu.y;
    bool left, top, internal;
    if (A.dbk_disable) { left = top = internal = false; }
    else { internal = true; left = cpx > 0; top = cpy > 0; }
    uint64_t lines = 0;
    auto add_line = [&](int v) { if (v >= 0 && v < 64) lines |= 1ull << v; };
    for (int t = cu.firsttu; t < cu.firsttu + cu.ntu; t++) {
      const DbTu &tu = A.tu[t];
      int ta[4];
      if (yv) { ta[0] = tu.b[0][0]; ta[1] = tu.b[0][1]; ta[2] = tu.b[0][2]; ta[3] = tu.b[0][3]; }
      else { ta[0] = a[0]; ta[1] = a[1]; ta[2] = a[2]; ta[3] = a[3]; }
      set_edges(dir, ta[0], ta[1], ta[2], ta[3], internal, false);
      len_from_tu(dir, cu, t, left, top, internal);
      const int16_t *tb = tu.b[ch];
      add_line(dir == HOR ? (tb[1] - cpy) / 4 : (tb[0] - cpx) / 4);
    }
    for (int pi = cu.firstpu; pi < cu.firstpu + cu.npu; pi++) {
      const DbPu &pu = A.pu[pi];
      int pa[4];
      if (yv) { pa[0] = pu.x; pa[1] = pu.y; pa[2] = pu.w; pa[3] = pu.h; }
      else { pa[0] = a[0]; pa[1] = a[1]; pa[2] = a[2]; pa[3] = a[3]; }
      const int pux = ch ? pu.cx : pu.x, puy = ch ? pu.cy : pu.y;
      const bool xoff = pux != cpx, yoff = puy != cpy;
      if (dir == VER) set_edges(VER, pa[0], pa[1], pa[2], pa[3], xoff ? internal : left, xoff);
      else set_edges(HOR, pa[0], pa[1], pa[2], pa[3], yoff ? internal : top, yoff);
      add_line(dir == HOR ? (puy - cpy) / 4 : (pux - cpx) / 4);
      if ((pu.sub & 1) || (cu.flags & DBC_AFFINE)) {
        if (dir == HOR) {
          for (int off = 8; off < pa[3]; off += 8) {
            set_edges(HOR, cu.x, cu.y + off, cu.w, 4, internal, true);
            add_line((puy + off - cpy) / 4);
          }
        } else {
          for (int off = 8; off < pa[2]; off += 8) {
            set_edges(VER, cu.x + off, cu.y, 4, cu.h, internal, true);
            add_line((pux + off - cpx) / 4);
          }
        }
        if (pu.w > 0) len_subblocks(dir, pu, pa[2], pa[3]);
      }
    }
    // an edge inside an inter, non-CIIP luma CU that is not a transform edge has only the motion part
    const bool fast = yv && !(cu.flags & DBC_INTRA) && !(cu.flags & DBC_CIIP);
    uint8_t *bs = A.bs[dir];
    const uint8_t *edge = A.edge[dir];
    auto bs_at = [&](int x, int y) {
      const int p = pos(a[0] + x, a[1] + y);
      if (!edge[p]) return;
      if (fast && bs[p] == 0 && (dir == VER ? x : y) > 0) bs[p] = (uint8_t)motion_bs(dir, a[0] + x, a[1] + y, 0);
      else bs[p] = (uint8_t)boundary_strength(cui, dir, a[0] + x, a[1] + y);
    };
    if (yv) {
      const bool ver = dir == VER;
      for (uint64_t m = lines; m; m &= m - 1) {
        const int o = __ffsll((unsigned long long)m) - 1;
        const int o4 = o * 4;
        if (o4 >= (ver ? a[2] : a[3])) continue;
        if (ver) { for (int y = 0; y < a[3]; y += 4) bs_at(o4, y); }
        else { for (int x = 0; x < a[2]; x += 4) bs_at(x, o4); }
      }
    } else {
      for (int y = 0; y < a[3]; y += 4)
        for (int x = 0; x < a[2]; x += 4) bs_at(x, y);
    }
    for (uint64_t m = lines; m; m &= m - 1) {
      const int e = __ffsll((unsigned long long)m) - 1;
      if (yv) emit_luma(cui, dir, e);
      if ((cu.flags & DBC_CVALID) && (!(cu.flags & DBC_ISP) || e == 0)) emit_chroma(cui, dir, e);
    }
  }
};

// index maps: CU per 4x4 luma / 2x2 chroma unit, TU likewise (an ISP CU's luma area holds -(first TU) - 2)
__global__ __launch_bounds__(256) void k_dbkp_maps(DbkPlanArgs A) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  auto fill = [&](int32_t *m, int x, int y, int w, int h, int s, int v, bool atomic) {
    for (int j = y >> s; j < cdiv(y + h, s); j++)
      for (int k = x >> s; k < cdiv(x + w, s); k++) {
        if (atomic) atomicMax(&m[j * A.W4 + k], v);   // later TUs win (the host planner's order)
        else m[j * A.W4 + k] = v;
      }
  };
  if (i < A.ncu) {
    const DbCu &c = A.cu[i];
    // (a later CU wins where two cover a unit, as the host planner's fill in CU order)
    if (c.flags & DBC_YVALID) fill(A.cu_map[0], c.x, c.y, c.w, c.h, 2, i, true);
    if (c.flags & DBC_CVALID) fill(A.cu_map[1], c.cx, c.cy, c.cw, c.ch, 1, i, true);
  } else if (i < A.ncu + A.ntu) {
    const int t = i - A.ncu;
    const DbTu &tu = A.tu[t];
    const DbCu &c = A.cu[tu.cu];
    const int16_t *b0 = tu.b[0], *b1 = tu.b[1];
    if (b0[2] > 0 && b0[3] > 0) {
      if (c.flags & DBC_ISP) {
        if (t == c.firsttu) fill(A.tu_map[0], c.x, c.y, c.w, c.h, 2, -t - 2, false);
      } else {
        fill(A.tu_map[0], b0[0], b0[1], b0[2], b0[3], 2, t, true);
      }
    }
    if (b1[2] > 0 && b1[3] > 0) fill(A.tu_map[1], b1[0], b1[1], b1[2], b1[3], 1, t, true);
  }
}

// one thread per (CU, direction) of the pass's channel type. The host planner runs the CUs of a CTU in
// order, the chroma tree after the luma tree: pass 0 takes the chtype-0 CUs (they never overlap), pass 1
// the chtype-1 ones — after a clear of the scratch maps in a dual-tree picture (the host's per-pass reset),
// on top of the luma CUs' state for the chroma CUs of a local dual tree (the host's CU order within the CTU).
// A shard plans the CUs within VVCR_LF_HALO rows of its own rows.
template <int DIR>
__global__ __launch_bounds__(64) void k_dbkp_cu(DbkPlanArgs A) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= A.ncu) return;
  const DbCu &c = A.cu[i];
  if ((c.flags & DBC_CHTYPE ? 1 : 0) != A.pass) return;
  if (A.shard) {
    const int ctu = 1 << A.ctu_log2;
    int a[4];
    Planner::cu_area(c, a);
    const int ctu_y = a[1] & ~(ctu - 1);
    if (ctu_y + ctu <= A.ly0 || ctu_y >= A.ly1) return;
    if (!(a[1] + a[3] > A.ly0 && a[1] < A.ly1)) return;
  }
  Planner(A).deblock_cu(i, DIR);
}

// dense segment words -> the four lists (luma VER, chroma VER, luma HOR, chroma HOR), each list at
// A.out + k * A.cap; a workgroup reserves its run of each list with one atomic
__global__ __launch_bounds__(256) void k_dbkp_compact(DbkPlanArgs A, int n4) {
  __shared__ int s_cnt[4][4], s_base[4];
  const int i = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t wd[4] = {0, 0, 0, 0};
  if (i < n4) { wd[0] = A.segL[0][i]; wd[1] = A.segC[0][i]; wd[2] = A.segL[1][i]; wd[3] = A.segC[1][i]; }
  int rank[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const unsigned long long m = __ballot(wd[k] != 0);
    rank[k] = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) s_cnt[k][wv] = __popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    const int tot = s_cnt[k][0] + s_cnt[k][1] + s_cnt[k][2] + s_cnt[k][3];
    s_base[k] = tot ? atomicAdd(&A.counts[k], tot) : 0;
  }
  __syncthreads();
  if (i >= n4) return;
  const int x4 = i % A.W4, y4 = i / A.W4;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (!wd[k]) continue;
    int off = s_base[k] + rank[k];
    for (int q = 0; q < wv; q++) off += s_cnt[k][q];
    if (off < A.cap) A.out[(size_t)k * A.cap + off] = DbkSeg{(uint16_t)x4, (uint16_t)y4, wd[k]};
    else atomicOr(A.err, 4);
  }
}

}  // namespace

void launch_dbk_plan(const DbkPlanArgs &a0, hipStream_t s) {
  DbkPlanArgs a = a0;
  const size_t n4 = (size_t)a.W4 * a.H4;
  for (int k = 0; k < 2; k++) {
    VVCR_CHECK_HIP(hipMemsetAsync(a.cu_map[k], 0xff, n4 * sizeof(int32_t), s));
    VVCR_CHECK_HIP(hipMemsetAsync(a.tu_map[k], 0xff, n4 * sizeof(int32_t), s));
  }
  VVCR_CHECK_HIP(hipMemsetAsync(a.scratch0, 0, a.scratch_bytes + a.dense_bytes, s));
  VVCR_CHECK_HIP(hipMemsetAsync(a.counts, 0, 4 * sizeof(int32_t), s));
  const int nm = a.ncu + a.ntu;
  if (nm > 0) hipLaunchKernelGGL(k_dbkp_maps, dim3((nm + 255) / 256), dim3(256), 0, s, a);
  const dim3 g((a.ncu + 63) / 64);
  for (int pass = 0; pass < (a.chroma_pass ? 2 : 1); pass++) {
    a.pass = pass;
    if (pass == 1 && a.dual_tree) VVCR_CHECK_HIP(hipMemsetAsync(a.scratch0, 0, a.scratch_bytes, s));
    if (a.ncu > 0) {
      hipLaunchKernelGGL(k_dbkp_cu<0>, g, dim3(64), 0, s, a);
      hipLaunchKernelGGL(k_dbkp_cu<1>, g, dim3(64), 0, s, a);
    }
  }
  hipLaunchKernelGGL(k_dbkp_compact, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, a, (int)n4);
  VVCR_CHECK_HIP(hipGetLastError());
}
