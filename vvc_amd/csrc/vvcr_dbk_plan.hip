// vvcr_dbk_plan.hip — deblocking edge planning on the device (SURVEY.md K12 "metadata kernel"; r05): the
// control part of LoopFilter::xDeblockCU (LoopFilter.cpp:261-408) that vvcr_dbk_host.cpp runs on the
// host — edge flags and TU / PU / sub-block markers (xSetEdgefilterMultiple :627), filter lengths from
// transform sizes (:454) and of SbTMVP / affine sub-blocks (:550), xGetBoundaryStrengthSingle (:674), and
// the QP / length bookkeeping of xEdgeFilterLuma (:844-979) and xEdgeFilterChroma (:1087-1244). It is the
// same algorithm as the host planner (every rule cited there), restated per position: the edge state of a
// 4x4 unit (edge flag, boundary-strength marker / value, transform-edge flag, filter lengths) is written
// only by the CU that covers the unit, through calls whose effect on the unit follows from the CU's TU / PU
// records alone — xSetEdgefilterMultiple marks a line of units, the length rules read the neighbouring
// TU through the index maps, and the sub-block rule reads the transform-edge flags of units of the same
// PU, which are a predicate of the CU's TUs. So each unit on one of its CU's edge lines replays, per
// direction, exactly the calls of its CU that touch it, in the reference's order, with the state in
// registers:
//   1. the xSetEdgefilterMultiple calls of the TUs, the PU and its sub-block lines
//   2. the transform-size filter lengths of the TU whose edge holds the unit
//   3. the sub-block filter lengths of an SbTMVP / affine PU
//   4. the boundary strength
//   5. the segment words, appended to the four lists k_dbk reads (a workgroup-aggregated atomic a list; every
//      segment of one direction is independent, so the lists' order does not change the samples)
// The chroma-tree CUs of a picture (dual tree, or the chroma CUs of a local dual tree) run after the luma
// tree's, from a clean state (dual tree: the host's per-pass reset) or on top of the luma CU's state of the
// unit (local dual tree: the host's CU order within the CTU; the luma pass leaves it in a state map).
// Kernels, per picture, on the picture's lane before the deblocking filter:
//   k_dbkp_maps      CU index maps (luma 4x4 / chroma 2x2 units) and TU index maps, a wave per CU / TU
//                    record; the CU's waves list the units on their CUs' edge lines (items)
//   k_dbkp_units<P>  steps 1-5, a thread per item of pass P (both directions, split by block)
// Inputs: compact CU / PU / TU records (DbCu / DbPu / DbTu, vvcr_dbk.h, built by pack_dbk_inputs) and the
// 4x4 motion field (MotionRec) of the picture, uploaded with its work lists.
//
// Records are read from global memory where they are used, never copied into local structs: a run-time
// choice between two fields of a local struct is folded by the compiler into a load through a selected
// address, which puts the struct in scratch memory (measured: 400 bytes a lane, slower than the loads).
#include "vvcr_dbk.h"

namespace {

enum { VER = 0, HOR = 1 };
constexpr int MAXTU = 4;   // TUs of a CU (the 64-sample transform split of a 128 CU, ISP, the chroma of a 128 area)

__device__ __forceinline__ int cdiv(int a, int s) { return (a + (1 << s) - 1) >> s; }

// a map entry of this picture's generation -> its index (an ISP CU's luma area: -(first TU) - 2), else -1
__device__ __forceinline__ int map_val(const DbkPlanArgs &A, int32_t v) {
  if ((int)((uint32_t)v >> DBKP_GEN_SHIFT) != A.gen) return -1;
  const int i = v & DBKP_IDX_MASK;
  return (v & DBKP_ISP) ? -i - 2 : i;
}

// the edge state of one unit and direction (the reference's per-CTU m_aapucBS / m_aapbEdgeFilter /
// m_maxFilterLength* entries; chroma lengths of Cb only: Cr's equal them and are never read)
struct UnitState {
  int edge, bs, tedge, lp0, lq0, lp1, lq1;
};

// Records come in whole, as 16-byte loads into registers, and their fields are taken by shifts (r06: a lane
// used to read each 2-byte field where it was used: ~250 short loads of 64 scattered addresses per wave
// instruction kept the texture address units busy and the waves waiting). Fields are picked with constant
// indices only, so no record is ever addressed through a run-time index (that would put it in scratch).
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ int lo16s(uint32_t v) { return (int)(int16_t)(uint16_t)(v & 0xffffu); }
__device__ __forceinline__ int hi16s(uint32_t v) { return (int)(int16_t)(uint16_t)(v >> 16); }
// dword 7 of a DbTu: cbf | jccr << 8 | cqp[0] << 16 | cqp[1] << 24
__device__ __forceinline__ uint32_t tu_word7(const DbkPlanArgs &A, int t) { return ((const uint32_t *)(A.tu + t))[7]; }
__device__ __forceinline__ int w7_cqp(uint32_t w, int k) { return (int)(int8_t)(uint8_t)(w >> (16 + 8 * k)); }

// One CU: its record, its PU's and the luma / chroma areas of its TUs (b[0], b[1]: tb[k][0..3] = x | y << 16,
// w | h << 16 of luma, then of chroma)
struct Cu {
  uint32_t tb[MAXTU][4];
  int t0;                // its first TU's index
  int flags, qp, ntu, npu;
  int x, y, w, h, cx, cy;
  int a0, a1, a2, a3;    // luma area (a chroma-tree CU: its chroma area doubled)
  int yv, isp, ch, cpx, cpy;
  int left, top, internal;
  int sub;               // SbTMVP / affine: sub-block edges
  int puw;               // the PU's luma width (0: none)
  int pux, puy;          // the PU origin in the CU's channel
  int pa0, pa1, pa2, pa3;   // the PU's luma area (a chroma-tree CU: the CU's)
  // b[C][K] of TU k (C: 0 luma, 1 chroma; K: x, y, w, h)
  template <int C, int K> __device__ __forceinline__ int tb_f(int k) const {
    const uint32_t v = tb[k][2 * C + K / 2];
    return (K & 1) ? hi16s(v) : lo16s(v);
  }
};

__device__ __forceinline__ Cu load_cu(const DbkPlanArgs &A, int i) {
  const u32x4a *c = (const u32x4a *)(A.cu + i);
  const u32x4a c0 = c[0], c1 = c[1];   // x y w h cx cy cw ch | firstpu firsttu npu ntu qp flags
  Cu R;
  R.x = lo16s(c0.x); R.y = hi16s(c0.x); R.w = lo16s(c0.y); R.h = hi16s(c0.y); R.cx = lo16s(c0.z); R.cy = hi16s(c0.z);
  const int cw = lo16s(c0.w), chh = hi16s(c0.w);
  const int firstpu = (int)c1.x;
  R.t0 = (int)c1.y;
  R.npu = lo16s(c1.z); R.ntu = hi16s(c1.z);
  R.qp = lo16s(c1.w); R.flags = (int)(c1.w >> 16);
  if (R.ntu > MAXTU || R.npu > 1 || R.ntu < 0 || R.npu < 0) {   // never in VVC: inconsistent descriptors
    atomicOr(A.err, 2);
    R.ntu = min(max(R.ntu, 0), MAXTU); R.npu = min(max(R.npu, 0), 1);
  }
#pragma unroll
  for (int k = 0; k < MAXTU; k++) {
    u32x4a v = {0u, 0u, 0u, 0u};
    if (k < R.ntu) v = *(const u32x4a *)(A.tu + R.t0 + k);
    R.tb[k][0] = v.x; R.tb[k][1] = v.y; R.tb[k][2] = v.z; R.tb[k][3] = v.w;
  }
  u32x4a pv = {0u, 0u, 0u, 0u};   // x y w h cx cy sub
  if (R.npu) pv = *(const u32x4a *)(A.pu + max(firstpu, 0));
  R.yv = (R.flags & DBC_YVALID) ? 1 : 0;
  R.isp = (R.flags & DBC_ISP) ? 1 : 0;
  R.ch = (R.flags & DBC_CHTYPE) ? 1 : 0;
  R.a0 = R.yv ? R.x : 2 * R.cx; R.a1 = R.yv ? R.y : 2 * R.cy;
  R.a2 = R.yv ? R.w : 2 * cw; R.a3 = R.yv ? R.h : 2 * chh;
  R.cpx = R.ch ? R.cx : R.x; R.cpy = R.ch ? R.cy : R.y;
  if (A.dbk_disable) { R.left = R.top = R.internal = 0; }
  else { R.internal = 1; R.left = R.cpx > 0 && !(R.flags & DBC_NOLEFT); R.top = R.cpy > 0 && !(R.flags & DBC_NOTOP); }
  const int pX = lo16s(pv.x), pY = hi16s(pv.x), pW = lo16s(pv.y), pH = hi16s(pv.y), pCx = lo16s(pv.z), pCy = hi16s(pv.z);
  R.sub = R.npu && ((pv.w & 1) || (R.flags & DBC_AFFINE));
  R.puw = R.npu ? pW : 0;
  R.pux = R.npu ? (R.ch ? pCx : pX) : R.cpx;
  R.puy = R.npu ? (R.ch ? pCy : pY) : R.cpy;
  const bool own = R.npu && R.yv;
  R.pa0 = own ? pX : R.a0; R.pa1 = own ? pY : R.a1;
  R.pa2 = own ? pW : R.a2; R.pa3 = own ? pH : R.a3;
  return R;
}

__device__ __forceinline__ int bs_set(int v, int comp) { return v << (comp * 2); }

// One unit (x4, y4) of CU R in direction DIR
template <int DIR>
struct Unit {
  const DbkPlanArgs &A;
  const int (*ref_poc)[VVCR_MAX_REF];   // A.ref_poc in LDS
  const Cu &R;
  const int x4, y4;
  static constexpr bool ver = DIR == VER;

  // xSetEdgefilterMultiple(dir, x, y, w, h, val, edgeIdx) (:627) applied to this unit if its line holds it
  __device__ __forceinline__ void set_edges(UnitState &st, int x, int y, int w, int h, int val, bool edgeIdx) const {
    const bool hit = ver ? (x4 == (x >> 2) && y4 >= (y >> 2) && y4 < (y >> 2) + (h >> 2))
                         : (y4 == (y >> 2) && x4 >= (x >> 2) && x4 < (x >> 2) + (w >> 2));
    if (!hit) return;
    st.edge = val;
    if (st.bs && val) st.bs = 3;
    else if (!edgeIdx) st.bs = val;
  }

  // whether the length rule (:454) of TU k, component COMP (0 luma, 1 chroma), covers unit (ux, uy); then
  // (X, Y) are its component samples
  template <int COMP>
  __device__ __forceinline__ bool tu_edge(int k, int ux, int uy, int &X, int &Y) const {
    const int bx = R.tb_f<COMP, 0>(k), by = R.tb_f<COMP, 1>(k), bw = R.tb_f<COMP, 2>(k), bh = R.tb_f<COMP, 3>(k);
    if (bw <= 0 || bh <= 0) return false;
    const int cux = COMP ? R.cx : R.x, cuy = COMP ? R.cy : R.y;
    // (bx == cux ? left : internal): left implies internal
    if (!(ver ? (R.internal & ((bx != cux) | R.left)) : (R.internal & ((by != cuy) | R.top)))) return false;
    constexpr int g = COMP ? 1 : 2, step = 1 << g;   // the unit's component samples: (ux, uy) << g
    X = ux << g; Y = uy << g;
    if (!ver) return Y == by && X >= bx && X < bx + bw && ((X - bx) & (step - 1)) == 0;
    return X == bx && Y >= by && Y < by + bh && ((Y - by) & (step - 1)) == 0;
  }

  // the transform-edge flag of unit (ux, uy) of this CU after step 2 (the luma rule of its TUs)
  __device__ __forceinline__ bool tedge_at(int ux, int uy) const {
    bool e = false;
#pragma unroll
    for (int k = 0; k < MAXTU; k++) {
      int X, Y;
      if (k < R.ntu && tu_edge<0>(k, ux, uy, X, Y)) e = true;
    }
    return e;
  }

  // the index (in A.tu) of the CU's TU holding sample (x, y) of channel c (CodingStructure::getTU: the index
  // maps' last writer; an ISP CU's first sub-partition that holds it), -1 for none
  __device__ __forceinline__ int own_tu(int c, int x, int y) const {
    int f = -1;
    const int g = 2 - c;   // the index maps' unit: 4x4 luma / 2x2 chroma samples
#pragma unroll
    for (int k = MAXTU - 1; k >= 0; k--) {
      if (k >= R.ntu) continue;
      const int b0 = c ? R.tb_f<1, 0>(k) : R.tb_f<0, 0>(k), b1 = c ? R.tb_f<1, 1>(k) : R.tb_f<0, 1>(k);
      const int b2 = c ? R.tb_f<1, 2>(k) : R.tb_f<0, 2>(k), b3 = c ? R.tb_f<1, 3>(k) : R.tb_f<0, 3>(k);
      const bool in = b2 > 0 && b3 > 0 && (R.isp && c == 0 ? (x >= b0 && x < b0 + b2 && y >= b1 && y < b1 + b3)
                                                           : ((x >> g) >= (b0 >> g) && (x >> g) < ((b0 + b2 + (1 << g) - 1) >> g) &&
                                                              (y >> g) >= (b1 >> g) && (y >> g) < ((b1 + b3 + (1 << g) - 1) >> g)));
      if (in && (f < 0 || (R.isp && c == 0))) f = k;
    }
    return f < 0 ? -1 : R.t0 + f;
  }
  // a TU index found by own_tu / map_tu, or the error bit and the stand-in record (fb) for none
  __device__ __forceinline__ int use_tu(int t, int fb) const {
    if (t < 0) { atomicOr(A.err, 2); return fb; }
    return t;
  }

  // a TU index from an index map value t at the neighbouring unit (an ISP CU's luma area: its
  // sub-partition holding sample (x, y)); -1 for a hole
  __device__ __forceinline__ int map_tu(int t, int x, int y) const {
    if (t >= -1) return t;
    t = -t - 2;
    int r = t;
#pragma unroll 1
    for (int k = 0; k < 4 && t + k < A.ntu; k++) {
      const u32x2a v = *(const u32x2a *)(A.tu + t + k);   // b[0]: x | y << 16, w | h << 16
      const int bx = lo16s(v.x), by = hi16s(v.x), bw = lo16s(v.y), bh = hi16s(v.y);
      if (x >= bx && x < bx + bw && y >= by && y < by + bh) { r = t + k; break; }
    }
    return r;
  }
  __device__ __forceinline__ int map_cu(int i) const {
    if (i < 0) { atomicOr(A.err, 2); return 0; }   // "deblocking: no CU covers a neighbouring position"
    return i;
  }

  // the motion part of xGetBoundaryStrengthSingle (:748-812)
  __device__ __forceinline__ int motion_bs(const MotionRec &mp, const MotionRec &mq, int tmp) const {
    const int th = 8;
    // the same motion on both sides (one PU, or equal neighbours): no motion boundary
    if (mp.ref0 == mq.ref0 && mp.ref1 == mq.ref1 && mp.mv0x == mq.mv0x && mp.mv0y == mq.mv0y && mp.mv1x == mq.mv1x &&
        mp.mv1y == mq.mv1y && (mp.ref0 >= 0 || A.slice_type == 0))
      return tmp;
    if (A.slice_type == 0) {
      const int NONE = INT32_MIN;
      const int rP0 = mp.ref0 >= 0 ? ref_poc[0][mp.ref0] : NONE, rP1 = mp.ref1 >= 0 ? ref_poc[1][mp.ref1] : NONE;
      const int rQ0 = mq.ref0 >= 0 ? ref_poc[0][mq.ref0] : NONE, rQ1 = mq.ref1 >= 0 ? ref_poc[1][mq.ref1] : NONE;
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
    if (ref_poc[0][mp.ref0] != ref_poc[0][mq.ref0]) return tmp + 1;
    return (abs(mq.mv0x - mp.mv0x) >= th || abs(mq.mv0y - mp.mv0y) >= th) ? tmp + 1 : tmp;
  }

  // LoopFilter::xDeblockCU (the host planner's deblock_cu) restricted to this unit, which lies on line o of
  // the CU: the state it leaves there, and the unit's luma / chroma segment words (0: none)
  __device__ __forceinline__ void run(int o, UnitState &st, uint32_t &wl, uint32_t &wc) const {
    const int px = x4 * 4, py = y4 * 4;
    const int u = y4 * A.W4 + x4, pu = ver ? u - 1 : u - A.W4;
    // P side inside the CU (else through the index maps); none across the picture edge (left / top false)
    const bool pedge = ver ? x4 == 0 : y4 == 0;
    const bool pin = (ver ? x4 > (R.a0 >> 2) : y4 > (R.a1 >> 2)) || pedge;
    // the P side's index-map values and CU record and the motion of both sides, loaded up front (one round
    // of loads each; their uses below are conditional)
    int mcu = 0, mcu1 = 0, mtu0 = 0, mtu1 = 0;
    if (!pin) {
      const int32_t v0 = A.cu_map[0][pu], v1 = A.cu_map[1][pu], t0 = A.tu_map[0][pu], t1 = A.tu_map[1][pu];
      mcu1 = map_val(A, v1);
      mcu = R.ch ? mcu1 : map_val(A, v0);
      mtu0 = map_val(A, t0);
      mtu1 = map_val(A, t1);
    }
    // dword 7 of the P-side CU record: qp | flags << 16
    const uint32_t cPw = pin ? 0u : ((const uint32_t *)(A.cu + max(mcu, 0)))[7];
    const int fPm = (int)(cPw >> 16), qpPm = lo16s(cPw);
    // (no motion edge at the picture edge; no field: a picture without inter CUs never asks for motion)
    MotionRec mp{}, mq{};
    if (A.motion) { mp = A.motion[pedge ? u : pu]; mq = A.motion[u]; }
    // The TUs the rules read, each found once: the P side's luma / chroma TU at the sample left of / above
    // the unit's first sample (inside the CU: the CU's own TUs, else the neighbour's index-map entry; the
    // stand-in for none is the CU's first TU / record 0, with the error bit where a rule uses it), and the
    // unit's own TU in the CU's channel
    const int fbP = pin ? R.t0 : 0;
    const int tpL = pedge ? -1 : (pin ? own_tu(0, ver ? px - 1 : px, ver ? py : py - 1) : map_tu(mtu0, ver ? px - 1 : px, ver ? py : py - 1));
    const int cx2 = 2 * x4, cy2 = 2 * y4;   // the unit's first chroma sample
    const int tpC = pedge ? -1 : (pin ? own_tu(1, ver ? cx2 - 1 : cx2, ver ? cy2 : cy2 - 1) : mtu1);
    const int tqO = R.ch ? own_tu(1, cx2, cy2) : own_tu(0, px, py);
    // step 1 (TU calls, then the PU's call and its sub-block lines)
#pragma unroll
    for (int k = 0; k < MAXTU; k++) {
      if (k >= R.ntu) continue;
      if (R.yv) set_edges(st, R.tb_f<0, 0>(k), R.tb_f<0, 1>(k), R.tb_f<0, 2>(k), R.tb_f<0, 3>(k), R.internal, false);
      else set_edges(st, R.a0, R.a1, R.a2, R.a3, R.internal, false);
    }
    if (R.npu) {
      const int off = ver ? R.pux != R.cpx : R.puy != R.cpy;
      set_edges(st, R.pa0, R.pa1, R.pa2, R.pa3, R.internal & (off | (ver ? R.left : R.top)), off);
      if (R.sub) {
        if (ver) { for (int d = 8; d < R.pa2; d += 8) set_edges(st, R.x + d, R.y, 4, R.h, R.internal, true); }
        else { for (int d = 8; d < R.pa3; d += 8) set_edges(st, R.x, R.y + d, R.w, 4, R.internal, true); }
      }
    }
    // step 2 (the host interleaves it with step 1 per TU; the two write disjoint state)
#pragma unroll
    for (int k = 0; k < MAXTU; k++) {
      if (k >= R.ntu) continue;
      int X, Y;
      if (tu_edge<0>(k, x4, y4, X, Y)) {
        const int sizeQ = ver ? R.tb_f<0, 2>(k) : R.tb_f<0, 3>(k);
        const int tp = use_tu(tpL, fbP);   // (X - 1, Y) / (X, Y - 1): X, Y are px, py
        const int sizeP = ver ? A.tu[tp].b[0][2] : A.tu[tp].b[0][3];
        st.tedge = 1;
        const bool small = sizeP <= 4 || sizeQ <= 4;
        st.lq0 = small ? 1 : (sizeQ >= 32 ? 7 : 3);
        st.lp0 = small ? 1 : (sizeP >= 32 ? 7 : 3);
      }
      if (tu_edge<1>(k, x4, y4, X, Y)) {
        const int sizeQ = ver ? R.tb_f<1, 2>(k) : R.tb_f<1, 3>(k);
        const int tp = use_tu(tpC, fbP);   // X, Y: the unit's first chroma sample
        const int sizeP = ver ? A.tu[tp].b[1][2] : A.tu[tp].b[1][3];
        st.lq1 = st.lp1 = (sizeQ >= 8 && sizeP >= 8) ? 3 : 1;
      }
    }
    // step 3: sub-block lengths (:550), units every 8 samples across, every 4 along the PU
    if (R.sub && R.puw > 0) {
      const int outer = ver ? R.pa2 : R.pa3, inner = ver ? R.pa3 : R.pa2;
      const int a8 = ver ? px - R.pa0 : py - R.pa1, b4 = ver ? py - R.pa1 : px - R.pa0;
      if (a8 >= 0 && a8 < outer && !(a8 & 7) && b4 >= 0 && b4 < inner) {
        auto T = [&](int delta) { return ver ? tedge_at(x4 + delta / 4, y4) : tedge_at(x4, y4 + delta / 4); };
        if (st.tedge) {
          if (st.lq0 > 5) st.lq0 = 5;
          if (a8 > 0 && st.lp0 > 5) st.lp0 = 5;
        } else if (a8 > 0 && (T(-4) || a8 + 4 >= outer || T(4))) {
          st.lq0 = st.lp0 = 1;
        } else if (a8 > 0 && (T(-8) || a8 + 8 >= outer || T(8))) {
          st.lq0 = st.lp0 = 2;
        } else {
          st.lq0 = st.lp0 = 3;
        }
      }
    }
    // the P-side CU of the CU's channel
    if (!pin) map_cu(mcu);   // (a hole: the error bit; record 0 stands in, as in the host planner's lookup)
    const int fQ = R.flags;
    // step 4: xGetBoundaryStrengthSingle (:674); an edge inside an inter, non-CIIP luma CU that is not a
    // transform edge has only the motion part
    if (st.edge && (!R.yv || o * 4 < (ver ? R.a2 : R.a3))) {
      const bool fast = R.yv && !(fQ & DBC_INTRA) && !(fQ & DBC_CIIP);
      if (fast && st.bs == 0 && o > 0) {
        st.bs = motion_bs(mp, mq, 0);
      } else {
        const int marker = st.bs;
        const int fP = pin ? fQ : fPm;
        const bool iP = fP & DBC_INTRA, iQ = fQ & DBC_INTRA;
        if (iP || iQ) {
          const int bsY = (iP && (fP & DBC_BDPCM)) && (iQ && (fQ & DBC_BDPCM)) ? 0 : 2;
          const int bsC = (iP && (fP & DBC_BDPCMC)) && (iQ && (fQ & DBC_BDPCMC)) ? 0 : 2;
          st.bs = bs_set(bsY, 0) + bs_set(bsC, 1) + bs_set(bsC, 2);
        } else {
          const bool ciip = (fQ & DBC_CIIP) || (!pin && (fP & DBC_CIIP));
          if (marker && ciip) {
            st.bs = bs_set(2, 0) + bs_set(2, 1) + bs_set(2, 2);
          } else {
            int tmp = 0;
            if (marker) {
              // (the CU's channel: a luma CU's samples (px, py), a chroma-tree CU's (px, py) / 2)
              const int tq = use_tu(tqO, R.t0), tp = use_tu(R.ch ? tpC : tpL, fbP);
              const uint32_t wq = tu_word7(A, tq), wp = tu_word7(A, tp);
              const int cq = wq & 255, cp = wp & 255, jq = (wq >> 8) & 255, jp = (wp >> 8) & 255;
              if ((cq & 1) || (cp & 1)) tmp += bs_set(1, 0);
              if ((cq & 2) || (cp & 2) || jq || jp) tmp += bs_set(1, 1);
              if ((cq & 4) || (cp & 4) || jq || jp) tmp += bs_set(1, 2);
            }
            if ((tmp & 3) == 1) st.bs = tmp;
            else if (ciip) st.bs = 1;
            else if (!R.yv) st.bs = tmp;
            else if (marker != 0 && marker != 3) st.bs = tmp;
            else st.bs = motion_bs(mp, mq, tmp);
          }
        }
      }
    }
    // step 5: the segment words (xEdgeFilterLuma / xEdgeFilterChroma bookkeeping); none on a virtual
    // boundary (xDeriveEdgefilterParam, LoopFilter.cpp:433: the edge's filter flag is cleared)
#pragma unroll
    for (int i = 0; i < 3; i++)
      if (i < A.num_vb[DIR] && (ver ? px : py) == A.vb[DIR][i]) return;
    if (R.yv && (st.bs & 3)) {
      const int qpP = pin ? R.qp : qpPm, fP = pin ? fQ : fPm;
      const int qp = (qpP + R.qp + 1) >> 1;
      int lp = st.lp0, lq = st.lq0;
      bool pl = false, ql = false;
      if (lp > 3) {
        pl = true;
        if (lp > 5 && (fP & DBC_AFFINE)) lp = 5;
      }
      if (lq > 3) ql = true;
      if (!ver && (py & ((1 << A.ctu_log2) - 1)) == 0) pl = false;
      wl = (uint32_t)(st.bs & 3) | (uint32_t)lp << 2 | (uint32_t)lq << 5 | (uint32_t)(qp & 63) << 8 | (uint32_t)pl << 14 | (uint32_t)ql << 15;
    }
    if ((fQ & DBC_CVALID) && (!R.isp || o == 0)) {
      const int ctu = 1 << A.ctu_log2, parts = ctu / 4;
      const int r = ((R.a0 & (ctu - 1)) >> 2) + ((R.a1 & (ctu - 1)) >> 2) * parts;   // the CTU raster index of the host planner
      const int bS0 = (st.bs >> 2) & 3, bS1 = (st.bs >> 4) & 3;
      if (!((ver && (r % parts + o) % 4) || (!ver && (r / parts + o) % 4)) && (bS0 || bS1)) {
        // the P-side CU: of the chroma map when the luma one is of a tree-split area or the picture is dual tree
        int fP = pin ? fQ : fPm;
        if (!pin && R.ch == 0 && ((fPm & DBC_TREE) || A.dual_tree)) fP = (int)(((const uint32_t *)(A.cu + map_cu(mcu1)))[7] >> 16);
        const bool large = st.lp1 >= 3 && st.lq1 >= 3;
        const bool ctbh = !ver && (py & ((1 << A.ctu_log2) - 1)) == 0;
        uint32_t w = (uint32_t)large << 4 | (uint32_t)ctbh << 19;
        bool any = false;
        // (the P CU's channel: a luma CU's samples (px, py), a chroma-tree CU's (px, py) / 2)
        const int tq = use_tu(tqO, R.t0), tp = use_tu((fP & DBC_CHTYPE) ? tpC : tpL, fbP);
        const uint32_t wq = tu_word7(A, tq), wp = tu_word7(A, tp);
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const int b = k ? bS1 : bS0;
          if (!(b == 2 || (large && b == 1))) continue;
          const int qp = (w7_cqp(wq, k) + w7_cqp(wp, k) + 1) >> 1;
          w |= (uint32_t)b << (2 * k) | (uint32_t)((qp + 64) & 127) << (5 + 7 * k);
          any = true;
        }
        if (any) wc = w;
      }
    }
  }
};

__device__ __forceinline__ bool in_shard(const DbkPlanArgs &A, const Cu &R) {
  if (!A.shard) return true;
  const int ctu = 1 << A.ctu_log2;
  const int ctu_y = R.a1 & ~(ctu - 1);
  if (ctu_y + ctu <= A.ly0 || ctu_y >= A.ly1) return false;
  return R.a1 + R.a3 > A.ly0 && R.a1 < A.ly1;
}

// The lanes of a 256-lane workgroup with wl / wc != 0 append (x4, y4, w) to the luma / chroma list of
// direction dir (lists 2 dir, 2 dir + 1): one atomic per workgroup for both lists, the waves' runs placed
// by their counts in LDS (an atomic per wave and list put 10 k atomics a 4K picture on the same four
// counters; r06: a 64-bit atomic per wave for both lists, no barriers, 21.6 / 17.2 -> 28.5 / 25.4 us per 4K
// picture and direction: the same-address atomics serialise). more: the caller loops again (the LDS counts
// are reused: a third barrier).
__device__ __forceinline__ void append_wg(const DbkPlanArgs &A, int dir, uint32_t wl, uint32_t wc, int x4, int y4, bool more) {
  __shared__ int s_cnt[4][2];
  __shared__ int s_base[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long ml = __ballot(wl != 0), mc = __ballot(wc != 0);
  if (lane == 0) { s_cnt[wv][0] = __popcll(ml); s_cnt[wv][1] = __popcll(mc); }
  __syncthreads();
  if (threadIdx.x == 0) {
    // both lists' counts in one 64-bit atomic (counts[2 dir] and counts[2 dir + 1] are one aligned pair:
    // luma the low word)
    const unsigned long long tl = (unsigned)(s_cnt[0][0] + s_cnt[1][0] + s_cnt[2][0] + s_cnt[3][0]);
    const unsigned long long tc = (unsigned)(s_cnt[0][1] + s_cnt[1][1] + s_cnt[2][1] + s_cnt[3][1]);
    const unsigned long long old = (tl | tc) ? atomicAdd((unsigned long long *)(A.counts + 2 * dir), tl | tc << 32) : 0ull;
    s_base[0] = (int)(uint32_t)old;
    s_base[1] = (int)(uint32_t)(old >> 32);
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1;
  int bl = s_base[0] + __popcll(ml & below), bc = s_base[1] + __popcll(mc & below);
  for (int w = 0; w < wv; w++) { bl += s_cnt[w][0]; bc += s_cnt[w][1]; }
  if (wl) {
    if (bl < A.cap) A.out[(size_t)(2 * dir) * A.cap + bl] = DbkSeg{(uint16_t)x4, (uint16_t)y4, wl};
    else atomicOr(A.err, 4);
  }
  if (wc) {
    if (bc < A.cap) A.out[(size_t)(2 * dir + 1) * A.cap + bc] = DbkSeg{(uint16_t)x4, (uint16_t)y4, wc};
    else atomicOr(A.err, 4);
  }
  if (more) __syncthreads();
}

// index maps: CU per 4x4 luma / 2x2 chroma unit, TU likewise (an ISP CU's luma area holds -(first TU) - 2).
// A CU's record also lists the units on its edge lines: an item (CU index << 10 | line << 5 | unit along the
// line) per unit, in the list of its pass and direction (A.items + (2 * pass + dir) * cap, lengths
// A.nitems[2 * pass + dir]). Records are the CUs, then the TUs, a wave each, a lane per unit (r06, 4K
// pictures: 8 / 16 / 32 lanes per record, several records per wave, took 36 / 24 / 17 us against 11.8).
// a record's work with lanes s, s + st, ...: its map fills and, for a CU, its items. The records of one map
// never share a unit (luma blocks lie on the 4-sample grid, an ISP CU's sub-partitions map as the CU's area;
// chroma blocks on the 2-sample grid), so the fills are plain stores (r06: atomicMax "later record wins"
// made the kernel atomic-bound, 13 us per 4K picture); the generation tag tells a stale entry from this
// picture's.
__device__ __forceinline__ void maps_record(const DbkPlanArgs &A, int i, int s, int st) {
  auto fill = [&](int32_t *m, int x, int y, int w, int h, int sh, int v) {
    const int x0 = x >> sh, y0 = y >> sh, nx = cdiv(x + w, sh) - x0, ny = cdiv(y + h, sh) - y0;
    const int32_t e = (int32_t)((uint32_t)A.gen << DBKP_GEN_SHIFT | (uint32_t)v);
    for (int j = s; j < nx * ny; j += st) m[(y0 + j / nx) * A.W4 + x0 + j % nx] = e;
  };
  if (i < A.ncu) {
    const DbCu &c = A.cu[i];
    if (i > DBKP_IDX_MASK) { if (s == 0) atomicOr(A.err, 4); return; }
    if (c.flags & DBC_YVALID) fill(A.cu_map[0], c.x, c.y, c.w, c.h, 2, i);
    if (c.flags & DBC_CVALID) fill(A.cu_map[1], c.cx, c.cy, c.cw, c.ch, 1, i);
    // the units on its edge lines (lines and list offsets from pack_dbk_inputs), line by line
    const int yv = (c.flags & DBC_YVALID) ? 1 : 0, ch = (c.flags & DBC_CHTYPE) ? 1 : 0;
    const int wq = (yv ? c.w : 2 * c.cw) >> 2, hq = (yv ? c.h : 2 * c.ch) >> 2;
#pragma unroll
    for (int d = 0; d < 2; d++) {
      uint32_t m = c.lines[d];
      const int n = d == VER ? hq : wq;
      const int total = __popc(m) * n, k = 2 * ch + d;
      int base = c.item0[d];
      if (base + total > A.cap || n > 32) { if (s == 0 && total) atomicOr(A.err, 4); continue; }
      uint32_t *out = A.items + (size_t)k * A.cap;
      for (; m; m &= m - 1, base += n) {
        const uint32_t line = (uint32_t)(__ffs(m) - 1);
        for (int j = s; j < n; j += st) out[base + j] = (uint32_t)i << 10 | line << 5 | (uint32_t)j;
      }
    }
  } else if (i < A.ncu + A.ntu) {
    const int t = i - A.ncu;
    const DbTu &tu = A.tu[t];
    const int16_t *b0 = tu.b[0], *b1 = tu.b[1];
    if (b0[2] > 0 && b0[3] > 0) {
      const DbCu &c = A.cu[tu.cu];
      if (c.flags & DBC_ISP) {
        if (t == c.firsttu) fill(A.tu_map[0], c.x, c.y, c.w, c.h, 2, DBKP_ISP | t);
      } else {
        fill(A.tu_map[0], b0[0], b0[1], b0[2], b0[3], 2, t);
      }
    }
    if (b1[2] > 0 && b1[3] > 0) fill(A.tu_map[1], b1[0], b1[1], b1[2], b1[3], 1, t);
  }
}

// The planner's lane arithmetic (lane = threadIdx.x & 63, 64-bit ballots, 4 waves per 256-lane workgroup)
// assumes 64-lane waves (gfx950 has no other mode): anything else raises error bit 8 and does nothing.
__device__ __forceinline__ bool wave64(const DbkPlanArgs &A) {
  if (__builtin_amdgcn_wavefrontsize() == 64) return true;
  if (threadIdx.x == 0) atomicOr(A.err, 8);
  return false;
}

__global__ __launch_bounds__(256) void k_dbkp_maps(DbkPlanArgs A) {
  if (!wave64(A)) return;
  if (blockIdx.x == 0 && threadIdx.x < 4) A.counts[threadIdx.x] = 0;   // the lists' lengths (k_dbkp_units appends)
  maps_record(A, blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63, 64);
}

// The items of pass PASS, direction DIR (blockIdx.y), a lane each, grid-stride; local_dual: the luma pass
// leaves each unit's edge flag and boundary strength in A.state, the chroma pass starts from it
template <int DIR, int PASS>
__device__ __forceinline__ void items_dir(const DbkPlanArgs &A, const int (*rp)[VVCR_MAX_REF], int blk, int nblk) {
  const int k = 2 * PASS + DIR;
  const int total = min(DIR == VER ? A.nitems[2 * PASS] : A.nitems[2 * PASS + 1], A.cap);
  const bool local_dual = A.chroma_pass && !A.dual_tree;
  for (int j0 = blk * 256; j0 < total; j0 += nblk * 256) {
    const int j = j0 + threadIdx.x;
    uint32_t wl = 0, wc = 0;
    int x4 = 0, y4 = 0;
    if (j < total) {
      const uint32_t it = A.items[(size_t)k * A.cap + j];
      const Cu R = load_cu(A, (int)(it >> 10));
      const int o = (it >> 5) & 31, i = it & 31;
      if (in_shard(A, R)) {
      x4 = (R.a0 >> 2) + (DIR == VER ? o : i);
      y4 = (R.a1 >> 2) + (DIR == VER ? i : o);
      const int u = y4 * A.W4 + x4;
      UnitState st{};
      if (PASS == 1 && local_dual) {
        const int v = A.state[DIR][u];
        st.edge = v >> 7; st.bs = v & 63;
      }
#ifdef DBKP_ABL_RUN   // diagnostics ablation: no replay (results wrong)
      wl = R.flags == 0xffff ? 1u : 0u;
#else
      Unit<DIR>{A, rp, R, x4, y4}.run(o, st, wl, wc);
#endif
      if (PASS == 0 && local_dual) A.state[DIR][u] = (uint8_t)(st.edge << 7 | (st.bs & 63));
      }
    }
#ifdef DBKP_ABL_APPEND   // diagnostics ablation: no list append (results wrong)
    if ((wl | wc) == 0xffffffffu) A.out[j0 + threadIdx.x] = DbkSeg{(uint16_t)x4, (uint16_t)y4, wl};
#else
    append_wg(A, DIR, wl, wc, x4, y4, j0 + nblk * 256 < total);
#endif
  }
}

// the units on the edge lines of the CUs of one pass (pass 0: the luma tree, pass 1: the chroma tree), a
// thread each: blocks [0, gv) the vertical edges' items, the others the horizontal ones' (both directions in
// one launch: a launch per direction cost a dispatch gap per picture)
template <int PASS>
__global__ __launch_bounds__(256) void k_dbkp_units(DbkPlanArgs A, int gv) {
  if (!wave64(A)) return;
  __shared__ int s_ref_poc[2][VVCR_MAX_REF];
  if (threadIdx.x < 2 * VVCR_MAX_REF) {
    int v = 0;
#pragma unroll
    for (int k = 0; k < 2 * VVCR_MAX_REF; k++) v = threadIdx.x == k ? A.ref_poc[k / VVCR_MAX_REF][k % VVCR_MAX_REF] : v;   // constant indices
    s_ref_poc[threadIdx.x / VVCR_MAX_REF][threadIdx.x % VVCR_MAX_REF] = v;
  }
  __syncthreads();
  if ((int)blockIdx.x < gv) items_dir<VER, PASS>(A, s_ref_poc, blockIdx.x, gv);
  else items_dir<HOR, PASS>(A, s_ref_poc, blockIdx.x - gv, gridDim.x - gv);
}

}  // namespace

void launch_dbk_plan(const DbkPlanArgs &a, hipStream_t s) {
  const size_t n4 = (size_t)a.W4 * a.H4;
  // the four maps are one run (vvcr_api.cpp dbk_plan_args): cleared only when the generation restarts (a
  // picture's entries are told from older ones by their tag); the list lengths every picture, by k_dbkp_maps
  if (a.fill) VVCR_CHECK_HIP(hipMemsetAsync(a.cu_map[0], 0, (size_t)((const char *)(a.tu_map[1] + n4) - (const char *)a.cu_map[0]), s));
  const bool local_dual = a.chroma_pass && !a.dual_tree;
  if (local_dual) VVCR_CHECK_HIP(hipMemsetAsync(a.state[0], 0, 2 * a.state_pitch, s));
  const int nm = a.ncu + a.ntu;
  hipLaunchKernelGGL(k_dbkp_maps, dim3(std::max(1, (nm + 3) / 4)), dim3(256), 0, s, a);   // (also zeroes the list lengths)
  for (int pass = 0; pass < 2; pass++) {
    const int gv = std::min(2048, (a.nitems[2 * pass] + 255) / 256), gh = std::min(2048, (a.nitems[2 * pass + 1] + 255) / 256);
    if (gv + gh == 0) continue;   // (grid-stride beyond 2048 blocks a direction)
    if (pass == 0) hipLaunchKernelGGL(k_dbkp_units<0>, dim3(gv + gh), dim3(256), 0, s, a, gv);
    else hipLaunchKernelGGL(k_dbkp_units<1>, dim3(gv + gh), dim3(256), 0, s, a, gv);
  }
  VVCR_CHECK_HIP(hipGetLastError());
}
