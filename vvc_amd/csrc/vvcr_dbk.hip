// vvcr_dbk.hip — deblocking filter for gfx950 (LoopFilter.cpp:844-1667 sample decisions + filters).
//
// The host plans every 4-sample edge segment (vvcr_dbk_host.cpp); here four lanes decide and filter
// one segment: one luma line each (xEdgeFilterLuma :981-1081), or one line of Cb or Cr each
// (xEdgeFilterChroma :1163-1283), with the segment decisions exchanged by shuffles. All vertical edges of the picture are filtered before any horizontal
// edge, as loopFilterPic (:165-240) does. Segments of one direction never overlap: each side modifies
// at most maxFilterLength samples and reads at most one more, and the reference's length rules
// (transform size <= 4 -> 1, sub-block edges 8 apart -> <= 3, 32-sample transforms for 7) keep the
// read window of one edge clear of the writes of the next, so the in-place parallel pass equals the
// reference's sequential CU order.
#include "vvcr_dbk.h"
#include "vvcr_gen_tables.h"
#include <algorithm>

namespace {

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int calc_dp(const int16_t *s, int o, bool ctbh) {
  return ctbh ? abs(s[-o * 2] - 2 * s[-o * 2] + s[-o]) : abs(s[-o * 3] - 2 * s[-o * 2] + s[-o]);
}
__device__ __forceinline__ int calc_dq(const int16_t *s, int o) { return abs(s[0] - 2 * s[o] + s[o * 2]); }

// xUseStrongFiltering (:1566), JVET_Q0054 variant for long-tap sides
__device__ bool use_strong(const int16_t *s, int o, int d, int beta, int tc, bool pl, bool ql, int lenP, int lenQ, bool ctbh) {
  const int m4 = s[0], m3 = s[-o], m7 = s[o * 3], m0 = s[-o * 4], m2 = s[-o * 2];
  int sp3 = ctbh ? abs(m2 - m3) : abs(m0 - m3);
  int sq3 = abs(m7 - m4);
  const int dstrong = sp3 + sq3;
  if (pl || ql) {
    if (pl) {
      int mP4;
      if (lenP == 7) { sp3 += abs(s[-o * 5] - s[-o * 6] - s[-o * 7] + s[-o * 8]); mP4 = s[-o * 8]; }
      else mP4 = s[-o * 6];
      sp3 = (sp3 + abs(m0 - mP4) + 1) >> 1;
    }
    if (ql) {
      int m11;
      if (lenQ == 7) { sq3 += abs(s[o * 4] - s[o * 5] - s[o * 6] + s[o * 7]); m11 = s[o * 7]; }
      else m11 = s[o * 5];
      sq3 = (sq3 + abs(m11 - m7) + 1) >> 1;
    }
    return (sp3 + sq3) < (beta * 3 >> 5) && d < (beta >> 4) && abs(m3 - m4) < ((tc * 5 + 1) >> 1);
  }
  return dstrong < (beta >> 3) && d < (beta >> 2) && abs(m3 - m4) < ((tc * 5 + 1) >> 1);
}

// xFilteringPandQ (:1323) + xBilinearFilter (:1302). The per-tap coefficients are selected by the side's
// length with compile-time indices (an unrolled loop): local arrays indexed at run time live in scratch.
__device__ __forceinline__ int long_coef(int n, int i) {   // dbCoeffs7/5/3
  constexpr int c7[7] = {59, 50, 41, 32, 23, 14, 5}, c5[5] = {58, 45, 32, 19, 6}, c3[3] = {53, 32, 11};
  return n == 7 ? c7[i] : (n == 5 ? (i < 5 ? c5[i] : 0) : (i < 3 ? c3[i] : 0));
}
__device__ __forceinline__ int long_taper(int n, int i) {   // tc7 / tc3 (length 5 uses tc7)
  constexpr int t7[7] = {6, 5, 4, 3, 2, 1, 1}, t3[3] = {6, 4, 2};
  return n == 3 ? (i < 3 ? t3[i] : 0) : t7[i];
}
__device__ void filter_long(int16_t *src, int o, int nP, int nQ, int tc) {
  int16_t *sP = src - o, *sQ = src;
  const int refP = nP == 7 ? (sP[-6 * o] + sP[-7 * o] + 1) >> 1 : nP == 3 ? (sP[-2 * o] + sP[-3 * o] + 1) >> 1 : (sP[-4 * o] + sP[-5 * o] + 1) >> 1;
  const int refQ = nQ == 7 ? (sQ[6 * o] + sQ[7 * o] + 1) >> 1 : nQ == 3 ? (sQ[2 * o] + sQ[3 * o] + 1) >> 1 : (sQ[4 * o] + sQ[5 * o] + 1) >> 1;
  int mid;
  if (nP == nQ) {
    if (nP == 5)
      mid = (2 * (sP[0] + sQ[0] + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o]) + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] + 8) >> 4;
    else
      mid = (2 * (sP[0] + sQ[0]) + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] +
             sP[-5 * o] + sQ[5 * o] + sP[-6 * o] + sQ[6 * o] + 8) >> 4;
  } else {
    const bool swp = nQ > nP;
    const int16_t *pt = swp ? sQ : sP, *qt = swp ? sP : sQ;
    const int oP = swp ? o : -o, oQ = -oP;
    const int big = swp ? nQ : nP, small = swp ? nP : nQ;
    if (big == 7 && small == 5)
      mid = (2 * (sP[0] + sQ[0] + sP[-o] + sQ[o]) + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] +
             sP[-5 * o] + sQ[5 * o] + 8) >> 4;
    else if (big == 7 && small == 3)
      mid = (2 * (pt[0] + qt[0]) + qt[0] + 2 * (qt[oQ] + qt[2 * oQ]) + pt[oP] + qt[oQ] + pt[2 * oP] + pt[3 * oP] + pt[4 * oP] +
             pt[5 * oP] + pt[6 * oP] + 8) >> 4;
    else
      mid = (sP[0] + sQ[0] + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + 4) >> 3;
  }
  int vp[7], vq[7];
#pragma unroll
  for (int i = 0; i < 7; i++) {
    const int sp = i < nP ? sP[-o * i] : 0, sq = i < nQ ? sQ[o * i] : 0;
    const int cvp = (tc * long_taper(nP, i)) >> 1, cvq = (tc * long_taper(nQ, i)) >> 1;
    const int kp = long_coef(nP, i), kq = long_coef(nQ, i);
    vp[i] = clip3(sp - cvp, sp + cvp, (mid * kp + refP * (64 - kp) + 32) >> 6);
    vq[i] = clip3(sq - cvq, sq + cvq, (mid * kq + refQ * (64 - kq) + 32) >> 6);
  }
#pragma unroll
  for (int i = 0; i < 7; i++) {
    if (i < nP) sP[-o * i] = (int16_t)vp[i];
    if (i < nQ) sQ[o * i] = (int16_t)vq[i];
  }
}

// xPelFilterLuma (:1397)
__device__ void filter_luma_line(int16_t *s, int o, int tc, bool sw, int thrCut, bool fP, bool fQ, int maxv, bool pl, bool ql,
                                 int lenP, int lenQ) {
  const int m4 = s[0], m3 = s[-o], m5 = s[o], m2 = s[-o * 2], m6 = s[o * 2], m1 = s[-o * 3], m7 = s[o * 3], m0 = s[-o * 4];
  if (sw) {
    if (pl || ql) {
      filter_long(s, o, pl ? lenP : 3, ql ? lenQ : 3, tc);
    } else {
      s[-o] = (int16_t)clip3(m3 - 3 * tc, m3 + 3 * tc, (m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - 3 * tc, m4 + 3 * tc, (m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3);
      s[-o * 2] = (int16_t)clip3(m2 - 2 * tc, m2 + 2 * tc, (m1 + m2 + m3 + m4 + 2) >> 2);
      s[o] = (int16_t)clip3(m5 - 2 * tc, m5 + 2 * tc, (m3 + m4 + m5 + m6 + 2) >> 2);
      s[-o * 3] = (int16_t)clip3(m1 - tc, m1 + tc, (2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3);
    }
    return;
  }
  int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
  if (abs(delta) < thrCut) {
    delta = clip3(-tc, tc, delta);
    s[-o] = (int16_t)clip3(0, maxv, m3 + delta);
    s[0] = (int16_t)clip3(0, maxv, m4 - delta);
    const int tc2 = tc >> 1;
    if (fP) s[-o * 2] = (int16_t)clip3(0, maxv, m2 + clip3(-tc2, tc2, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
    if (fQ) s[o] = (int16_t)clip3(0, maxv, m5 + clip3(-tc2, tc2, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
  }
}

// xPelFilterChroma (:1497)
__device__ void filter_chroma_line(int16_t *s, int o, int tc, bool sw, int maxv, bool ctbh) {
  const int m0 = s[-o * 4], m1 = s[-o * 3], m2 = s[-o * 2], m3 = s[-o], m4 = s[0], m5 = s[o], m6 = s[o * 2], m7 = s[o * 3];
  if (sw) {
    if (ctbh) {
      s[-o] = (int16_t)clip3(m3 - tc, m3 + tc, (3 * m2 + 2 * m3 + m4 + m5 + m6 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - tc, m4 + tc, (2 * m2 + m3 + 2 * m4 + m5 + m6 + m7 + 4) >> 3);
      s[o] = (int16_t)clip3(m5 - tc, m5 + tc, (m2 + m3 + m4 + 2 * m5 + m6 + 2 * m7 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 2 * m6 + 3 * m7 + 4) >> 3);
    } else {
      s[-o * 3] = (int16_t)clip3(m1 - tc, m1 + tc, (3 * m0 + 2 * m1 + m2 + m3 + m4 + 4) >> 3);
      s[-o * 2] = (int16_t)clip3(m2 - tc, m2 + tc, (2 * m0 + m1 + 2 * m2 + m3 + m4 + m5 + 4) >> 3);
      s[-o] = (int16_t)clip3(m3 - tc, m3 + tc, (m0 + m1 + m2 + 2 * m3 + m4 + m5 + m6 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - tc, m4 + tc, (m1 + m2 + m3 + 2 * m4 + m5 + m6 + m7 + 4) >> 3);
      s[o] = (int16_t)clip3(m5 - tc, m5 + tc, (m2 + m3 + m4 + 2 * m5 + m6 + 2 * m7 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 2 * m6 + 3 * m7 + 4) >> 3);
    }
    return;
  }
  const int delta = clip3(-tc, tc, ((((m4 - m3) << 2) + m2 - m5 + 4) >> 3));
  s[-o] = (int16_t)clip3(0, maxv, m3 + delta);
  s[0] = (int16_t)clip3(0, maxv, m4 - delta);
}

__device__ __forceinline__ int tc_of(int idx, int bd) {
  const int t = vvcr_tab::dbk_tc[idx];
  return bd < 10 ? (t + 2) >> (10 - bd) : t << (bd - 10);
}

// Four lanes per 4-line luma segment, one line each: the segment decisions (xEdgeFilterLuma :981-1050)
// need lines 0 and 3, whose terms the lanes exchange by shuffles; each lane then filters its own line.
template <int DIR>
__device__ __forceinline__ void dbk_luma(const DbkParams &P, const DbkSeg *segs, int n, int blk) {
  const int t = blk * 256 + threadIdx.x;
  const int i = t >> 2, line = t & 3, l0 = (threadIdx.x & 63) & ~3;   // lane of line 0 of this segment
  const bool valid = i < n;
  const DbkSeg sg = valid ? segs[i] : DbkSeg{0, 0, 0};
  const uint32_t w = sg.w;
  const int bs = w & 3, lenP = (w >> 2) & 7, lenQ = (w >> 5) & 7;
  int qp = (w >> 8) & 63;
  const bool pl = (w >> 14) & 1, ql = (w >> 15) & 1;
  const DPlane &Y = P.pl[0];
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int o = DIR == 0 ? 1 : Y.stride;
  const int step = DIR == 0 ? Y.stride : 1;
  if (P.ladf_num) {
    // luma-adaptive QP offset (LoopFilter::deriveLADFShift :815-840): the mean of p0 and q0 on lines 0 and 3,
    // taken before this segment is filtered; the lanes of lines 0 and 3 hold the terms
    const int16_t *q0 = Y.p + (size_t)(sg.y4 * 4) * Y.stride + sg.x4 * 4 + line * step;
    const int e = valid ? (int)q0[0] + (int)q0[-o] : 0;
    const uint32_t level = (uint32_t)(__shfl(e, l0) + __shfl(e, l0 + 3)) >> 2;
    // the bounds increase strictly, so the reference's loop-until-below is the last interval above
    int sh = P.ladf_qp_offset[0];
#pragma unroll
    for (int k = 1; k < 5; k++)
      if (k < P.ladf_num && level > (uint32_t)P.ladf_lower_bound[k]) sh = P.ladf_qp_offset[k];
    qp += sh;
  }
  const int tc = tc_of(clip3(0, 65, qp + 2 * (bs - 1) + 2 * P.tc_offset_div2), bd);
  const int beta = vvcr_tab::dbk_beta[clip3(0, 63, qp + 2 * P.beta_offset_div2)] * (1 << (bd - 8));
  const int sideThr = (beta + (beta >> 1)) >> 3;
  const int thrCut = tc * 10;
  int16_t *s = Y.p + (size_t)(sg.y4 * 4) * Y.stride + sg.x4 * 4 + line * step;
  // this line's terms (all lanes compute, lines 0 and 3 are used)
  int dp = 0, dq = 0, dpL = 0, dqL = 0;
  if (valid) {
    dp = calc_dp(s, o, false);
    dq = calc_dq(s, o);
    dpL = dp; dqL = dq;
    if (pl) dpL = (dpL + calc_dp(s - 3 * o, o, false) + 1) >> 1;
    if (ql) dqL = (dqL + calc_dq(s + 3 * o, o) + 1) >> 1;
  }
  const int dp0 = __shfl(dp, l0), dq0 = __shfl(dq, l0), dp3 = __shfl(dp, l0 + 3), dq3 = __shfl(dq, l0 + 3);
  const int dp0L = __shfl(dpL, l0), dq0L = __shfl(dqL, l0), dp3L = __shfl(dpL, l0 + 3), dq3L = __shfl(dqL, l0 + 3);
  // long-filter decision
  bool longStrong = false, fPL = false, fQL = false;
  if (pl || ql) {
    const int d0L = dp0L + dq0L, d3L = dp3L + dq3L;
    if (d0L + d3L < beta) {
      fPL = dp0L + dp3L < sideThr;
      fQL = dq0L + dq3L < sideThr;
      const int myd = line == 0 ? d0L : d3L;
      const bool st = valid && (line == 0 || line == 3) && use_strong(s, o, 2 * myd, beta, tc, pl, ql, lenP, lenQ, false);
      longStrong = __shfl((int)st, l0) && __shfl((int)st, l0 + 3);
    }
  }
  // normal / strong short-filter decision
  const int d0 = dp0 + dq0, d3 = dp3 + dq3;
  bool fP = false, fQ = false, sw = false;
  const bool on = !longStrong && d0 + d3 < beta;
  if (!longStrong) {
    if (lenP > 1 && lenQ > 1) { fP = dp0 + dp3 < sideThr; fQ = dq0 + dq3 < sideThr; }
    bool st = false;
    if (on && lenP > 2 && lenQ > 2 && valid && (line == 0 || line == 3))
      st = use_strong(s, o, 2 * (line == 0 ? d0 : d3), beta, tc, false, false, 7, 7, false);
    sw = __shfl((int)st, l0) && __shfl((int)st, l0 + 3);
  }
  if (!valid) return;
  if (longStrong) filter_luma_line(s, o, tc, true, thrCut, fPL, fQL, maxv, pl, ql, lenP, lenQ);
  else if (on) filter_luma_line(s, o, tc, sw, thrCut, fP, fQ, maxv, false, false, 7, 7);
}

// Four lanes per chroma segment: (component, line) = (lane >> 1, lane & 1); the strong-filter decision
// of a component uses both of its lines (xEdgeFilterChroma :1163-1283), exchanged by shuffles.
template <int DIR>
__device__ __forceinline__ void dbk_chroma(const DbkParams &P, const DbkSeg *segs, int n, int blk) {
  const int t = blk * 256 + threadIdx.x;
  const int i = t >> 2, k = (t >> 1) & 1, l = t & 1, lp = (threadIdx.x & 63) & ~1;   // lp: line 0 of this component
  const bool valid = i < n;
  const DbkSeg sg = valid ? segs[i] : DbkSeg{0, 0, 0};
  const uint32_t w = sg.w;
  const bool large = (w >> 4) & 1, ctbh = (w >> 19) & 1;
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int bs = (w >> (2 * k)) & 3;
  const bool act = valid && (bs == 2 || (large && bs == 1));
  const int qp = (int)((w >> (5 + 7 * k)) & 127) - 64;
  const DPlane &C = P.pl[1 + k];
  const int o = DIR == 0 ? 1 : C.stride;
  const int step = DIR == 0 ? C.stride : 1;
  const int tc = tc_of(clip3(0, 65, qp + 2 * (bs - 1) + 2 * P.tc_offset_div2), bd);
  int16_t *s = C.p + (size_t)(sg.y4 * 2) * C.stride + sg.x4 * 2 + l * step;
  int d = 0;
  const int beta = vvcr_tab::dbk_beta[clip3(0, 63, qp + 2 * P.beta_offset_div2)] * (1 << (bd - 8));
  if (act && large) d = calc_dp(s, o, ctbh) + calc_dq(s, o);
  const int dsum = __shfl(d, lp) + __shfl(d, lp + 1);
  bool st = false;
  if (act && large && dsum < beta) st = use_strong(s, o, 2 * d, beta, tc, false, false, 7, 7, ctbh);
  const bool sw = __shfl((int)st, lp) && __shfl((int)st, lp + 1);
  if (act) filter_chroma_line(s, o, tc, sw, maxv, ctbh);
}

// One launch per direction: the first gL workgroups take the luma segments, the others the chroma ones
// (the planes are independent; the vertical launch precedes the horizontal one). The list lengths come from
// device memory (the device planner writes them): each workgroup takes 64 segments per pass and loops
// while segments remain.
template <int DIR>
__global__ __launch_bounds__(256) void k_dbk(DbkParams P, const DbkSeg *segL, const DbkSeg *segC, const int32_t *cnt, int gL) {
  const int nL = cnt[0], nC = cnt[1];
  if ((int)blockIdx.x < gL) {
    for (int b = blockIdx.x; b * 64 < nL; b += gL) dbk_luma<DIR>(P, segL, nL, b);
  } else {
    const int gC = (int)gridDim.x - gL;
    for (int b = (int)blockIdx.x - gL; b * 64 < nC; b += gC) dbk_chroma<DIR>(P, segC, nC, b);
  }
}

}  // namespace

void launch_dbk(const DbkParams &p, const DbkSeg *const segs[2][2], const int32_t *counts, const int g[2][2], hipStream_t s) {
  for (int dir = 0; dir < 2; dir++) {
    const int gL = std::max(1, g[dir][0]), gC = std::max(1, g[dir][1]);
    if (g[dir][0] + g[dir][1] == 0) continue;
    if (dir == 0) hipLaunchKernelGGL(k_dbk<0>, dim3(gL + gC), dim3(256), 0, s, p, segs[0][0], segs[0][1], counts, gL);
    else hipLaunchKernelGGL(k_dbk<1>, dim3(gL + gC), dim3(256), 0, s, p, segs[1][0], segs[1][1], counts + 2, gL);
    VVCR_CHECK_HIP(hipGetLastError());
  }
}
