// vvcr_mc.hip — motion-compensated prediction for gfx950 (k_mc_basic).
//
// One 64-lane wave per McJob (<= 16x16 luma block + its 4:2:0 chroma, one or two lists). The reference
// windows are gathered with 8-byte loads of aligned 4-sample chunks (every active window of the job in
// one phase, all loads in flight before the first LDS write) into LDS; a window that reaches outside the
// picture is gathered per sample with clamped coordinates instead (equivalent to VTM's edge-replicated
// 288-sample margin, Picture::extendPicBorder Picture.cpp:737, plus clipMv Mv.cpp:54: every filter phase
// sums to 64, so a clamped run of equal samples filters to the same value whatever the phase).
//
// Filtering is InterpolationFilter::filter<N,isVertical,isFirst,isLast> (InterpolationFilter.cpp:548-650)
// as the H-then-V pass of xPredInterBlk (InterPrediction.cpp:784-803) for EVERY fraction: a zero fraction
// takes the identity phase {.., 64, ..}, whose intermediate is exact (16 s - 8192 fits int16), and the
// 2-D roundings then equal the copy / H-only / V-only branches (((64 t + off2) >> sh2) == t;
// ((16 X - 2^19) >> 6) == ((X - 2^15) >> 2); (16 X + 2^9) >> 10 == (X + 32) >> 6). One code path, no
// divergence on fractions.
//
// Arithmetic is packed: samples are int16 pairs in LDS dwords and each tap pair is one v_dot2c_i32_i16.
// An output whose first tap sits on an even sample uses the pair-aligned coefficients A = (c0,c1)(c2,c3)..,
// one starting on an odd sample the shifted set B = (0,c0)(c1,c2)..(c_{N-1},0) over the same aligned
// pairs, so every LDS read is an aligned dword. The H pass writes its outputs transposed (column-major,
// vertical pairs packed), so the V pass reads aligned vertical pairs the same way. Results combine like
// AreaBuf::addAvg (Buffer.cpp:447), addWeightedAvg (BCW, Buffer.cpp:350), explicit WP
// (WeightPrediction.cpp:157-378), the GEO blend (InterpolationFilter::xWeightedGeoBlk :997) or the
// uni-prediction rounding, and leave as 8-byte row stores.
#include "vvcr_internal.h"
#include "vvcr_tables.h"
#include "vvcr_mcdev.h"

namespace {

using namespace mcdev;

__constant__ int8_t c_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
__constant__ int8_t c_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
__constant__ int8_t c_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
__constant__ int8_t c_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int8_t c_bcw_w1[5] = VVCR_BCW_W1;
// GEO split geometry (Rom.cpp g_angle2mask / g_Dis / g_angle2mirror, CommonDef.h GEO_* sizes)
__constant__ int8_t c_geo_angle2mask[32] = {0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1, 0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1};
__constant__ int8_t c_geo_dis[32] = {8, 8, 8, 8, 4, 4, 2, 1, 0, -1, -2, -4, -4, -8, -8, -8, -8, -8, -8, -8, -4, -4, -2, -1, 0, 1, 2, 4, 4, 8, 8, 8};
__constant__ int8_t c_geo_angle2mirror[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 2};
__constant__ int8_t c_geo_mask_angle[6] = {0, 2, 3, 4, 5, 8};   // the angle in 0..8 that generated each stored mask
constexpr int GEO_WEIGHT_MASK_SIZE = 224, GEO_MASK_OFFSET = 16;

// Blending weight of one sample: the g_globalGeoWeights entry (Rom.cpp:778-801) that
// InterpolationFilter::xWeightedGeoBlk (InterpolationFilter.cpp:1014-1046) walks to, computed in place.
__device__ __forceinline__ int geo_weight(int angle, int offX, int offY, int lx, int ly) {
  const int mir = c_geo_angle2mirror[angle];
  const int X = mir == 1 ? GEO_WEIGHT_MASK_SIZE - 1 - offX - lx : offX + lx;
  const int Y = mir == 2 ? GEO_WEIGHT_MASK_SIZE - 1 - offY - ly : offY + ly;
  const int b = c_geo_mask_angle[c_geo_angle2mask[angle]];
  const int dX = c_geo_dis[b], dY = c_geo_dis[(b + 8) & 31];
  const int rho = (dX << 8) + (dY << 8);
  const int wIdx = (((X + GEO_MASK_OFFSET) << 1) + 1) * dX + (((Y + GEO_MASK_OFFSET) << 1) + 1) * dY - rho;
  return clampi((32 + wIdx + 4) >> 3, 0, 8);
}

// LDS geometry (int16 samples). Windows hold aligned 4-sample chunks: element e of a row is the sample at
// picture column ax + e, ax = window origin rounded down to a multiple of 4.
constexpr int LP = 28, LR = 24;     // luma window: 7 chunks per row, 23 rows (+1 pad row for the last pair)
constexpr int CP = 16, CR = 12;     // chroma window: 4 chunks, 11 rows (+1)
constexpr int TP = 26, CTP = 14;    // H-pass outputs, column-major: rows per column (even: aligned pairs)

// Combine one sample of the two lists: uni rounding (already final when rnd), WP, GEO blend, BCW, addAvg.
__device__ __forceinline__ int combine(const McParams &P, const McJob &J, int comp, int x, int y, int a, int b) {
  const int cs = comp ? 1 : 0;
  const bool l0 = J.flags & MC_L0, l1 = J.flags & MC_L1, bi = l0 && l1;
  const int bd = P.bd, maxv = (1 << bd) - 1, headRoom = max(2, IF_INTERNAL_PREC - bd);
  if (!bi) {
    if (J.flags & MC_WP) return wp_uni(P.wp, l0 ? 0 : 1, l0 ? (J.ridx & 15) : (J.ridx >> 4), comp, a, headRoom, maxv);
    return a;
  }
  if (J.flags & MC_WP) return wp_bi(P.wp, J.ridx & 15, J.ridx >> 4, comp, a, b, headRoom, maxv);
  if (J.flags & MC_GEO) {
    // xWeightedGeoBlk: (w*p0 + (8-w)*p1 + offset) >> (headRoom + 3)
    const int w = geo_weight(J.aux & 31, (J.aux >> 8) & 255, (J.aux >> 16) & 255, ((J.x >> cs) + x - (J.pu_x >> cs)) << cs,
                             ((J.y >> cs) + y - (J.pu_y >> cs)) << cs);
    const int shiftW = headRoom + 3;
    const int offset = (1 << (shiftW - 1)) + (IF_INTERNAL_OFFS << 3);
    return clampi((w * a + (8 - w) * b + offset) >> shiftW, 0, maxv);
  }
  if (J.bcw != 2) {   // AreaBuf<Pel>::addWeightedAvg (Buffer.cpp:350)
    const int w1 = c_bcw_w1[J.bcw], w0 = 8 - w1;
    const int shiftNum = headRoom + 3;
    const int offset = (1 << (shiftNum - 1)) + (IF_INTERNAL_OFFS << 3);
    return clampi((a * w0 + b * w1 + offset) >> shiftNum, 0, maxv);
  }
  const int shiftNum = headRoom + 1;   // AreaBuf<Pel>::addAvg (Buffer.cpp:447)
  const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
  return clampi((a + b + offset) >> shiftNum, 0, maxv);
}

// window geometry of one (component, list)
struct Win {
  const int16_t *p;
  int stride, pw, ph, ax, oy, s, frac_x, frac_y;
  bool on, inside;
};
__device__ __forceinline__ Win make_win(const McParams &P, const McJob &J, int comp, int l) {
  Win w;
  const int cs = comp ? 1 : 0, N = comp ? 4 : 8, half = N / 2 - 1, fb = 4 + cs;
  w.on = ((J.flags & (l ? MC_L1 : MC_L0)) != 0) && ((J.flags & (comp ? MC_CHROMA : MC_LUMA)) != 0);
  const DPlane &R = P.ref[J.slot[l] < 0 ? 0 : J.slot[l]][comp];
  const int mvx = J.mv[l][0], mvy = J.mv[l][1], mask = (1 << fb) - 1;
  w.frac_x = mvx & mask;
  w.frac_y = mvy & mask;
  const int ox = (J.x >> cs) + (mvx >> fb) - half;
  w.oy = (J.y >> cs) + (mvy >> fb) - half;
  w.s = ox & 3;
  w.ax = ox - w.s;
  const int ww = (J.w >> cs) + N - 1, wh = (J.h >> cs) + N - 1;
  w.p = R.p; w.stride = R.stride; w.pw = R.w; w.ph = R.h;
  w.inside = w.ax >= 0 && ox + ww <= R.w && w.oy >= 0 && w.oy + wh <= R.h;
  return w;
}

// Field-wise select of one of two windows (keeps both in registers; a selected reference would not).
__device__ __forceinline__ Win sel_win(bool second, const Win &a, const Win &b) {
  Win w;
  w.on = second ? b.on : a.on;
  w.inside = second ? b.inside : a.inside;
  w.frac_x = second ? b.frac_x : a.frac_x;
  w.frac_y = second ? b.frac_y : a.frac_y;
  w.oy = second ? b.oy : a.oy;
  w.s = second ? b.s : a.s;
  w.ax = second ? b.ax : a.ax;
  w.p = second ? b.p : a.p;
  w.stride = second ? b.stride : a.stride;
  w.pw = second ? b.pw : a.pw;
  w.ph = second ? b.ph : a.ph;
  return w;
}

// Two waves per job: with both lists, wave l filters list l (luma, then its chroma); with one list,
// wave 0 filters the luma and wave 1 the chroma. Wave 0 stores the luma, wave 1 the chroma.
__global__ __launch_bounds__(128) void k_mc_basic(McParams P, const McJob *__restrict__ jobs, int njobs) {
  __shared__ __attribute__((aligned(16))) int16_t s_lwin[2][LR * LP];   // luma windows per list
  __shared__ __attribute__((aligned(16))) int16_t s_cwin[4][CR * CP];   // chroma windows, combo = 2 * (comp - 1) + list
  __shared__ __attribute__((aligned(16))) int16_t s_lt[2][16 * TP];     // luma H outputs [col][row]
  __shared__ __attribute__((aligned(16))) int16_t s_ct[4][8 * CTP];     // chroma H outputs [col][row]
  __shared__ __attribute__((aligned(16))) int16_t s_lo[2][256];         // luma V outputs per list [y * w + x]
  __shared__ __attribute__((aligned(16))) int16_t s_co[4][64];          // chroma V outputs [y * cw + x]
  __shared__ uint32_t s_ctap[4][2][5];                                   // chroma taps: [combo][H/V][A0 A1 B0 B1 B2]
  const int j = blockIdx.x;
  if (j >= njobs) return;
  const McJob J = jobs[j];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int w = J.w, h = J.h, lw = __ffs(w) - 1;
  const int cw = w >> 1, chh = h >> 1, lcw = lw - 1;
  const bool bi = (J.flags & MC_L0) && (J.flags & MC_L1);
  const int la = (J.flags & MC_L0) ? 0 : 1;   // the list of a uni-predicted block
  const bool rnd = !bi && !(J.flags & MC_KEEP14) && !(J.flags & MC_WP);
  const int bd = P.bd, maxv = (1 << bd) - 1, headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);
  const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
  const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
  // this wave's share: the luma of list ll (if dol) and the chroma of list cl (if doc)
  const int ll = bi ? wave : la, cl = bi ? wave : la;
  const bool dol = (J.flags & MC_LUMA) && (bi || wave == 0), doc = (J.flags & MC_CHROMA) && (bi || wave == 1);

  Win wl[2], wc[4];
#pragma unroll
  for (int l = 0; l < 2; l++) wl[l] = make_win(P, J, 0, l);
#pragma unroll
  for (int k = 0; k < 4; k++) wc[k] = make_win(P, J, 1 + (k >> 1), k & 1);
  bool inside = true;
#pragma unroll
  for (int l = 0; l < 2; l++) inside = inside && (!wl[l].on || wl[l].inside);
#pragma unroll
  for (int k = 0; k < 4; k++) inside = inside && (!wc[k].on || wc[k].inside);
  const Win WL = sel_win(ll, wl[0], wl[1]), WC1 = sel_win(cl, wc[0], wc[1]), WC2 = sel_win(cl, wc[2], wc[3]);

  // chroma taps per combo (lanes 0..7 of wave 0): H from the horizontal fraction, V from the vertical one
  if (tid < 8) {
    const int k = tid >> 1, v = tid & 1;
    // explicit selects: a lane-indexed J.mv[][] would put the job record in scratch
    const int m0 = v ? J.mv[0][1] : J.mv[0][0], m1 = v ? J.mv[1][1] : J.mv[1][0];
    const int mvf = ((k & 1) ? m1 : m0) & 31;
    const Taps<4> t = make_taps<4>(c_chroma[mvf]);
    s_ctap[k][v][0] = t.A[0]; s_ctap[k][v][1] = t.A[1];
    s_ctap[k][v][2] = t.B[0]; s_ctap[k][v][3] = t.B[1]; s_ctap[k][v][4] = t.B[2];
  }

  // ---- gather (each wave its share; all of a lane's loads before its LDS writes)
  int16_t *lwin = s_lwin[ll];
  int16_t *cwin1 = s_cwin[cl], *cwin2 = s_cwin[2 + cl];
  if (inside) {
    uint2 vl[3], vc[2][2];
    if (dol)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int i = lane + 64 * k, r = i / 7, c = i - 7 * r;
        if (r < h + 7) vl[k] = *(const uint2 *)(WL.p + (size_t)(WL.oy + r) * WL.stride + WL.ax + 4 * c);
      }
    if (doc)
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const Win &W = k ? WC2 : WC1;
        const int r = lane >> 2, c = lane & 3;
        if (r < chh + 3) vc[k][0] = *(const uint2 *)(W.p + (size_t)(W.oy + r) * W.stride + W.ax + 4 * c);
      }
    if (dol)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int i = lane + 64 * k, r = i / 7, c = i - 7 * r;
        if (r < h + 7) *(uint2 *)&lwin[r * LP + 4 * c] = vl[k];
      }
    if (doc)
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int r = lane >> 2, c = lane & 3;
        if (r < chh + 3) *(uint2 *)&(k ? cwin2 : cwin1)[r * CP + 4 * c] = vc[k][0];
      }
  } else {
    // a window reaches outside the picture: per-sample gather with clamped coordinates, same layout
    if (dol)
      for (int i = lane; i < (h + 7) * LP; i += 64) {
        const int r = i / LP, e = i - LP * r;
        lwin[i] = WL.p[(size_t)clampi(WL.oy + r, 0, WL.ph - 1) * WL.stride + clampi(WL.ax + e, 0, WL.pw - 1)];
      }
    if (doc)
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const Win &W = k ? WC2 : WC1;
        int16_t *dst = k ? cwin2 : cwin1;
        for (int i = lane; i < (chh + 3) * CP; i += 64) {
          const int r = i / CP, e = i - CP * r;
          dst[i] = W.p[(size_t)clampi(W.oy + r, 0, W.ph - 1) * W.stride + clampi(W.ax + e, 0, W.pw - 1)];
        }
      }
  }
  __syncthreads();

  // ---- H pass: luma (items: 2 rows x 4 columns), then the two chroma combos of the wave's list
  const bool is4x4 = (w == 4 && h == 4);
  const bool alt = (J.flags & MC_ALT_HPEL) != 0;
  if (dol) {
    const int fx = WL.frac_x;
    const Taps<8> th = make_taps<8>((fx == 8 && alt) ? c_alt_hpel : (is4x4 ? c_luma4x4[fx] : c_luma[fx]));
    const int lnq = lw - 2, nrp = (h + 8) >> 1;
    const int rp = lane >> lnq, q = lane & ((1 << lnq) - 1);
    if (rp < nrp) {
      const uint32_t *r0 = (const uint32_t *)lwin + (2 * rp) * (LP / 2) + (WL.s >> 1) + 2 * q;
      uint32_t w0[6], w1[6];
#pragma unroll
      for (int k = 0; k < 6; k++) { w0[k] = r0[k]; w1[k] = r0[LP / 2 + k]; }
      int a[4], b[4];
      if (WL.s & 1) { fir4<8, 1>(w0, th, a); fir4<8, 1>(w1, th, b); }
      else { fir4<8, 0>(w0, th, a); fir4<8, 0>(w1, th, b); }
      uint32_t *dst = (uint32_t *)s_lt[ll];
#pragma unroll
      for (int jj = 0; jj < 4; jj++)
        dst[((4 * q + jj) * TP + 2 * rp) >> 1] = pk((int16_t)((a[jj] + off1) >> sh1), (int16_t)((b[jj] + off1) >> sh1));
    }
  }
  if (doc && lane < 32) {
    const int cc = lane >> 4, it = lane & 15, k = 2 * cc + cl;   // combo: component cc + 1, list cl
    const int lnq = lcw >= 2 ? lcw - 2 : 0, nrp = (chh + 4) >> 1;
    const int rp = it >> lnq, q = it & ((1 << lnq) - 1);
    const int s = cc ? WC2.s : WC1.s;
    if (rp < nrp) {
      Taps<4> t;
      t.A[0] = s_ctap[k][0][0]; t.A[1] = s_ctap[k][0][1];
      t.B[0] = s_ctap[k][0][2]; t.B[1] = s_ctap[k][0][3]; t.B[2] = s_ctap[k][0][4];
      const uint32_t *r0 = (const uint32_t *)s_cwin[k] + (2 * rp) * (CP / 2) + (s >> 1) + 2 * q;
      uint32_t w0[5], w1[5];
#pragma unroll
      for (int m = 0; m < 5; m++) { w0[m] = r0[m]; w1[m] = r0[CP / 2 + m]; }
      int a[4], b[4];
      fir4_var<4>(w0, t, s & 1, a);
      fir4_var<4>(w1, t, s & 1, b);
      uint32_t *dst = (uint32_t *)s_ct[k];
#pragma unroll
      for (int jj = 0; jj < 4; jj++)
        dst[((4 * q + jj) * CTP + 2 * rp) >> 1] = pk((int16_t)((a[jj] + off1) >> sh1), (int16_t)((b[jj] + off1) >> sh1));
    }
  }
  __syncthreads();

  // ---- V pass: items of one column x 4 rows (luma, then the chroma combos of the wave's list)
  if (dol) {
    const int fy = WL.frac_y;
    const Taps<8> tv = make_taps<8>((fy == 8 && alt) ? c_alt_hpel : (is4x4 ? c_luma4x4[fy] : c_luma[fy]));
    const int x = lane & (w - 1), g = lane >> lw;
    if (4 * g < h) {
      const uint32_t *c0 = (const uint32_t *)s_lt[ll] + ((x * TP + 4 * g) >> 1);
      uint32_t wv[6];
#pragma unroll
      for (int k = 0; k < 6; k++) wv[k] = c0[k];
      int o[4];
      fir4<8, 0>(wv, tv, o);
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        int v = (int16_t)((o[jj] + off2) >> sh2);
        if (rnd) v = clampi(v, 0, maxv);
        s_lo[ll][(4 * g + jj) * w + x] = (int16_t)v;
      }
    }
  }
  if (doc && lane < 32) {
    const int cc = lane >> 4, k = 2 * cc + cl, x = lane & 7, g = (lane >> 3) & 1;
    if (x < cw && 4 * g < chh) {
      Taps<4> t;
      t.A[0] = s_ctap[k][1][0]; t.A[1] = s_ctap[k][1][1];
      t.B[0] = s_ctap[k][1][2]; t.B[1] = s_ctap[k][1][3]; t.B[2] = s_ctap[k][1][4];
      const uint32_t *c0 = (const uint32_t *)s_ct[k] + ((x * CTP + 4 * g) >> 1);
      uint32_t wv[4];
#pragma unroll
      for (int m = 0; m < 4; m++) wv[m] = c0[m];
      int o[4];
      fir4<4, 0>(wv, t, o);
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        if (4 * g + jj >= chh) break;
        int v = (int16_t)((o[jj] + off2) >> sh2);
        if (rnd) v = clampi(v, 0, maxv);
        s_co[k][(4 * g + jj) * cw + x] = (int16_t)v;
      }
    }
  }
  __syncthreads();

  // ---- combine and store: 4 (chroma of 4-wide blocks: 2) consecutive samples of a row per lane;
  // wave 0 the luma, wave 1 the chroma
  if (wave == 0 && (J.flags & MC_LUMA)) {
    if (lane * 4 < w * h) {
      const int i = lane * 4, y = i >> lw, x = i & (w - 1);
      const uint2 a = *(const uint2 *)&s_lo[la][i];
      uint2 b = a;
      if (bi) b = *(const uint2 *)&s_lo[1][i];
      int v[4] = {lo16(a.x), hi16(a.x), lo16(a.y), hi16(a.y)};
      const int u[4] = {lo16(b.x), hi16(b.x), lo16(b.y), hi16(b.y)};
      if (!rnd)
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = combine(P, J, 0, x + t, y, v[t], u[t]);
      const DPlane &o = P.out[0];
      *(uint2 *)(o.p + (size_t)(J.y + y) * o.stride + J.x + x) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
    }
  }
  if (wave == 1 && (J.flags & MC_CHROMA)) {
    const int comp = 1 + (lane >> 5), k = lane & 31;
    const int ka = 2 * (comp - 1) + la, kb = 2 * (comp - 1) + 1;
    const DPlane &o = P.out[comp];
    if (cw >= 4) {
      if (k * 4 < cw * chh) {
        const int i = k * 4, y = i >> lcw, x = i & (cw - 1);
        const uint2 a = *(const uint2 *)&s_co[ka][i];
        uint2 b = a;
        if (bi) b = *(const uint2 *)&s_co[kb][i];
        int v[4] = {lo16(a.x), hi16(a.x), lo16(a.y), hi16(a.y)};
        const int u[4] = {lo16(b.x), hi16(b.x), lo16(b.y), hi16(b.y)};
        if (!rnd)
#pragma unroll
          for (int t = 0; t < 4; t++) v[t] = combine(P, J, comp, x + t, y, v[t], u[t]);
        *(uint2 *)(o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
      }
    } else {   // 2-wide chroma (4-wide luma blocks)
      if (k * 2 < cw * chh) {
        const int i = k * 2, y = i >> lcw, x = i & (cw - 1);
        const uint32_t a = *(const uint32_t *)&s_co[ka][i];
        uint32_t b = a;
        if (bi) b = *(const uint32_t *)&s_co[kb][i];
        int v[2] = {lo16(a), hi16(a)};
        const int u[2] = {lo16(b), hi16(b)};
        if (!rnd)
#pragma unroll
          for (int t = 0; t < 2; t++) v[t] = combine(P, J, comp, x + t, y, v[t], u[t]);
        *(uint32_t *)(o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x) = pk(v[0], v[1]);
      }
    }
  }
}

}  // namespace

void launch_mc_basic(const McParams &p, const McJob *jobs, int njobs, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mc_basic, dim3(njobs), dim3(128), 0, s, p, jobs, njobs);
}
