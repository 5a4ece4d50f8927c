// vvcr_mc.hip — motion-compensated prediction for gfx950 (k_mc_basic).
//
// k_mc_basic: two waves per McJob (<= 16x16 luma block + its 4:2:0 chroma, one or two lists); k_mc_tile:
// four waves per 32x32 tile of a PU of at least 32x32. The reference windows are gathered in aligned
// 4- / 8-sample chunks (every window of a wave in one phase, all loads in flight before the first LDS
// write) into LDS, rows clamped to the picture and chunks that cross the left / right picture edge
// loaded per sample with clamped columns (equivalent to VTM's edge-replicated 288-sample margin,
// Picture::extendPicBorder Picture.cpp:737, plus clipMv Mv.cpp:54: every filter phase sums to 64, so a
// clamped run of equal samples filters to the same value whatever the phase).
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

#ifdef VVCR_MC_PROF
// Diagnostics build only: per-workgroup start / end timestamps (s_memrealtime, 100 MHz) of k_mc with the
// workgroup's first job (tools/mc_prof.py).
__device__ unsigned long long g_mcprof[1 << 16][4];
extern "C" int vvcr_mc_prof_read(unsigned long long *dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mcprof), (size_t)n * 4 * 8);
}
#endif

namespace {

using namespace mcdev;

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

// Packed taps (mcdev::make_taps) of every filter phase, built at compile time: a wave's taps are then
// plain scalar loads, not per-job unpacking of the int8 tables.
struct McTapTables {
  Taps<8> l[16], l4[16], alt;
  Taps<4> c[32];
};
constexpr int8_t k_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
constexpr int8_t k_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
constexpr int8_t k_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
constexpr int8_t k_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
constexpr McTapTables make_mc_taps() {
  McTapTables t{};
  for (int f = 0; f < 16; f++) {
    t.l[f] = make_taps<8>(k_luma[f]);
    t.l4[f] = make_taps<8>(k_luma4x4[f]);
  }
  t.alt = make_taps<8>(k_alt_hpel);
  for (int f = 0; f < 32; f++) t.c[f] = make_taps<4>(k_chroma[f]);
  return t;
}
__constant__ McTapTables c_mtaps = make_mc_taps();
// luma taps of a fraction: the 6-tap set of 4x4 blocks (InterpolationFilter::m_lumaFilter4x4), the
// alternative half-sample filter of IMV_HPEL CUs, else the 8-tap set
__device__ __forceinline__ const Taps<8> &luma_taps(int frac, bool alt, bool is4x4) {
  return (frac == 8 && alt) ? c_mtaps.alt : (is4x4 ? c_mtaps.l4[frac] : c_mtaps.l[frac]);
}

// window geometry of one (component, list)
struct Win {
  const int16_t *p;
  int stride, pw, ph, ax, oy, s, frac_x, frac_y;
  bool on;
};
// comp / l may be runtime (wave-uniform) values: the job's per-list fields are picked with selects,
// never indexed (a runtime index into the job record would copy it to scratch)
__device__ __forceinline__ Win make_win(const McParams &P, const McJob &J, int comp, int l) {
  Win w;
  const int cs = comp ? 1 : 0, N = comp ? 4 : 8, half = N / 2 - 1, fb = 4 + cs;
  w.on = ((J.flags & (l ? MC_L1 : MC_L0)) != 0) && ((J.flags & (comp ? MC_CHROMA : MC_LUMA)) != 0);
  const int slot = l ? J.slot[1] : J.slot[0];
  const DPlane &R = P.ref.get(slot < 0 ? 0 : slot, comp);
  const int mvx = l ? J.mv[1][0] : J.mv[0][0], mvy = l ? J.mv[1][1] : J.mv[0][1], mask = (1 << fb) - 1;
  w.frac_x = mvx & mask;
  w.frac_y = mvy & mask;
  const int ox = (J.x >> cs) + (mvx >> fb) - half;
  w.oy = (J.y >> cs) + (mvy >> fb) - half;
  w.s = ox & 3;
  w.ax = ox - w.s;
  w.p = R.p; w.stride = R.stride; w.pw = R.w; w.ph = R.h;
  return w;
}

// The default bi-prediction average (AreaBuf::addAvg, Buffer.cpp:447) when no other combine applies.
__device__ __forceinline__ bool plain_avg(const McJob &J) { return !(J.flags & (MC_WP | MC_GEO)) && J.bcw == 2; }

// Combine-and-store of 4 consecutive samples of one row (2 for 2-wide chroma): the uni rounding is
// already final when rnd; the default average takes the short path; WP / GEO / BCW go through combine().
template <int NS>
__device__ __forceinline__ void combine_store(const McParams &P, const McJob &J, int comp, bool bi, bool rnd, int x, int y,
                                              const int16_t *pa, const int16_t *pb, int16_t *dst) {
  int v[NS], u[NS];
  if (NS == 4) {
    const uint2 a = *(const uint2 *)pa;
    const uint2 b = bi ? *(const uint2 *)pb : a;
    v[0] = lo16(a.x); v[1] = hi16(a.x); v[2 % NS] = lo16(a.y); v[3 % NS] = hi16(a.y);
    u[0] = lo16(b.x); u[1] = hi16(b.x); u[2 % NS] = lo16(b.y); u[3 % NS] = hi16(b.y);
  } else {
    const uint32_t a = *(const uint32_t *)pa;
    const uint32_t b = bi ? *(const uint32_t *)pb : a;
    v[0] = lo16(a); v[1] = hi16(a);
    u[0] = lo16(b); u[1] = hi16(b);
  }
  if (!rnd) {
    if (bi && plain_avg(J)) {
      const int headRoom = max(2, IF_INTERNAL_PREC - P.bd), shiftNum = headRoom + 1;
      const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS, maxv = (1 << P.bd) - 1;
#pragma unroll
      for (int t = 0; t < NS; t++) v[t] = clampi((v[t] + u[t] + offset) >> shiftNum, 0, maxv);
    } else {
#pragma unroll
      for (int t = 0; t < NS; t++) v[t] = combine(P, J, comp, x + t, y, v[t], u[t]);
    }
  }
  if (NS == 4) *(uint2 *)dst = make_uint2(pk(v[0], v[1]), pk(v[2 % NS], v[3 % NS]));
  else *(uint32_t *)dst = pk(v[0], v[1]);
}

// Two waves per job: with both lists, wave l filters list l (luma, then its chroma); with one list,
// wave 0 filters the luma and wave 1 the chroma. Wave 0 stores the luma, wave 1 the chroma.
struct BasicLds {
  alignas(16) int16_t lwin[2][LR * LP];   // luma windows per list
  alignas(16) int16_t cwin[4][CR * CP];   // chroma windows, combo = 2 * (comp - 1) + list
  alignas(16) int16_t lt[2][16 * TP];     // luma H outputs [col][row]
  alignas(16) int16_t ct[4][8 * CTP];     // chroma H outputs [col][row]
  alignas(16) int16_t lo[2][256];         // luma V outputs per list [y * w + x]
  alignas(16) int16_t co[4][64];          // chroma V outputs [y * cw + x]
};

// One job on 128 lanes (tid 0..127) with LDS L; the caller's workgroup runs two jobs, so every
// __syncthreads here is reached the same number of times by both (three, unconditionally).
__device__ __forceinline__ void mc_basic(const McParams &P, const McJob *__restrict__ jobs, int njobs, int j, int tid, BasicLds &L) {
  auto &s_lwin = L.lwin;
  auto &s_cwin = L.cwin;
  auto &s_lt = L.lt;
  auto &s_ct = L.ct;
  auto &s_lo = L.lo;
  auto &s_co = L.co;
  if (j >= njobs) return;
  const McJob J = load_uniform(jobs + j);
  // readfirstlane: the wave index is uniform, and everything derived from it (list, component, window,
  // taps) then stays in SGPRs instead of being computed per lane
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
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
  const int ll = bi ? wave : la, cl = ll;
  const bool dol = (J.flags & MC_LUMA) && (bi || wave == 0), doc = (J.flags & MC_CHROMA) && (bi || wave == 1);
  const Win WL = make_win(P, J, 0, ll), WC1 = make_win(P, J, 1, cl), WC2 = make_win(P, J, 2, cl);
  // Cb and Cr of one list share the MV, hence the taps
  const Taps<4> &tcH = c_mtaps.c[WC1.frac_x], &tcV = c_mtaps.c[WC1.frac_y];

  // ---- gather (each wave its share; all of a lane's loads before its LDS writes), 4-sample chunks
  int16_t *lwin = s_lwin[ll];
  int16_t *cwin1 = s_cwin[cl], *cwin2 = s_cwin[2 + cl];
  {
    uint2 vl0 = {}, vl1 = {}, vl2 = {}, vc0 = {}, vc1 = {};
    auto lch = [&](int k) {   // luma chunk k of this lane (index clamped: every lane loads)
      const int i = min(lane + 64 * k, (h + 7) * 7 - 1), r = i / 7, c = i - 7 * r;
      return chunk4(WL.p, WL.stride, WL.pw, WL.ph, WL.oy + r, WL.ax + 4 * c);
    };
    auto cch = [&](const Win &W) {
      const int i = min(lane, (chh + 3) * 4 - 1), r = i >> 2, c = i & 3;
      return chunk4(W.p, W.stride, W.pw, W.ph, W.oy + r, W.ax + 4 * c);
    };
    if (dol) { vl0 = lch(0); vl1 = lch(1); vl2 = lch(2); }
    if (doc) { vc0 = cch(WC1); vc1 = cch(WC2); }
    if (dol) {
      auto put = [&](int k, uint2 v) {
        const int i = lane + 64 * k, r = i / 7, c = i - 7 * r;
        if (r < h + 7) *(uint2 *)&lwin[r * LP + 4 * c] = v;
      };
      put(0, vl0); put(1, vl1); put(2, vl2);
    }
    if (doc && (lane >> 2) < chh + 3) {
      const int r = lane >> 2, c = lane & 3;
      *(uint2 *)&cwin1[r * CP + 4 * c] = vc0;
      *(uint2 *)&cwin2[r * CP + 4 * c] = vc1;
    }
  }
  __syncthreads();

  // ---- H pass: luma (items: 2 rows x 4 columns), then the two chroma combos of the wave's list
  const bool is4x4 = (w == 4 && h == 4);
  const bool alt = (J.flags & MC_ALT_HPEL) != 0;
  if (dol) {
    const Taps<8> &th = luma_taps(WL.frac_x, alt, is4x4);
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
      const uint32_t *r0 = (const uint32_t *)s_cwin[k] + (2 * rp) * (CP / 2) + (s >> 1) + 2 * q;
      uint32_t w0[5], w1[5];
#pragma unroll
      for (int m = 0; m < 5; m++) { w0[m] = r0[m]; w1[m] = r0[CP / 2 + m]; }
      int a[4], b[4];
      fir4_var<4>(w0, tcH, s & 1, a);
      fir4_var<4>(w1, tcH, s & 1, b);
      uint32_t *dst = (uint32_t *)s_ct[k];
#pragma unroll
      for (int jj = 0; jj < 4; jj++)
        dst[((4 * q + jj) * CTP + 2 * rp) >> 1] = pk((int16_t)((a[jj] + off1) >> sh1), (int16_t)((b[jj] + off1) >> sh1));
    }
  }
  __syncthreads();

  // ---- V pass: items of one column x 4 rows (luma, then the chroma combos of the wave's list)
  if (dol) {
    const Taps<8> &tv = luma_taps(WL.frac_y, alt, is4x4);
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
      const uint32_t *c0 = (const uint32_t *)s_ct[k] + ((x * CTP + 4 * g) >> 1);
      uint32_t wv[4];
#pragma unroll
      for (int m = 0; m < 4; m++) wv[m] = c0[m];
      int o[4];
      fir4<4, 0>(wv, tcV, o);
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
      const DPlane &o = P.out[0];
      combine_store<4>(P, J, 0, bi, rnd, x, y, &s_lo[la][i], &s_lo[1][i], o.p + (size_t)(J.y + y) * o.stride + J.x + x);
    }
  }
  if (wave == 1 && (J.flags & MC_CHROMA)) {
    const int comp = 1 + (lane >> 5), k = lane & 31;
    const int ka = 2 * (comp - 1) + la, kb = 2 * (comp - 1) + 1;
    const DPlane &o = P.out[comp];
    if (cw >= 4) {
      if (k * 4 < cw * chh) {
        const int i = k * 4, y = i >> lcw, x = i & (cw - 1);
        combine_store<4>(P, J, comp, bi, rnd, x, y, &s_co[ka][i], &s_co[kb][i], o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x);
      }
    } else {   // 2-wide chroma (4-wide luma blocks)
      if (k * 2 < cw * chh) {
        const int i = k * 2, y = i >> lcw, x = i & (cw - 1);
        combine_store<2>(P, J, comp, bi, rnd, x, y, &s_co[ka][i], &s_co[kb][i], o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_mc_tile: 32x32 luma tiles (+ 16x16 chroma) of PUs of at least 32x32, four waves per tile. The same
// arithmetic as k_mc_basic; a larger tile shares the window halo and the per-job set-up among 4x the
// samples. Every wave owns one luma window (list) and one chroma window (component, list) for all
// passes, so its set-up is scalar and computed once:
//   bi   luma list l on waves {2l, 2l+1}; chroma (comp, list) = (wave >> 1, wave & 1)
//   uni  luma on all waves (gather / H) and waves 0, 1 (V); chroma Cb / Cr on waves 2 / 3
//   gather   16-byte chunks of 8 aligned samples
//   H pass   luma items of 2 rows x 4 columns; chroma items of 2 rows x 4 columns
//   V pass   luma items of 1 column x 8 rows; chroma 1 column x 4 rows
//   combine  all 256 lanes, 4 luma samples each; lanes 0..127 4 chroma samples each
// ------------------------------------------------------------------------------------------------
constexpr int TL_LP = 48, TL_LR = 40;    // luma window: 6 chunks of 8 per row, 39 rows (+1 pad)
constexpr int TL_CP = 32, TL_CR = 20;    // chroma window: 4 chunks, 19 rows (+1 pad)
constexpr int TL_TP = 42, TL_CTP = 22;   // H outputs, column-major: rows per column (odd dword pitch)
constexpr int TL_LWIN = TL_LR * TL_LP, TL_CWIN = TL_CR * TL_CP;

struct TileLds {
  alignas(16) int16_t win[2 * TL_LWIN + 4 * TL_CWIN];   // windows, then (after the H pass) the V outputs
  alignas(16) int16_t lt[2][32 * TL_TP];                // luma H outputs [col][row]
  alignas(16) int16_t ct[4][16 * TL_CTP];               // chroma H outputs [col][row]
};

__device__ __forceinline__ void mc_tile(const McParams &P, const McJob *__restrict__ jobs, int njobs, int j, TileLds &L) {
  auto &s_win = L.win;
  auto &s_lt = L.lt;
  auto &s_ct = L.ct;
  int16_t *const s_lwin = s_win, *const s_cwin = s_win + 2 * TL_LWIN;
  int16_t *const s_lo = s_win;                    // luma V outputs [list][y * 32 + x]
  int16_t *const s_co = s_win + 2 * TL_LWIN;      // chroma V outputs [combo][y * 16 + x]
  if (j >= njobs) return;
  const McJob J = load_uniform(jobs + j);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool bi = (J.flags & MC_L0) && (J.flags & MC_L1);
  const int la = (J.flags & MC_L0) ? 0 : 1;
  const bool rnd = !bi && !(J.flags & MC_KEEP14) && !(J.flags & MC_WP);
  const int bd = P.bd, maxv = (1 << bd) - 1, headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);
  const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
  const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
  const bool alt = (J.flags & MC_ALT_HPEL) != 0;
  const bool doL = (J.flags & MC_LUMA) != 0, doC = (J.flags & MC_CHROMA) != 0;

  // this wave's luma list and lanes, and its chroma window
  const int ll = bi ? (wave >> 1) : la;
  const int lidx = bi ? (tid & 127) : tid, lstep = bi ? 128 : 256;
  const bool chw = doC && (bi || wave >= 2);
  const int ccomp = bi ? (wave >> 1) : (wave & 1);   // 0 = Cb, 1 = Cr
  const int clist = bi ? (wave & 1) : la;
  const int combo = 2 * ccomp + clist;
  const Win WL = make_win(P, J, 0, ll);
  const Win WC = make_win(P, J, 1 + ccomp, clist);
  // 16-byte chunks: the window origins rounded down to a multiple of 8 samples
  const int lax = WL.ax & ~7, lsh = WL.ax - lax + WL.s;   // first tap column within the LDS row
  const int cax = WC.ax & ~7, csh = WC.ax - cax + WC.s;
  int16_t *lwin = s_lwin + ll * TL_LWIN;
  int16_t *cwin = s_cwin + combo * TL_CWIN;

  // ---- gather (clamped indices: every lane loads, no branch around the loads)
  {
    auto lsrc = [&](int k) {
      const int i = min(lidx + lstep * k, 39 * 6 - 1), r = i / 6, c = i - 6 * r;
      return chunk8(WL.p, WL.stride, WL.pw, WL.ph, WL.oy + r, lax + 8 * c);
    };
    auto ldst = [&](int k) {
      const int i = lidx + lstep * k, r = i / 6, c = i - 6 * r;
      return (uint4 *)&lwin[r * TL_LP + 8 * c];
    };
    auto csrc = [&](int k) {
      const int i = min(lane + 64 * k, 19 * 4 - 1), r = i >> 2, c = i & 3;
      return chunk8(WC.p, WC.stride, WC.pw, WC.ph, WC.oy + r, cax + 8 * c);
    };
    auto cdst = [&](int k) {
      const int i = lane + 64 * k, r = i >> 2, c = i & 3;
      return (uint4 *)&cwin[r * TL_CP + 8 * c];
    };
    uint4 vl0 = {}, vl1 = {}, vc0 = {}, vc1 = {};
    if (doL) { vl0 = lsrc(0); vl1 = lsrc(1); }
    if (chw) { vc0 = csrc(0); vc1 = csrc(1); }
    if (doL) {
      if (lidx < 39 * 6) *ldst(0) = vl0;
      if (lidx + lstep < 39 * 6) *ldst(1) = vl1;
    }
    if (chw) {
      if (lane < 19 * 4) *cdst(0) = vc0;
      if (lane + 64 < 19 * 4) *cdst(1) = vc1;
    }
  }
  __syncthreads();

  // ---- H pass
  // luma items: row pair rp (0..19) x 8-column segment g (0..3), 80 per list, spread over the list's waves
  const int hl_n = bi ? 40 : 20, hl_i = lane + hl_n * (bi ? (wave & 1) : wave);
  if (doL && lane < hl_n) {
    const Taps<8> &th = luma_taps(WL.frac_x, alt, false);
    const int rp = hl_i >> 2, g = hl_i & 3;
    const uint32_t *r0 = (const uint32_t *)lwin + (2 * rp) * (TL_LP / 2) + (lsh >> 1) + 4 * g;
    uint32_t w0[8], w1[8];
#pragma unroll
    for (int m = 0; m < 8; m++) { w0[m] = r0[m]; w1[m] = r0[TL_LP / 2 + m]; }
    int a[8], b[8];
    {
      int a0[4], a1[4], b0[4], b1[4];
      if (lsh & 1) { fir4<8, 1>(w0, th, a0); fir4<8, 1>(w0 + 2, th, a1); fir4<8, 1>(w1, th, b0); fir4<8, 1>(w1 + 2, th, b1); }
      else { fir4<8, 0>(w0, th, a0); fir4<8, 0>(w0 + 2, th, a1); fir4<8, 0>(w1, th, b0); fir4<8, 0>(w1 + 2, th, b1); }
#pragma unroll
      for (int m = 0; m < 4; m++) { a[m] = a0[m]; a[4 + m] = a1[m]; b[m] = b0[m]; b[4 + m] = b1[m]; }
    }
    uint32_t *dst = (uint32_t *)s_lt[ll] + ((8 * g * TL_TP + 2 * rp) >> 1);
#pragma unroll
    for (int jj = 0; jj < 8; jj++) dst[jj * (TL_TP / 2)] = pack_h(a[jj], b[jj], sh1);
  }
  if (chw && lane < 40) {   // item: row pair rp (0..9) x quad q (0..3)
    const Taps<4> &t = c_mtaps.c[WC.frac_x];
    const int rp = lane >> 2, q = lane & 3;
    const uint32_t *r0 = (const uint32_t *)cwin + (2 * rp) * (TL_CP / 2) + (csh >> 1) + 2 * q;
    uint32_t w0[5], w1[5];
#pragma unroll
    for (int m = 0; m < 5; m++) { w0[m] = r0[m]; w1[m] = r0[TL_CP / 2 + m]; }
    int a[4], b[4];
    if (csh & 1) { fir4<4, 1>(w0, t, a); fir4<4, 1>(w1, t, b); }
    else { fir4<4, 0>(w0, t, a); fir4<4, 0>(w1, t, b); }
    uint32_t *dst = (uint32_t *)s_ct[combo] + ((4 * q * TL_CTP + 2 * rp) >> 1);
#pragma unroll
    for (int jj = 0; jj < 4; jj++) dst[jj * (TL_CTP / 2)] = pack_h(a[jj], b[jj], sh1);
  }
  __syncthreads();

  // ---- V pass (outputs over the windows, which nobody reads any more)
  if (doL && (bi || wave < 2)) {
    const Taps<8> &tv = luma_taps(WL.frac_y, alt, false);
    const int i = tid & 127, x = i & 31, g = i >> 5;   // column x, rows 8g .. 8g+7
    const uint32_t *c0 = (const uint32_t *)s_lt[ll] + ((x * TL_TP + 8 * g) >> 1);
    uint32_t wv[8];
#pragma unroll
    for (int m = 0; m < 8; m++) wv[m] = c0[m];
    int o0[4], o1[4];
    fir4<8, 0>(wv, tv, o0);
    fir4<8, 0>(wv + 2, tv, o1);
    int16_t *dst = s_lo + ll * 1024 + 8 * g * 32 + x;
#pragma unroll
    for (int m = 0; m < 8; m++) {
      int v = (int16_t)(((m < 4 ? o0[m & 3] : o1[m & 3]) + off2) >> sh2);
      if (rnd) v = clampi(v, 0, maxv);
      dst[m * 32] = (int16_t)v;
    }
  }
  if (chw) {
    const Taps<4> &t = c_mtaps.c[WC.frac_y];
    const int x = lane & 15, g = lane >> 4;   // column x, rows 4g .. 4g+3
    const uint32_t *c0 = (const uint32_t *)s_ct[combo] + ((x * TL_CTP + 4 * g) >> 1);
    uint32_t wv[4];
#pragma unroll
    for (int m = 0; m < 4; m++) wv[m] = c0[m];
    int o[4];
    fir4<4, 0>(wv, t, o);
    int16_t *dst = s_co + combo * 256 + 4 * g * 16 + x;
#pragma unroll
    for (int m = 0; m < 4; m++) {
      int v = (int16_t)((o[m] + off2) >> sh2);
      if (rnd) v = clampi(v, 0, maxv);
      dst[m * 16] = (int16_t)v;
    }
  }
  __syncthreads();

  // ---- combine and store (8-byte row stores)
  if (doL) {
    const int i = tid * 4, y = i >> 5, x = i & 31;
    const DPlane &o = P.out[0];
    combine_store<4>(P, J, 0, bi, rnd, x, y, &s_lo[la * 1024 + i], &s_lo[1024 + i], o.p + (size_t)(J.y + y) * o.stride + J.x + x);
  }
  if (doC && wave < 2) {
    const int comp = 1 + wave, i = lane * 4, y = i >> 4, x = i & 15;
    const int ka = 2 * (comp - 1) + la, kb = 2 * (comp - 1) + 1;
    const DPlane &o = P.out[comp];
    combine_store<4>(P, J, comp, bi, rnd, x, y, &s_co[ka * 256 + i], &s_co[kb * 256 + i],
                     o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x);
  }
}

// One launch for the plain MC of a picture: the first ntile workgroups take a 32x32 tile each, the
// others two <= 16x16 jobs (128 lanes each); both layouts share one LDS allocation.
constexpr int MC_LDS = sizeof(TileLds) > 2 * sizeof(BasicLds) ? sizeof(TileLds) : 2 * sizeof(BasicLds);
__global__ __launch_bounds__(256) void k_mc(McParams P, const McJob *__restrict__ jobs, int ntile, int nbasic) {
  __shared__ __attribute__((aligned(16))) char raw[MC_LDS];
  // XCD-aware order (measured on the 4K B pictures in isolation, interleaved A/B: 22.4 -> 18.9 us; the same
  // order made k_alf 0.30 -> 0.52 ms per step, its luma / chroma mix then unbalanced across XCDs, and
  // k_mc_affine 2 % slower: both keep the dispatcher's round-robin order)
  const int b = xcd_swizzle(blockIdx.x, gridDim.x);
#ifdef VVCR_MC_PROF
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  struct Stamp {
    unsigned long long t0;
    int b;
    const McJob *j;
    __device__ ~Stamp() {
      __syncthreads();
      if (threadIdx.x == 0 && b < (1 << 16)) {
        unsigned int xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_mcprof[b][0] = t0;
        g_mcprof[b][1] = __builtin_amdgcn_s_memrealtime();
        g_mcprof[b][2] = (unsigned long long)(uint16_t)j->x | (unsigned long long)(uint16_t)j->y << 16 |
                         (unsigned long long)j->w << 32 | (unsigned long long)j->h << 40 | (unsigned long long)(xcc & 15) << 48;
        g_mcprof[b][3] = (unsigned long long)j->flags;
      }
    }
  } stamp{t_start, b, jobs + (b < ntile ? b : ntile + 2 * (b - ntile))};
#endif
  if (b < ntile) {
    mc_tile(P, jobs, ntile, b, *reinterpret_cast<TileLds *>(raw));
  } else {
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
    mc_basic(P, jobs + ntile, nbasic, 2 * (b - ntile) + half, threadIdx.x & 127,
             *reinterpret_cast<BasicLds *>(raw + half * sizeof(BasicLds)));
  }
}

}  // namespace

void launch_mc(const McParams &p, const McJob *jobs, int ntile, int nbasic, hipStream_t s) {
  const int g = ntile + (nbasic + 1) / 2;
  if (g > 0) hipLaunchKernelGGL(k_mc, dim3(g), dim3(256), 0, s, p, jobs, ntile, nbasic);
}
