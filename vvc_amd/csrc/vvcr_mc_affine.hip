// vvcr_mc_affine.hip — affine motion compensation with PROF for gfx950 (k_mc_affine).
//
// Two waves (128 lanes) per <= 16x16 luma tile of an affine PU, two tiles per workgroup (InterPrediction::xPredAffineBlk,
// InterPrediction.cpp:890-1272): 4x4 luma sub-block MVs from the control-point model, the 6-tap
// m_lumaFilter4x4 (InterpolationFilter.cpp:57), PROF gradient correction (applyPROFCore Buffer.cpp:45),
// 4x4 chroma sub-blocks with the mean MV of two luma sub-blocks, then the bi / BCW / WP combine.
//
// Reference samples: the 11x11 windows of the sub-blocks overlap almost completely (neighbouring affine
// sub-block MVs differ by a fraction of a sample), so per list the tile gathers the UNION of its
// sub-block windows once — whole aligned 4-sample chunks, one 8-byte load per lane per chunk — and each
// sub-block filters from its offset inside that union (a 16x16 tile: ~24x24 samples instead of
// 16 x 121). A tile whose union does not fit the buffer (strongly diverging MVs) gathers every
// sub-block window on its own (per-sample); one that reaches outside the picture gathers per sample
// with clamped coordinates (= the reference's edge-extended margin, Picture::extendPicBorder).
//
// Filtering is the separable H-then-V form for every fraction (identity phase for zero fractions; see
// vvcr_mc.hip), with packed int16 pairs and v_dot2c (vvcr_mcdev.h): lanes hold different sub-blocks, so
// taps come from LDS tables indexed by each lane's fraction and the pair parity is per lane (fir4_var).
#include "vvcr_internal.h"
#include "vvcr_tables.h"
#include "vvcr_mcdev.h"

namespace {

using namespace mcdev;

constexpr int8_t kLuma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
constexpr int8_t kChroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int8_t a_bcw_w1[5] = VVCR_BCW_W1;

// packed taps: luma 6-tap (taps 1..6 of m_lumaFilter4x4) A0..A2 B0..B3; chroma A0 A1 B0 B1 B2 (8 dwords a row)
struct TapTables {
  uint32_t l[16][8];
  uint32_t c[32][8];
};
constexpr TapTables make_tables() {
  TapTables t{};
  for (int f = 0; f < 16; f++) {
    const Taps<6> a = make_taps<6>(&kLuma4x4[f][1]);
    for (int k = 0; k < 3; k++) t.l[f][k] = a.A[k];
    for (int k = 0; k < 4; k++) t.l[f][3 + k] = a.B[k];
  }
  for (int f = 0; f < 32; f++) {
    const Taps<4> a = make_taps<4>(kChroma[f]);
    for (int k = 0; k < 2; k++) t.c[f][k] = a.A[k];
    for (int k = 0; k < 3; k++) t.c[f][2 + k] = a.B[k];
  }
  return t;
}
__constant__ TapTables a_taps = make_tables();

__device__ __forceinline__ void round_affine(int &x, int &y, int s) {   // roundAffineMv (Mv.cpp:47)
  const int o = 1 << (s - 1);
  x = (x + o - (x >= 0)) >> s;
  y = (y + o - (y >= 0)) >> s;
}

// LDS geometry (int16 samples)
constexpr int LUP = 48, LUR = 44, LWS = LUP * LUR;   // luma union window per list: 12 chunks x 44 rows
constexpr int LSBP = 12, LSBS = 11 * LSBP;            // fallback: per sub-block 11 rows x 12
constexpr int CUP = 32, CUR = 17, CWS = CUP * CUR;    // chroma union per (component, list): 8 chunks x 16 rows (+1 pad row)
constexpr int CSBP = 8, CSBS = 7 * CSBP;              // fallback: per chroma sub-block 7 rows x 8
constexpr int HTC = 10, HTS = 4 * HTC;                // luma H outputs [sub-block][col][10 rows]
constexpr int CTC = 8, CTS = 4 * CTC;                 // chroma H outputs [sub-block][col][8 rows]
static_assert(16 * LSBS <= LWS && 4 * CSBS <= CWS, "fallback windows fit the union buffers");

// Where the window of a sub-block lies in its list's buffer: element (r, e) of the window (row r, column
// e, relative to the window's top-left tap) is buf[base + (ey + r) * pitch + ex + e].
struct Place {
  int base, pitch, ex, ey;
};

struct AffLds {
  alignas(16) int16_t lw[2][LWS];
  alignas(16) int16_t cw[4][CWS];       // combo k = 2 * (comp - 1) + list
  alignas(16) int16_t ht[2][16 * HTS];
  alignas(16) int16_t ct[4][4 * CTS];
  alignas(16) uint32_t tl[16][8];
  alignas(16) uint32_t tc[32][8];
  int sbmv[2][16][2];     // MC MV of each luma sub-block (clamped)
  int stmv[2][16][2];     // stored MV (before the picture clamp) for chroma
  int csmv[2][4][2];      // chroma sub-block MVs
  int box[2][2][4];       // union boxes: [luma / chroma][list][x0 x1 y0 y1]
};

// One job on 128 lanes (lane 0..127) with LDS L; the workgroup runs two jobs, so every __syncthreads
// here is reached unconditionally (the same number of times by both).
__device__ __forceinline__ void mc_affine(const McParams &P, const AffJob *__restrict__ jobs, int njobs, const AffPu *__restrict__ pus,
                                          int j, int lane, AffLds &L) {
  auto &s_lw = L.lw;
  auto &s_cw = L.cw;
  auto &s_ht = L.ht;
  auto &s_ct = L.ct;
  auto &s_tl = L.tl;
  auto &s_tc = L.tc;
  auto &s_sbmv = L.sbmv;
  auto &s_stmv = L.stmv;
  auto &s_csmv = L.csmv;
  auto &s_box = L.box;
  // after the H passes the chroma windows are dead: chroma predictions [combo][y * 8 + x] and the luma
  // prediction per list [y * 16 + x] live there
  int16_t(*s_co)[64] = (int16_t(*)[64])s_cw[0];
  int16_t(*s_lo)[256] = (int16_t(*)[256])s_cw[1];

  if (j >= njobs) return;
  const AffJob J = jobs[j];
  const AffPu U = pus[J.pu];
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const bool bi = U.l[0].present && U.l[1].present;
  // per-list flags as scalars: a lane-indexed U.l[l] would copy the PU record to scratch
  const bool pres[2] = {U.l[0].present != 0, U.l[1].present != 0}, prof[2] = {U.l[0].prof != 0, U.l[1].prof != 0};
  auto PRES = [&](int l) { return l ? pres[1] : pres[0]; };
  const int w = J.w, h = J.h;           // 8 or 16 (affine PUs are >= 8x8, tiled by 16)
  const int lnsx = w == 16 ? 2 : 1, nsx = 1 << lnsx, nsb = (w >> 2) * (h >> 2);
  const int cw = w >> 1, chh = h >> 1, ncx = cw >> 2, ncb = (cw >> 2) * (chh >> 2);
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);

  // packed tap tables (global, L2-resident) -> LDS
  (&s_tl[0][0])[lane] = (&a_taps.l[0][0])[lane];
#pragma unroll
  for (int k = 0; k < 2; k++) (&s_tc[0][0])[lane + 128 * k] = (&a_taps.c[0][0])[lane + 128 * k];

  // ---- sub-block MVs of both lists (:1102-1140); MV clamp of xPredAffineBlk (:936-939), relative to the PU
  const int iHorMax = (P.pic_w + 8 - U.x - 1) << 4, iHorMin = (-P.ctu - 8 - U.x + 1) << 4;
  const int iVerMax = (P.pic_h + 8 - U.y - 1) << 4, iVerMin = (-P.ctu - 8 - U.y + 1) << 4;
  const int MVLIM = (1 << 17) - 1;
  int bx0 = 1 << 30, bx1 = -(1 << 30), by0 = 1 << 30, by1 = -(1 << 30);   // window box of this lane's sub-block
  if (lane < 32) {
    const int l = lane >> 4, sb = lane & 15;
    const AffList &A = pus[J.pu].l[l];      // lane-dependent list: read from global (a local copy would go to scratch)
    if (A.present && sb < nsb) {
      const int sw = (J.x - U.x) + (sb & (nsx - 1)) * 4, shh = (J.y - U.y) + (sb >> lnsx) * 4;
      int mx, my;
      if (!A.spread) {
        mx = A.mvx + A.dhx * (2 + sw) + A.dvx * (2 + shh);
        my = A.mvy + A.dhy * (2 + sw) + A.dvy * (2 + shh);
      } else {
        mx = A.mvx + A.dhx * (U.w >> 1) + A.dvx * (U.h >> 1);
        my = A.mvy + A.dhy * (U.w >> 1) + A.dvy * (U.h >> 1);
      }
      round_affine(mx, my, 7);
      mx = clampi(mx, -MVLIM - 1, MVLIM);
      my = clampi(my, -MVLIM - 1, MVLIM);
      s_stmv[l][sb][0] = mx; s_stmv[l][sb][1] = my;
      const int cmx = clampi(mx, iHorMin, iHorMax), cmy = clampi(my, iVerMin, iVerMax);
      s_sbmv[l][sb][0] = cmx;
      s_sbmv[l][sb][1] = cmy;
      bx0 = J.x + (sb & (nsx - 1)) * 4 + (cmx >> 4) - 3;
      by0 = J.y + (sb >> lnsx) * 4 + (cmy >> 4) - 3;
      bx1 = bx0 + 11;
      by1 = by0 + 11;
    }
  }
  // union box per list: min / max over the 16 lanes of the list (xor shuffles stay inside the group)
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) {
    bx0 = min(bx0, __shfl_xor(bx0, m)); bx1 = max(bx1, __shfl_xor(bx1, m));
    by0 = min(by0, __shfl_xor(by0, m)); by1 = max(by1, __shfl_xor(by1, m));
  }
  if (lane == 0 || lane == 16) {   // wave 0 holds the MV lanes; the box reaches the other wave through LDS
    s_box[0][lane >> 4][0] = bx0; s_box[0][lane >> 4][1] = bx1;
    s_box[0][lane >> 4][2] = by0; s_box[0][lane >> 4][3] = by1;
  }
  __syncthreads();
  // chroma: 4x4 sub-blocks, MV = mean of two luma sub-block MVs (:1142-1160)
  int cx0 = 1 << 30, cx1 = -(1 << 30), cy0 = 1 << 30, cy1 = -(1 << 30);
  if (lane < 8) {
    const int l = lane >> 2, cb = lane & 3;
    if (pus[J.pu].l[l].present && cb < ncb) {
      const int cxs = (cb % ncx) * 2, cys = (cb / ncx) * 2;   // luma sub-block indices in the tile
      const int a = cys * nsx + cxs, b = (cys + 1) * nsx + cxs + 1;
      int mx = s_stmv[l][a][0] + s_stmv[l][b][0], my = s_stmv[l][a][1] + s_stmv[l][b][1];
      round_affine(mx, my, 1);
      const int cmx = clampi(mx, iHorMin, iHorMax), cmy = clampi(my, iVerMin, iVerMax);
      s_csmv[l][cb][0] = cmx;
      s_csmv[l][cb][1] = cmy;
      cx0 = (J.x >> 1) + (cb % ncx) * 4 + (cmx >> 5) - 1;
      cy0 = (J.y >> 1) + (cb / ncx) * 4 + (cmy >> 5) - 1;
      cx1 = cx0 + 7;
      cy1 = cy0 + 7;
    }
  }
#pragma unroll
  for (int m = 2; m >= 1; m >>= 1) {
    cx0 = min(cx0, __shfl_xor(cx0, m)); cx1 = max(cx1, __shfl_xor(cx1, m));
    cy0 = min(cy0, __shfl_xor(cy0, m)); cy1 = max(cy1, __shfl_xor(cy1, m));
  }
  if (lane == 0 || lane == 4) {   // chroma union box per list (Cb and Cr share the MVs and the plane size)
    s_box[1][lane >> 2][0] = cx0; s_box[1][lane >> 2][1] = cx1;
    s_box[1][lane >> 2][2] = cy0; s_box[1][lane >> 2][3] = cy1;
  }
  __syncthreads();
  int ubox[2][4], cbox[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      ubox[l][q] = __builtin_amdgcn_readfirstlane(s_box[0][l][q]);
      cbox[l][q] = __builtin_amdgcn_readfirstlane(s_box[1][l][q]);
    }

  // ---- window buffers. Per list (luma) and per (component, list) (chroma): the union box of the
  // sub-block windows (reduced above), its aligned origin, and the mode.
  int lax[2], loy[2], lrows[2], lnch[2], lmode[2];   // mode: 0 union box, 2 per sub-block
  int cax[4], coy[4], crows[4], cnch[4], cmode[4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    lmode[l] = 0; lax[l] = loy[l] = lrows[l] = lnch[l] = 0;
    if (!U.l[l].present) continue;
    const DPlane &R = P.ref.get(U.l[l].slot, 0);
    const int x0 = ubox[l][0], x1 = ubox[l][1], y0 = ubox[l][2], y1 = ubox[l][3];
    lax[l] = x0 & ~3; loy[l] = y0;
    lnch[l] = (x1 - lax[l] + 3) >> 2; lrows[l] = y1 - y0;
    if (lnch[l] * 4 > LUP || lrows[l] > LUR || lrows[l] * (lnch[l] <= 8 ? 8 : 16) > 8 * 64) lmode[l] = 2;
    (void)R;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int l = k & 1, comp = 1 + (k >> 1);
    cmode[k] = 0; cax[k] = coy[k] = crows[k] = cnch[k] = 0;
    if (!U.l[l].present) continue;
    const DPlane &R = P.ref.get(U.l[l].slot, comp);
    const int x0 = cbox[l][0], x1 = cbox[l][1], y0 = cbox[l][2], y1 = cbox[l][3];
    cax[k] = x0 & ~3; coy[k] = y0;
    cnch[k] = (x1 - cax[k] + 3) >> 2; crows[k] = y1 - y0;
    if (cnch[k] > 8 || crows[k] > 16) cmode[k] = 2;
    (void)R;
  }

  // ---- gather: union boxes in 4-sample chunks (all in flight before the LDS writes; rows clamped to the
  // picture, edge chunks per sample: chunk4), per-sub-block windows per sample in batches of 8
  {
    uint2 vl[2][4], vc[4];
#pragma unroll
    for (int l = 0; l < 2; l++) {
      if (!U.l[l].present || lmode[l] != 0) continue;
      const DPlane &R = P.ref.get(U.l[l].slot, 0);
      const int lg = lnch[l] <= 8 ? 3 : 4, n = lrows[l] << lg;   // chunk slots per row: 8 or 16
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = lane + 128 * k, r = i >> lg, c = i & ((1 << lg) - 1);
        if (i < n && c < lnch[l]) vl[l][k] = chunk4(R.p, R.stride, R.w, R.h, loy[l] + r, lax[l] + 4 * c);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (!U.l[k & 1].present || cmode[k] != 0) continue;
      const DPlane &R = P.ref.get(U.l[k & 1].slot, 1 + (k >> 1));
      const int n = crows[k] << 3;   // 8 chunk slots per row
      {
        const int i = lane, r = i >> 3, c = i & 7;
        if (i < n && c < cnch[k]) vc[k] = chunk4(R.p, R.stride, R.w, R.h, coy[k] + r, cax[k] + 4 * c);
      }
    }
#pragma unroll
    for (int l = 0; l < 2; l++) {
      if (!U.l[l].present || lmode[l] != 0) continue;
      const int lg = lnch[l] <= 8 ? 3 : 4, n = lrows[l] << lg;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = lane + 128 * k, r = i >> lg, c = i & ((1 << lg) - 1);
        if (i < n && c < lnch[l]) *(uint2 *)&s_lw[l][r * LUP + 4 * c] = vl[l][k];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (!U.l[k & 1].present || cmode[k] != 0) continue;
      const int n = crows[k] << 3;
      {
        const int i = lane, r = i >> 3, c = i & 7;
        if (i < n && c < cnch[k]) *(uint2 *)&s_cw[k][r * CUP + 4 * c] = vc[k];
      }
    }
    // per-sub-block windows
#pragma unroll
    for (int l = 0; l < 2; l++) {
      if (!U.l[l].present || lmode[l] == 0) continue;
      const DPlane &R = P.ref.get(U.l[l].slot, 0);
      for (int i0 = lane; i0 < nsb * LSBS; i0 += 8 * 128) {
        int16_t v[8];
#pragma unroll
        for (int b = 0; b < 8; b++) {
          const int i = min(i0 + 128 * b, nsb * LSBS - 1);
          const int sb = i / LSBS, rem = i - sb * LSBS, r = rem / LSBP, e = rem - r * LSBP;
          const int ox = J.x + (sb & (nsx - 1)) * 4 + (s_sbmv[l][sb][0] >> 4) - 3, oy = J.y + (sb >> lnsx) * 4 + (s_sbmv[l][sb][1] >> 4) - 3;
          v[b] = R.p[(size_t)clampi(oy + r, 0, R.h - 1) * R.stride + clampi(ox + e, 0, R.w - 1)];
        }
#pragma unroll
        for (int b = 0; b < 8; b++)
          if (i0 + 128 * b < nsb * LSBS) s_lw[l][i0 + 128 * b] = v[b];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int l = k & 1;
      if (!U.l[l].present || cmode[k] == 0) continue;
      const DPlane &R = P.ref.get(U.l[l].slot, 1 + (k >> 1));
      for (int i0 = lane; i0 < ncb * CSBS; i0 += 8 * 128) {
        int16_t v[8];
#pragma unroll
        for (int b = 0; b < 8; b++) {
          const int i = min(i0 + 128 * b, ncb * CSBS - 1);
          const int cb = i / CSBS, rem = i - cb * CSBS, r = rem / CSBP, e = rem - r * CSBP;
          const int ox = (J.x >> 1) + (cb % ncx) * 4 + (s_csmv[l][cb][0] >> 5) - 1, oy = (J.y >> 1) + (cb / ncx) * 4 + (s_csmv[l][cb][1] >> 5) - 1;
          v[b] = R.p[(size_t)clampi(oy + r, 0, R.h - 1) * R.stride + clampi(ox + e, 0, R.w - 1)];
        }
#pragma unroll
        for (int b = 0; b < 8; b++)
          if (i0 + 128 * b < ncb * CSBS) s_cw[k][i0 + 128 * b] = v[b];
      }
    }
  }
  __syncthreads();

  // placement of a luma sub-block window of list l / a chroma sub-block window of combo k
  auto lplace = [&](int l, int sb) -> Place {
    const int lm = l ? lmode[1] : lmode[0];
    if (lm == 2) return Place{sb * LSBS, LSBP, 0, 0};
    const int ox = J.x + (sb & (nsx - 1)) * 4 + (s_sbmv[l][sb][0] >> 4) - 3, oy = J.y + (sb >> lnsx) * 4 + (s_sbmv[l][sb][1] >> 4) - 3;
    return Place{0, LUP, ox - (l ? lax[1] : lax[0]), oy - (l ? loy[1] : loy[0])};
  };
  auto csel = [&](const int (&a)[4], int k) { return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3]; };
  auto cplace = [&](int k, int cb) -> Place {
    const int l = k & 1;
    if (csel(cmode, k) == 2) return Place{cb * CSBS, CSBP, 0, 0};
    const int ox = (J.x >> 1) + (cb % ncx) * 4 + (s_csmv[l][cb][0] >> 5) - 1, oy = (J.y >> 1) + (cb / ncx) * 4 + (s_csmv[l][cb][1] >> 5) - 1;
    return Place{0, CUP, ox - csel(cax, k), oy - csel(coy, k)};
  };

  // ---- H passes. Luma items (list, sub-block, row pair): window rows 1..10 (the V taps read 1..9), the
  // 6 taps of output column c at window columns c+1..c+6. Chroma items (combo, sub-block, row pair).
  const int nl = (U.l[0].present ? 1 : 0) + (U.l[1].present ? 1 : 0);
  const int lfirst = U.l[0].present ? 0 : 1;
#pragma unroll
  for (int it = 0; it < 2; it++) {
    const int i = lane + 128 * it, per = nsb * 5;
    if (i < nl * per) {
      const int l = i >= per ? 1 : lfirst, rem = i >= per ? i - per : i;
      const int sb = rem / 5, rp = rem - sb * 5;
      const Place pl = lplace(l, sb);
      const int b = pl.ex + 1, par = b & 1;
      const uint32_t *r0 = (const uint32_t *)(s_lw[l] + pl.base + (pl.ey + 1 + 2 * rp) * pl.pitch) + ((b - par) >> 1);
      uint32_t w0[5], w1[5];
#pragma unroll
      for (int k = 0; k < 5; k++) { w0[k] = r0[k]; w1[k] = r0[pl.pitch / 2 + k]; }
      const uint32_t *tp = s_tl[s_sbmv[l][sb][0] & 15];
      Taps<6> t;
#pragma unroll
      for (int k = 0; k < 3; k++) t.A[k] = tp[k];
#pragma unroll
      for (int k = 0; k < 4; k++) t.B[k] = tp[3 + k];
      int a[4], c[4];
      fir4_var<6>(w0, t, par, a);
      fir4_var<6>(w1, t, par, c);
      uint32_t *dst = (uint32_t *)(s_ht[l] + sb * HTS);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[(q * HTC + 2 * rp) >> 1] = pk((int16_t)((a[q] + off1) >> sh1), (int16_t)((c[q] + off1) >> sh1));
    }
  }
  if (lane < 64) {
    const int k = lane >> 4, cb = (lane >> 2) & 3, rp = lane & 3, l = k & 1;
    if (PRES(l) && cb < ncb) {
      const Place pl = cplace(k, cb);
      const int b = pl.ex, par = b & 1;
      const uint32_t *r0 = (const uint32_t *)(s_cw[k] + pl.base + (pl.ey + 2 * rp) * pl.pitch) + ((b - par) >> 1);
      uint32_t w0[4], w1[4];
#pragma unroll
      for (int m = 0; m < 4; m++) { w0[m] = r0[m]; w1[m] = r0[pl.pitch / 2 + m]; }
      const uint32_t *tp = s_tc[s_csmv[l][cb][0] & 31];
      Taps<4> t;
      t.A[0] = tp[0]; t.A[1] = tp[1]; t.B[0] = tp[2]; t.B[1] = tp[3]; t.B[2] = tp[4];
      int a[4], c[4];
      fir4_var<4>(w0, t, par, a);
      fir4_var<4>(w1, t, par, c);
      uint32_t *dst = (uint32_t *)(s_ct[k] + cb * CTS);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[(q * CTC + 2 * rp) >> 1] = pk((int16_t)((a[q] + off1) >> sh1), (int16_t)((c[q] + off1) >> sh1));
    }
  }
  __syncthreads();

  // ---- V passes: items (list, sub-block, column) / (combo, sub-block, column), 4 output rows each
  const bool rndc = !bi && !U.wp;     // chroma and non-PROF luma: final samples for uni without WP
  {
    const int i = lane, per = nsb * 4;
    if (i < nl * per) {
      const int l = i >= per ? 1 : lfirst, rem = i >= per ? i - per : i;
      const int sb = rem >> 2, c = rem & 3;
      const bool rnd = rndc && !(l ? prof[1] : prof[0]);
      const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
      const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
      const uint32_t *col = (const uint32_t *)(s_ht[l] + sb * HTS + c * HTC);
      uint32_t wv[5];
#pragma unroll
      for (int k = 0; k < 5; k++) wv[k] = col[k];
      const uint32_t *tp = s_tl[s_sbmv[l][sb][1] & 15];
      Taps<6> t;
#pragma unroll
      for (int k = 0; k < 3; k++) t.A[k] = tp[k];
#pragma unroll
      for (int k = 0; k < 4; k++) t.B[k] = tp[3 + k];
      int o[4];
      fir4<6, 0>(wv, t, o);
      const int x = (sb & (nsx - 1)) * 4 + c, y0 = (sb >> lnsx) * 4;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        int v = (int16_t)((o[q] + off2) >> sh2);
        if (rnd) v = clampi(v, 0, maxv);
        s_lo[l][(y0 + q) * 16 + x] = (int16_t)v;
      }
    }
  }
  if (lane >= 64) {   // the second wave (the first has the luma V items of list 0)
    const int k = (lane >> 4) & 3, cb = (lane >> 2) & 3, c = lane & 3, l = k & 1;
    if (PRES(l) && cb < ncb) {
      const int sh2 = rndc ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
      const int off2 = rndc ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
      const uint32_t *col = (const uint32_t *)(s_ct[k] + cb * CTS + c * CTC);
      uint32_t wv[4];
#pragma unroll
      for (int m = 0; m < 4; m++) wv[m] = col[m];
      const uint32_t *tp = s_tc[s_csmv[l][cb][1] & 31];
      Taps<4> t;
      t.A[0] = tp[0]; t.A[1] = tp[1]; t.B[0] = tp[2]; t.B[1] = tp[3]; t.B[2] = tp[4];
      int o[4];
      fir4<4, 0>(wv, t, o);
      const int x = (cb % ncx) * 4 + c, y0 = (cb / ncx) * 4;
#pragma unroll
      for (int q = 0; q < 4; q++) {   // s_co aliases the chroma windows: the H pass (before the barrier) read them
        int v = (int16_t)((o[q] + off2) >> sh2);
        if (rndc) v = clampi(v, 0, maxv);
        s_co[k][(y0 + q) * 8 + x] = (int16_t)v;
      }
    }
  }
  __syncthreads();

  // ---- PROF (:1209-1251) on the 14-bit luma prediction of each list that uses it: a ring of integer
  // samples around each sub-block, gradients (shift 6), dMv per position, applyPROFCore. A lane takes a
  // 4-sample row chunk of one sub-block: its row and the rows above / below come from the prediction
  // (or the ring at the sub-block's top / bottom), the left / right neighbours of the chunk from the ring;
  // results are written back after every lane of the wave has read its neighbours (list l is wave l:
  // the wave's LDS accesses execute in order, the asm statement keeps the compiler from moving them).
#pragma unroll
  for (int l = 0; l < 2; l++) {
    const AffList &A = U.l[l];
    if (!A.present || !A.prof) continue;
    const int dILimit = 1 << max(bd + 1, 13);
    const int shiftNum = headRoom, offset = (1 << (shiftNum - 1)) + IF_INTERNAL_OFFS;
    int res[4] = {0, 0, 0, 0};
    const bool act = (lane >> 6) == l && (lane & 63) * 4 < w * h;   // list l in wave l
    const int i = (lane & 63) * 4, y = i / w, x0 = i - y * w;
    if (act) {
      const int sb = (y >> 2) * nsx + (x0 >> 2);
      const int xo = (s_sbmv[l][sb][0] & 15) >> 3, yo = (s_sbmv[l][sb][1] & 15) >> 3;
      const Place pl = lplace(l, sb);
      const int16_t *swin = s_lw[l] + pl.base + (pl.ey + 3 + yo) * pl.pitch + pl.ex + 3 + xo;   // ring origin
      const int py = y & 3;
      auto ring = [&](int ex, int ey) -> int { return (int16_t)((swin[ey * pl.pitch + ex] << headRoom) - IF_INTERNAL_OFFS); };
      const uint2 cr = *(const uint2 *)&s_lo[l][y * 16 + x0];
      const uint2 ur = *(const uint2 *)&s_lo[l][max(y - 1, 0) * 16 + x0];
      const uint2 dr = *(const uint2 *)&s_lo[l][min(y + 1, 15) * 16 + x0];
      const int c[4] = {lo16(cr.x), hi16(cr.x), lo16(cr.y), hi16(cr.y)};
      const int u4[4] = {lo16(ur.x), hi16(ur.x), lo16(ur.y), hi16(ur.y)};
      const int d4[4] = {lo16(dr.x), hi16(dr.x), lo16(dr.y), hi16(dr.y)};
      const int left = ring(-1, py), right = ring(4, py);
      // dMv of the sample (px, py) of a sub-block: uniform part per px, lane part 4 * dv * py
      const int lx = 4 * A.dvx * py - 6 * A.dhx - 6 * A.dvx, ly = 4 * A.dvy * py - 6 * A.dhy - 6 * A.dvy;
#pragma unroll
      for (int px = 0; px < 4; px++) {
        const int up = py > 0 ? u4[px] : ring(px, -1), dn = py < 3 ? d4[px] : ring(px, 4);
        const int lf = px == 0 ? left : c[px - 1], rt = px == 3 ? right : c[px + 1];
        const int gX = (rt >> 6) - (lf >> 6), gY = (dn >> 6) - (up >> 6);
        int dmx = 4 * A.dhx * px + lx, dmy = 4 * A.dhy * px + ly;
        round_affine(dmx, dmy, 8);
        dmx = clampi(dmx, -31, 31);
        dmy = clampi(dmy, -31, 31);
        const int dI = clampi(dmx * gX + dmy * gY, -dILimit, dILimit - 1);
        int v = (int16_t)(c[px] + dI);
        if (!bi && !U.wp) v = clampi((v + offset) >> shiftNum, 0, maxv);
        res[px] = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (act) *(uint2 *)&s_lo[l][y * 16 + x0] = make_uint2(pk(res[0], res[1]), pk(res[2], res[3]));
  }
  __syncthreads();

  // ---- combine (xWeightedAverage: addAvg / addWeightedAvg; weighted prediction; uni already final
  // without WP) and store 4 consecutive samples of a row per lane
  auto combine = [&](int comp, int a, int b) -> int {
    if (!bi) {
      const int l = U.l[0].present ? 0 : 1;
      return U.wp ? wp_uni(P.wp, l, U.l[l].ridx, comp, a, headRoom, maxv) : a;
    }
    if (U.wp) return wp_bi(P.wp, U.l[0].ridx, U.l[1].ridx, comp, a, b, headRoom, maxv);
    if (U.bcw != 2) {
      const int w1 = a_bcw_w1[U.bcw], w0 = 8 - w1;
      const int shiftNum = headRoom + 3;
      const int offset = (1 << (shiftNum - 1)) + (IF_INTERNAL_OFFS << 3);
      return clampi((a * w0 + b * w1 + offset) >> shiftNum, 0, maxv);
    }
    const int shiftNum = headRoom + 1;
    const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
    return clampi((a + b + offset) >> shiftNum, 0, maxv);
  };
  const int la = U.l[0].present ? 0 : 1;
  if (lane * 4 < w * h) {
    const int i = lane * 4, y = i / w, x = i - y * w;
    const uint2 a = *(const uint2 *)&s_lo[la][y * 16 + x];
    const uint2 b = bi ? *(const uint2 *)&s_lo[1][y * 16 + x] : a;
    const int v0 = combine(0, lo16(a.x), lo16(b.x)), v1 = combine(0, hi16(a.x), hi16(b.x));
    const int v2 = combine(0, lo16(a.y), lo16(b.y)), v3 = combine(0, hi16(a.y), hi16(b.y));
    const DPlane &o = P.out[0];
    *(uint2 *)(o.p + (size_t)(J.y + y) * o.stride + J.x + x) = make_uint2(pk(v0, v1), pk(v2, v3));
  }
  if (lane >= 64) {
    const int comp = 1 + ((lane >> 5) & 1), i = (lane & 31) * 4;
    if (i < cw * chh) {
      const int y = i / cw, x = i - y * cw, ka = 2 * (comp - 1) + la, kb = 2 * (comp - 1) + 1;
      const uint2 a = *(const uint2 *)&s_co[ka][y * 8 + x];
      const uint2 b = bi ? *(const uint2 *)&s_co[kb][y * 8 + x] : a;
      const int v0 = combine(comp, lo16(a.x), lo16(b.x)), v1 = combine(comp, hi16(a.x), hi16(b.x));
      const int v2 = combine(comp, lo16(a.y), lo16(b.y)), v3 = combine(comp, hi16(a.y), hi16(b.y));
      const DPlane &o = P.out[comp];
      *(uint2 *)(o.p + (size_t)((J.y >> 1) + y) * o.stride + (J.x >> 1) + x) = make_uint2(pk(v0, v1), pk(v2, v3));
    }
  }
}

__global__ __launch_bounds__(256) void k_mc_affine(McParams P, const AffJob *__restrict__ jobs, int njobs, const AffPu *__restrict__ pus) {
  __shared__ AffLds lds[2];
  const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
  mc_affine(P, jobs, njobs, pus, 2 * blockIdx.x + half, threadIdx.x & 127, lds[half]);
}

}  // namespace

void launch_mc_affine(const McParams &p, const AffJob *jobs, int njobs, const AffPu *pus, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mc_affine, dim3((njobs + 1) / 2), dim3(256), 0, s, p, jobs, njobs, pus);
}
