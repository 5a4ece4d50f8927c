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
// sub-block filters from its offset inside that union (a 16x16 tile: ~24x28 samples instead of
// 16 x 121). The union buffers are sized for the unions of ordinary affine motion (luma <= 32 x 25,
// chroma <= 16 x 13 per list: every tile of the test streams fits) so that a 256-lane workgroup of two
// tiles needs < 20 KB of LDS and eight fit a CU (the kernel is latency-bound: its time scales with
// the workgroups per CU). A list whose union does not fit (strongly diverging MVs) reads its window
// samples straight from the reference picture instead (per sample, clamped), in the H pass and PROF.
// Chunks that reach outside the picture are loaded per sample with clamped coordinates (= the
// reference's edge-extended margin, Picture::extendPicBorder).
//
// Filtering is the separable H-then-V form for every fraction (identity phase for zero fractions; see
// vvcr_mc.hip), with packed int16 pairs and v_dot2c (vvcr_mcdev.h): lanes hold different sub-blocks, so
// taps come from LDS tables indexed by each lane's fraction and the pair parity is per lane (fir4_var).
#include "vvcr_internal.h"
#include <cstdlib>

#ifndef AFF_XCD_RUN
#define AFF_XCD_RUN 32
#endif
#ifndef AFF_ABL
#define AFF_ABL 0   // diagnostics ablations (results wrong): 1 no PROF, 2 no chroma, 4 no luma H, 8 no luma V, 16 no gather
#endif
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
constexpr int LUP = 36, LUR = 25, LWS = LUP * LUR;   // luma union window per list: 8 chunks x 25 rows, pitch 18 dwords (H-pass reads of neighbouring row pairs and sub-blocks in different banks)
constexpr int CUP = 16, CUR = 14, CWS = CUP * CUR;    // chroma union per (component, list): 4 chunks x 13 rows (+1 pad row)
constexpr int HTC = 10, HTS = 4 * HTC;                // luma H outputs [sub-block][col][10 rows]
constexpr int CTC = 8, CTS = 4 * CTC;                 // chroma H outputs [sub-block][col][8 rows]
// after the H passes the chroma windows hold the chroma predictions [combo][y * 8 + x], then the luma
// prediction per list [y * 16 + x]
static_assert(4 * 64 + 2 * 256 <= 4 * CWS, "predictions fit the chroma window buffers");

// Where the window of a sub-block lies in its list's union buffer: element (r, e) of the window (row r,
// column e, relative to the window's top-left tap) is buf[(ey + r) * pitch + ex + e]; ox / oy: the window's
// top-left tap in the reference picture (the global fallback reads there).
struct Place {
  int pitch, ex, ey, ox, oy;
};

// N sample pairs of row r of a sub-block window, from window element e0 on (pair k = elements e0 + 2k,
// e0 + 2k + 1): aligned dwords of the union buffer, or (glob) per sample from the reference picture with
// clamped coordinates
template <int N>
__device__ __forceinline__ void win_pairs(bool glob, const int16_t *buf, const Place &pl, const DPlane &R, int r, int e0, uint32_t (&w)[N]) {
  if (!glob) {
    const uint32_t *q = (const uint32_t *)(buf + (pl.ey + r) * pl.pitch + pl.ex + e0);
#pragma unroll
    for (int k = 0; k < N; k++) w[k] = q[k];
  } else {
    const int16_t *row = R.p + (size_t)clampi(pl.oy + r, 0, R.h - 1) * R.stride;
#pragma unroll
    for (int k = 0; k < N; k++)
      w[k] = pk(row[clampi(pl.ox + e0 + 2 * k, 0, R.w - 1)], row[clampi(pl.ox + e0 + 2 * k + 1, 0, R.w - 1)]);
  }
}


// ------------------------------------------------------------------------------------------------
// k_mc_affine: ONE WAVE per tile (r05). The r04 form ran two tiles on four waves of a workgroup, so every
// phase of both tiles met at a four-wave barrier; here a tile's phases are wave-local (its barriers are
// LDS waits) and the lists are processed one after the other through one union window and one H buffer,
// both lists' window samples gathered into registers up front (6.2 KB of LDS per wave instead of 10).
// Phases: sub-block MVs and union boxes (shuffle reductions, boxes by readlane) -> gather of every union
// window into registers -> per list: window to LDS, H pass (+ the chroma H of both lists with the first),
// V pass, PROF in place -> combine and store.
// ------------------------------------------------------------------------------------------------
struct AffLds1 {
  alignas(16) int16_t lw[LWS];          // the current list's luma union window
  alignas(16) int16_t cw[4][CWS];       // chroma union windows, combo k = 2 * (comp - 1) + list; then the predictions
  alignas(16) int16_t ht[16 * HTS];     // luma H outputs of the current list [sub-block][col][10 rows]
  alignas(16) int16_t ct[4][4 * CTS];   // chroma H outputs
  int sbmv[2][16][2];                   // MC MV of each luma sub-block (clamped)
  int csmv[2][4][2];                    // chroma sub-block MVs
};

__device__ __forceinline__ void mc_affine1(const McParams &P, const AffJob &J, const AffPu &U, bool force_glob, AffLds1 &L) {
  const int lane = threadIdx.x;
  int16_t(*s_co)[64] = (int16_t(*)[64])L.cw[0];              // after the chroma H pass: chroma predictions
  int16_t(*s_lo)[256] = (int16_t(*)[256])(L.cw[0] + 4 * 64);  // and the luma prediction per list
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const bool pres[2] = {U.l[0].present != 0, U.l[1].present != 0}, prof[2] = {U.l[0].prof != 0, U.l[1].prof != 0};
  const bool bi = pres[0] && pres[1];
  auto PRES = [&](int l) { return l ? pres[1] : pres[0]; };
  const int slot0 = pres[0] ? U.l[0].slot : 0, slot1 = pres[1] ? U.l[1].slot : 0;
  const DPlane RL0 = P.ref.get(slot0, 0), RL1 = P.ref.get(slot1, 0);
  const DPlane RC00 = P.ref.get(slot0, 1), RC01 = P.ref.get(slot1, 1), RC10 = P.ref.get(slot0, 2), RC11 = P.ref.get(slot1, 2);
  auto lref = [&](int l) { DPlane d = RL0; d.p = l ? RL1.p : RL0.p; return d; };
  auto cref = [&](int k) { DPlane d = RC00; d.p = k == 0 ? RC00.p : k == 1 ? RC01.p : k == 2 ? RC10.p : RC11.p; return d; };
  const int w = J.w, h = J.h;           // 8 or 16 (affine PUs are >= 8x8, tiled by 16)
  const int lnsx = w == 16 ? 2 : 1, nsx = 1 << lnsx, nsb = (w >> 2) * (h >> 2);
  const int cw = w >> 1, chh = h >> 1, ncx = cw >> 2, ncb = (cw >> 2) * (chh >> 2);
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);

  // ---- sub-block MVs of both lists (:1102-1140), MV clamp of xPredAffineBlk (:936-939): lanes 0..31 the
  // luma sub-blocks (list = lane / 16), lanes 32..39 the chroma sub-blocks (list = (lane - 32) / 4)
  const int iHorMax = (P.pic_w + 8 - U.x - 1) << 4, iHorMin = (-P.ctu - 8 - U.x + 1) << 4;
  const int iVerMax = (P.pic_h + 8 - U.y - 1) << 4, iVerMin = (-P.ctu - 8 - U.y + 1) << 4;
  const int MVLIM = (1 << 17) - 1;
  auto stored_mv = [&](const AffList &A, int sb, int &mx, int &my) {
    const int sw = (J.x - U.x) + (sb & (nsx - 1)) * 4, shh = (J.y - U.y) + (sb >> lnsx) * 4;
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
  };
  int bx0 = 1 << 30, bx1 = -(1 << 30), by0 = 1 << 30, by1 = -(1 << 30);
  int cx0 = 1 << 30, cx1 = -(1 << 30), cy0 = 1 << 30, cy1 = -(1 << 30);
  if (lane < 32) {
    const int l = lane >> 4, sb = lane & 15;
    const AffList &A = l ? U.l[1] : U.l[0];
    if (PRES(l) && sb < nsb) {
      int mx, my;
      stored_mv(A, sb, mx, my);
      const int cmx = clampi(mx, iHorMin, iHorMax), cmy = clampi(my, iVerMin, iVerMax);
      L.sbmv[l][sb][0] = cmx;
      L.sbmv[l][sb][1] = cmy;
      bx0 = J.x + (sb & (nsx - 1)) * 4 + (cmx >> 4) - 3;
      by0 = J.y + (sb >> lnsx) * 4 + (cmy >> 4) - 3;
      bx1 = bx0 + 11;
      by1 = by0 + 11;
    }
  } else if (lane < 40) {   // chroma: 4x4 sub-blocks, MV = mean of two luma sub-block MVs (:1142-1160)
    const int l = (lane >> 2) & 1, cb = lane & 3;
    const AffList &A = l ? U.l[1] : U.l[0];
    if (PRES(l) && cb < ncb) {
      const int cxs = (cb % ncx) * 2, cys = (cb / ncx) * 2;
      int ax, ay, bx, by;
      stored_mv(A, cys * nsx + cxs, ax, ay);
      stored_mv(A, (cys + 1) * nsx + cxs + 1, bx, by);
      int mx = ax + bx, my = ay + by;
      round_affine(mx, my, 1);
      const int cmx = clampi(mx, iHorMin, iHorMax), cmy = clampi(my, iVerMin, iVerMax);
      L.csmv[l][cb][0] = cmx;
      L.csmv[l][cb][1] = cmy;
      cx0 = (J.x >> 1) + (cb % ncx) * 4 + (cmx >> 5) - 1;
      cy0 = (J.y >> 1) + (cb / ncx) * 4 + (cmy >> 5) - 1;
      cx1 = cx0 + 7;
      cy1 = cy0 + 7;
    }
  }
  // union boxes: min / max over the 16 luma / 4 chroma lanes of a list, then read out by readlane
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) {
    bx0 = min(bx0, __shfl_xor(bx0, m)); bx1 = max(bx1, __shfl_xor(bx1, m));
    by0 = min(by0, __shfl_xor(by0, m)); by1 = max(by1, __shfl_xor(by1, m));
  }
#pragma unroll
  for (int m = 2; m >= 1; m >>= 1) {
    cx0 = min(cx0, __shfl_xor(cx0, m)); cx1 = max(cx1, __shfl_xor(cx1, m));
    cy0 = min(cy0, __shfl_xor(cy0, m)); cy1 = max(cy1, __shfl_xor(cy1, m));
  }
  int ubox[2][4], cbox[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    ubox[l][0] = __builtin_amdgcn_readlane(bx0, 16 * l); ubox[l][1] = __builtin_amdgcn_readlane(bx1, 16 * l);
    ubox[l][2] = __builtin_amdgcn_readlane(by0, 16 * l); ubox[l][3] = __builtin_amdgcn_readlane(by1, 16 * l);
    cbox[l][0] = __builtin_amdgcn_readlane(cx0, 32 + 4 * l); cbox[l][1] = __builtin_amdgcn_readlane(cx1, 32 + 4 * l);
    cbox[l][2] = __builtin_amdgcn_readlane(cy0, 32 + 4 * l); cbox[l][3] = __builtin_amdgcn_readlane(cy1, 32 + 4 * l);
  }

  // ---- window placement per list / (component, list): aligned origin of the union box, or (mode 2) reads
  // from the reference picture when the union does not fit the buffers
  int lax[2], loy[2], lrows[2], lnch[2], lmode[2];
  int cax[4], coy[4], crows[4], cnch[4], cmode[4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    lmode[l] = 0; lax[l] = loy[l] = lrows[l] = lnch[l] = 0;
    if (!PRES(l)) continue;
    lax[l] = ubox[l][0] & ~3; loy[l] = ubox[l][2];
    lnch[l] = (ubox[l][1] - lax[l] + 3) >> 2; lrows[l] = ubox[l][3] - ubox[l][2];
    if (lnch[l] > 8 || lrows[l] > LUR || force_glob) lmode[l] = 2;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int l = k & 1;
    cmode[k] = 0; cax[k] = coy[k] = crows[k] = cnch[k] = 0;
    if (!PRES(l)) continue;
    cax[k] = cbox[l][0] & ~3; coy[k] = cbox[l][2];
    cnch[k] = (cbox[l][1] - cax[k] + 3) >> 2; crows[k] = cbox[l][3] - cbox[l][2];
    if (cnch[k] * 4 > CUP || crows[k] > CUR - 1 || force_glob) cmode[k] = 2;
  }

  // ---- gather every union window into registers (all loads in flight at once): luma 8 chunk slots per
  // row (<= 25 rows: 4 items per lane and list), chroma 4 slots per row (<= 13 rows: one item)
  uint2 vl[2][4], vc[4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!PRES(l) || lmode[l] != 0 || (AFF_ABL & 16)) continue;
    const DPlane R = lref(l);
    const int n = lrows[l] << 3;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int i = lane + 64 * k, r = i >> 3, c = i & 7;
      if (i < n && c < lnch[l]) vl[l][k] = chunk4(R.p, R.stride, R.w, R.h, loy[l] + r, lax[l] + 4 * c);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (!PRES(k & 1) || cmode[k] != 0 || (AFF_ABL & 16)) continue;
    const DPlane R = cref(k);
    const int r = lane >> 2, c = lane & 3;
    if ((lane >> 2) < crows[k] && c < cnch[k]) vc[k] = chunk4(R.p, R.stride, R.w, R.h, coy[k] + r, cax[k] + 4 * c);
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (!PRES(k & 1) || cmode[k] != 0) continue;
    const int r = lane >> 2, c = lane & 3;
    if (r < crows[k] && c < cnch[k]) *(uint2 *)&L.cw[k][r * CUP + 4 * c] = vc[k];
  }

  auto csel = [&](const int (&a)[4], int k) { return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3]; };
  auto cglob = [&](int k) { return csel(cmode, k) == 2; };
  auto cplace = [&](int k, int cb) -> Place {
    const int l = k & 1;
    const int ox = (J.x >> 1) + (cb % ncx) * 4 + (L.csmv[l][cb][0] >> 5) - 1, oy = (J.y >> 1) + (cb / ncx) * 4 + (L.csmv[l][cb][1] >> 5) - 1;
    if (cglob(k)) return Place{0, 0, 0, ox, oy};
    return Place{CUP, ox - csel(cax, k), oy - csel(coy, k), ox, oy};
  };
  const bool rndc = !bi && !U.wp;     // chroma and non-PROF luma: final samples for uni without WP

  // ---- the lists one after the other
  bool first = true;
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!PRES(l)) continue;
    const bool glob = lmode[l] == 2;
    const DPlane R = lref(l);
    const AffList &A = l ? U.l[1] : U.l[0];
    if (!glob) {
      const int n = lrows[l] << 3;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = lane + 64 * k, r = i >> 3, c = i & 7;
        if (i < n && c < lnch[l]) *(uint2 *)&L.lw[r * LUP + 4 * c] = vl[l][k];
      }
    }
    __syncthreads();   // the window (and, on the first list, the MVs and chroma windows) visible to every lane
    auto lplace = [&](int sb) -> Place {
      const int ox = J.x + (sb & (nsx - 1)) * 4 + (L.sbmv[l][sb][0] >> 4) - 3, oy = J.y + (sb >> lnsx) * 4 + (L.sbmv[l][sb][1] >> 4) - 3;
      if (glob) return Place{0, 0, 0, ox, oy};
      return Place{LUP, ox - lax[l], oy - loy[l], ox, oy};
    };
    // H pass: items (sub-block, row pair): window rows 1..10, the 6 taps of output column c at window
    // columns c+1..c+6
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int i = lane + 64 * it;
      if (i < nsb * 5 && !(AFF_ABL & 4)) {
        const int sb = i / 5, rp = i - sb * 5;
        const Place pl = lplace(sb);
        const int b = pl.ex + 1, par = b & 1;
        uint32_t w0[5], w1[5];
        win_pairs<5>(glob, L.lw, pl, R, 1 + 2 * rp, 1 - par, w0);
        win_pairs<5>(glob, L.lw, pl, R, 2 + 2 * rp, 1 - par, w1);
        const uint32_t *tp = a_taps.l[L.sbmv[l][sb][0] & 15];
        Taps<6> t;
#pragma unroll
        for (int k = 0; k < 3; k++) t.A[k] = tp[k];
#pragma unroll
        for (int k = 0; k < 4; k++) t.B[k] = tp[3 + k];
        int a[4], c[4];
        fir4_var<6>(w0, t, par, a);
        fir4_var<6>(w1, t, par, c);
        uint32_t *dst = (uint32_t *)(L.ht + sb * HTS);
#pragma unroll
        for (int q = 0; q < 4; q++) dst[(q * HTC + 2 * rp) >> 1] = pk((int16_t)((a[q] + off1) >> sh1), (int16_t)((c[q] + off1) >> sh1));
      }
    }
    if (first && !(AFF_ABL & 2)) {   // chroma H of both lists: items (combo, sub-block, row pair)
      const int k = lane >> 4, cb = (lane >> 2) & 3, rp = lane & 3, cl = k & 1;
      if (PRES(cl) && cb < ncb) {
        const Place pl = cplace(k, cb);
        const int b = pl.ex, par = b & 1;
        const DPlane CR = cref(k);
        uint32_t w0[4], w1[4];
        win_pairs<4>(cglob(k), L.cw[k], pl, CR, 2 * rp, -par, w0);
        win_pairs<4>(cglob(k), L.cw[k], pl, CR, 2 * rp + 1, -par, w1);
        const uint32_t *tp = a_taps.c[L.csmv[cl][cb][0] & 31];
        Taps<4> t;
        t.A[0] = tp[0]; t.A[1] = tp[1]; t.B[0] = tp[2]; t.B[1] = tp[3]; t.B[2] = tp[4];
        int a[4], c[4];
        fir4_var<4>(w0, t, par, a);
        fir4_var<4>(w1, t, par, c);
        uint32_t *dst = (uint32_t *)(L.ct[k] + cb * CTS);
#pragma unroll
        for (int q = 0; q < 4; q++) dst[(q * CTC + 2 * rp) >> 1] = pk((int16_t)((a[q] + off1) >> sh1), (int16_t)((c[q] + off1) >> sh1));
      }
    }
    __syncthreads();
    // V pass: items (sub-block, column), 4 output rows each
    if (lane < nsb * 4 && !(AFF_ABL & 8)) {
      const int sb = lane >> 2, c = lane & 3;
      const bool rnd = rndc && !(l ? prof[1] : prof[0]);
      const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
      const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
      const uint32_t *col = (const uint32_t *)(L.ht + sb * HTS + c * HTC);
      uint32_t wv[5];
#pragma unroll
      for (int k = 0; k < 5; k++) wv[k] = col[k];
      const uint32_t *tp = a_taps.l[L.sbmv[l][sb][1] & 15];
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
    if (first && !(AFF_ABL & 2)) {   // chroma V: items (combo, sub-block, column); s_co takes the chroma windows' storage
      const int k = lane >> 4, cb = (lane >> 2) & 3, c = lane & 3, cl = k & 1;
      if (PRES(cl) && cb < ncb) {
        const int sh2 = rndc ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
        const int off2 = rndc ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
        const uint32_t *col = (const uint32_t *)(L.ct[k] + cb * CTS + c * CTC);
        uint32_t wv[4];
#pragma unroll
        for (int m = 0; m < 4; m++) wv[m] = col[m];
        const uint32_t *tp = a_taps.c[L.csmv[cl][cb][1] & 31];
        Taps<4> t;
        t.A[0] = tp[0]; t.A[1] = tp[1]; t.B[0] = tp[2]; t.B[1] = tp[3]; t.B[2] = tp[4];
        int o[4];
        fir4<4, 0>(wv, t, o);
        const int x = (cb % ncx) * 4 + c, y0 = (cb / ncx) * 4;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          int v = (int16_t)((o[q] + off2) >> sh2);
          if (rndc) v = clampi(v, 0, maxv);
          s_co[k][(y0 + q) * 8 + x] = (int16_t)v;
        }
      }
    }
    if (A.prof && !(AFF_ABL & 1)) {
      __syncthreads();
      // PROF (:1209-1251) on the 14-bit luma prediction: a lane takes a 4-sample row chunk; its row and the
      // rows above / below come from the prediction (or the integer ring at the sub-block's top / bottom),
      // the left / right neighbours of the chunk from the ring; written back once every lane has read (one
      // wave: its LDS accesses execute in order)
      const int dILimit = 1 << max(bd + 1, 13);
      const int shiftNum = headRoom, offset = (1 << (shiftNum - 1)) + IF_INTERNAL_OFFS;
      int res[4] = {0, 0, 0, 0};
      const bool act = lane * 4 < w * h;
      const int i = lane * 4, y = i / w, x0 = i - y * w;
      if (act) {
        const int sb = (y >> 2) * nsx + (x0 >> 2);
        const int xo = (L.sbmv[l][sb][0] & 15) >> 3, yo = (L.sbmv[l][sb][1] & 15) >> 3;
        const Place pl = lplace(sb);
        const int16_t *swin = L.lw + (pl.ey + 3 + yo) * pl.pitch + pl.ex + 3 + xo;   // ring origin
        const int py = y & 3;
        auto ring = [&](int ex, int ey) -> int {
          const int v = glob ? R.p[(size_t)clampi(pl.oy + 3 + yo + ey, 0, R.h - 1) * R.stride + clampi(pl.ox + 3 + xo + ex, 0, R.w - 1)]
                             : swin[ey * pl.pitch + ex];
          return (int16_t)((v << headRoom) - IF_INTERNAL_OFFS);
        };
        const uint2 cr = *(const uint2 *)&s_lo[l][y * 16 + x0];
        const uint2 ur = *(const uint2 *)&s_lo[l][max(y - 1, 0) * 16 + x0];
        const uint2 dr = *(const uint2 *)&s_lo[l][min(y + 1, 15) * 16 + x0];
        const int c[4] = {lo16(cr.x), hi16(cr.x), lo16(cr.y), hi16(cr.y)};
        const int u4[4] = {lo16(ur.x), hi16(ur.x), lo16(ur.y), hi16(ur.y)};
        const int d4[4] = {lo16(dr.x), hi16(dr.x), lo16(dr.y), hi16(dr.y)};
        const int left = ring(-1, py), right = ring(4, py);
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
    __syncthreads();   // the next list's window replaces this one's (the PROF ring reads above)
    first = false;
  }

  // ---- combine (xWeightedAverage: addAvg / addWeightedAvg; weighted prediction; uni already final
  // without WP) and store 4 consecutive samples of a row per lane: luma, then chroma
  auto combine = [&](int comp, int a, int b) -> int {
    if (!bi) {
      const int l = pres[0] ? 0 : 1;
      return U.wp ? wp_uni(*P.wpd, l, l ? U.l[1].ridx : U.l[0].ridx, comp, a, headRoom, maxv) : a;
    }
    if (U.wp) return wp_bi(*P.wpd, U.l[0].ridx, U.l[1].ridx, comp, a, b, headRoom, maxv);
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
  auto store4 = [&](int comp, int x, int y, int v0, int v1, int v2, int v3) {
    if (U.recon & MC_RECON) {
      if (U.recon & (MC_RESI << comp)) {
        const DPlane &r = P.resi[comp];
        const uint2 q = *(const uint2 *)(r.p + (size_t)y * r.stride + x);
        v0 = clampi(v0 + lo16(q.x), 0, maxv); v1 = clampi(v1 + hi16(q.x), 0, maxv);
        v2 = clampi(v2 + lo16(q.y), 0, maxv); v3 = clampi(v3 + hi16(q.y), 0, maxv);
      }
      const DPlane &o = P.reco[comp];
      *(uint2 *)(o.p + (size_t)y * o.stride + x) = make_uint2(pk(v0, v1), pk(v2, v3));
    } else {
      const DPlane &o = P.out[comp];
      *(uint2 *)(o.p + (size_t)y * o.stride + x) = make_uint2(pk(v0, v1), pk(v2, v3));
    }
  };
  const int la = pres[0] ? 0 : 1;
  if (lane * 4 < w * h) {
    const int i = lane * 4, y = i / w, x = i - y * w;
    const uint2 a = *(const uint2 *)&s_lo[la][y * 16 + x];
    const uint2 b = bi ? *(const uint2 *)&s_lo[1][y * 16 + x] : a;
    store4(0, J.x + x, J.y + y, combine(0, lo16(a.x), lo16(b.x)), combine(0, hi16(a.x), hi16(b.x)),
           combine(0, lo16(a.y), lo16(b.y)), combine(0, hi16(a.y), hi16(b.y)));
  }
  {
    const int comp = 1 + (lane >> 5), i = (lane & 31) * 4;
    if (i < cw * chh) {
      const int y = i / cw, x = i - y * cw, ka = 2 * (comp - 1) + la, kb = 2 * (comp - 1) + 1;
      const uint2 a = *(const uint2 *)&s_co[ka][y * 8 + x];
      const uint2 b = bi ? *(const uint2 *)&s_co[kb][y * 8 + x] : a;
      store4(comp, (J.x >> 1) + x, (J.y >> 1) + y, combine(comp, lo16(a.x), lo16(b.x)), combine(comp, hi16(a.x), hi16(b.x)),
             combine(comp, lo16(a.y), lo16(b.y)), combine(comp, hi16(a.y), hi16(b.y)));
    }
  }
}

// A tile of one of the batch's pictures per workgroup (picture p: blocks [job0[p], job0[p + 1]))
__global__ __launch_bounds__(64) void k_mc_affine(ExtBatch B) {
  __shared__ AffLds1 L;
  // XCD runs of 32 tiles (xcd_run_swizzle): neighbouring tiles' windows share an L2
#if AFF_XCD_RUN > 0
  const int j = xcd_run_swizzle((int)blockIdx.x, (int)gridDim.x, AFF_XCD_RUN);
#else
  const int j = (int)blockIdx.x;
#endif
  if (j >= B.job0[B.npic]) return;
  int p = 0;
#pragma unroll
  for (int q = 1; q < MC_MAXPIC; q++)
    if (q < B.npic && j >= B.job0[q]) p = q;
  const McParams &P = B.pic[p];   // (p uniform: scalar-offset reads of the kernel argument)
  const AffJob J = load_uniform((const AffJob *)B.jobs[p] + (j - B.job0[p]));
  const AffPu U = load_uniform(B.pus[p] + J.pu);
  mc_affine1(P, J, U, B.force_glob != 0, L);
}

}  // namespace

void launch_mc_affine(ExtBatch &b, hipStream_t s) {
  // VVCR_AFF_FALLBACK=1 (tests): every list reads its windows from the reference picture, the path of
  // unions that do not fit the LDS buffers
  static const int force = [] { const char *e = getenv("VVCR_AFF_FALLBACK"); return e && e[0] == '1' ? 1 : 0; }();
  b.force_glob = force;
  b.job0[0] = 0;
  for (int p = 0; p < MC_MAXPIC; p++) b.job0[p + 1] = b.job0[p] + (p < b.npic ? b.njobs[p] : 0);
  const int n = b.job0[b.npic];
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mc_affine, dim3(n), dim3(64), 0, s, b);
}
