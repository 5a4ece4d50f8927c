// vvcr_mc_ext.hip — the inter tools beyond plain interpolation, for gfx950.
//
// k_mc_bidir: one wave per bi-predicted block of <= 16x16 luma that needs decoder-side MV refinement
//   (DMVR, InterPrediction::xProcessDMVR InterPrediction.cpp:2133-2326: bilinear pre-MC of a +-2 search
//   window, 25-point SAD with row subsampling, parabolic sub-pel refinement, final MC from the padded
//   prefetch window) and/or bi-directional optical flow (BDOF, applyBiOptFlow :1274-1367 with the
//   integer-sample extension of xPredInterBlk :812-850 and the gradient / sum / average cores of
//   Buffer.cpp:88-199). The block is one DMVR sub-block (min(16, PU size)) or one xSubPuBio tile.
// (k_mc_affine: vvcr_mc_affine.hip)
// Reference windows are staged in LDS with coordinates clamped to the picture (and, for DMVR, to the
// prefetched window, reproducing xPad's edge replication).
#include "vvcr_internal.h"
#include "vvcr_tables.h"

#define BIDIR_WG 64
#ifndef BIDIR_XCD_RUN
#define BIDIR_XCD_RUN 32
#endif

namespace {

__constant__ int8_t x_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
__constant__ int8_t x_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
__constant__ int8_t x_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int8_t x_bcw_w1[5] = VVCR_BCW_W1;
__constant__ int8_t x_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
// DMVR search order (InterPrediction.h:99 m_pSearchOffset)
__constant__ int8_t x_search[25][2] = {{-2, -2}, {-1, -2}, {0, -2}, {1, -2}, {2, -2}, {-2, -1}, {-1, -1}, {0, -1}, {1, -1},
                                       {2, -1},  {-2, 0},  {-1, 0}, {0, 0},  {1, 0},  {2, 0},  {-2, 1}, {-1, 1}, {0, 1},
                                       {1, 1},   {2, 1},   {-2, 2}, {-1, 2}, {0, 2},  {1, 2},  {2, 2}};

constexpr int IF_INTERNAL_PREC = 14;
constexpr int IF_FILTER_PREC = 6;
constexpr int IF_INTERNAL_OFFS = 1 << (IF_INTERNAL_PREC - 1);

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Picture sample with the coordinate first clamped to a window [x0,x1]x[y0,y1] (DMVR padded prefetch
// buffer) and then to the picture (edge-extended reference picture).
struct Clamp {
  int x0, x1, y0, y1;
};
__device__ __forceinline__ int sample(const DPlane &P, int x, int y, const Clamp &c) {
  x = clampi(clampi(x, c.x0, c.x1), 0, P.w - 1);
  y = clampi(clampi(y, c.y0, c.y1), 0, P.h - 1);
  return P.p[(size_t)y * P.stride + x];
}

// ---------------------------------------------------------------------------------------------
// DMVR helpers
// ---------------------------------------------------------------------------------------------
__device__ int div_for_maxq7(long long N, long long D) {   // InterPrediction.cpp:1866
  int sign = 0, q = 0;
  if (N < 0) { sign = 1; N = -N; }
  D <<= 3;
  if (N >= D) { N -= D; q++; }
  q <<= 1;
  D >>= 1;
  if (N >= D) { N -= D; q++; }
  q <<= 1;
  if (N >= (D >> 1)) q++;
  return sign ? -q : q;
}

__device__ void subpel_surface(const unsigned long long *s, int *d) {   // xSubPelErrorSrfc :1897
  long long num = (long long)((s[1] - s[3]) << 4);
  long long den = (long long)(s[1] + s[3] - (s[0] << 1));
  if (den != 0) {
    if (s[1] != s[0] && s[3] != s[0]) d[0] = div_for_maxq7(num, den);
    else d[0] = s[1] == s[0] ? -8 : 8;
  }
  num = (long long)((s[2] - s[4]) << 4);
  den = (long long)(s[2] + s[4] - (s[0] << 1));
  if (den != 0) {
    if (s[2] != s[0] && s[4] != s[0]) d[1] = div_for_maxq7(num, den);
    else d[1] = s[2] == s[0] ? -8 : 8;
  }
}

constexpr int WS = 24;        // LDS window stride (<= 16 + 7 columns)
constexpr int BS = 20;        // bilinear buffer stride (16 + 4)
constexpr int PS = 18;        // BDOF buffers: (16 + 2) with the 1-sample ring
constexpr int CWS = 12;       // chroma window stride (<= 8 + 3 columns)
constexpr int LWIN = 23 * WS, CWIN = 11 * CWS;

// Gather of one window (clamped like sample()) into per-lane registers: item i = idx + STEP * k of a
// window of pitch PITCH, ITS items per lane.
template <int ITS, int PITCH, int STEP>
__device__ __forceinline__ void gather_regs(const DPlane &P, int ox, int oy, int ww, int wh, const Clamp &c, int idx, int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = idx + STEP * k;
    const int r = i / PITCH, col = i - r * PITCH;
    if (col < ww && r < wh) v[k] = (int16_t)sample(P, ox + col, oy + r, c);
  }
}
template <int ITS, int STEP>
__device__ __forceinline__ void regs_to_lds(int16_t *dst, int size, int idx, const int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = idx + STEP * k;
    if (i < size) dst[i] = v[k];
  }
}

// Taps of one interpolation (identity for a zero fraction: H-then-V with identity rows gives the copy /
// 1-D branches' results exactly, see k_mc_affine), read at a wave-uniform fraction.
__device__ __forceinline__ void luma_taps8(int f, bool alt, int (&t)[8]) {
  const int8_t *c = (alt && f == 8) ? x_alt_hpel : x_luma[f];
#pragma unroll
  for (int u = 0; u < 8; u++) t[u] = f ? c[u] : (u == 3 ? 64 : 0);
}
__device__ __forceinline__ void chroma_taps4(int f, int (&t)[4]) {
#pragma unroll
  for (int u = 0; u < 4; u++) t[u] = f ? x_chroma[f][u] : (u == 1 ? 64 : 0);
}

// k_mc_bidir: ONE WAVE per block (a DMVR sub-block or an xSubPuBio tile: 16x16, 16x8 or 8x16 luma),
// every phase wave-local (a one-wave workgroup: its barriers are only LDS waits), no per-sample global
// gathers and no idle waves behind a workgroup barrier (the r04 form: four waves, nine barrier phases,
// 3-6 % of HBM). Phases:
//  1. gather: both lists' luma prefetch windows (w+7)x(h+7) and the four (component, list) chroma
//     windows (w/2+3)x(h/2+3) of the unrefined MVs (xPrefetch, InterPrediction.cpp:2050) as 16- / 8-byte
//     chunks from the even column at or before the window (rows clamped; a chunk crossing the left / right
//     picture edge gathers its samples with clamped columns: the edge-extended margin, Picture.cpp:737);
//  2. DMVR (xProcessDMVR :2133-2326): bilinear pre-MC of the search windows as sample pairs; the 25-point
//     SAD with row subsampling, a lane per (sampled row, vertical offset) holding both lists' rows in
//     registers and the five horizontal offsets as packed v_sad_u16 sums, rows added by shuffles; the
//     minimum (xDMVRCost's scan order as one key reduction) and the parabolic sub-pel refinement
//     (xSubPelErrorSurface :1897) computed redundantly by every lane;
//  3. final MC: the refined windows read from the staged prefetch windows with coordinates clamped to them
//     (xPad's replication); luma H pass as four outputs per lane on aligned sample pairs with parity tap
//     sets (the k_mc scheme), written transposed, so the V pass reads vertical pairs as aligned dwords;
//     chroma H / V by pairs, both lists of a chroma pair on one lane, averaged (addAvg, Buffer.cpp:447);
//  4. BDOF (applyBiOptFlow :1274-1367): a lane owns one row of 4 samples of a 4x4 unit; it computes its
//     samples' gradients and the unit window terms, the four lanes of a unit add their 6x6 window sums by
//     two shuffles, and each lane applies (vx, vy) to its own samples: no unit table, no extra phase.
// Every output row leaves as one 8-byte (luma) or 4-byte (chroma) store; with MC_RECON the residual is
// added and the reconstruction written into the picture (AreaBuf::reconstruct, Buffer.cpp:590).
constexpr int8_t bk_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
constexpr int8_t bk_alt[8] = VVCR_LUMA_ALT_HPEL;
constexpr int8_t bk_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__host__ __device__ constexpr uint32_t bpk(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }
struct BiTaps {
  uint32_t h[2][16][2][2][5];   // luma H [alt][frac][parity][T0 / T1][pair] (k_mc's cell_hset)
  uint32_t va[2][16][4];        // luma V, first tap on an even row: (c0,c1)(c2,c3)(c4,c5)(c6,c7)
  uint32_t vb[2][16][5];        // luma V, first tap on an odd row: (0,c0)(c1,c2)(c3,c4)(c5,c6)(c7,0)
  uint32_t c[32][2];            // chroma pairs (c0,c1)(c2,c3)
};
constexpr BiTaps make_bitaps() {
  BiTaps t{};
  for (int a = 0; a < 2; a++)
    for (int f = 0; f < 16; f++) {
      int c[8] = {};
      for (int u = 0; u < 8; u++) c[u] = (a && f == 8) ? bk_alt[u] : bk_luma[f][u];
      uint32_t A[5] = {}, B[5] = {};
      for (int k = 0; k < 4; k++) A[k] = bpk(c[2 * k], c[2 * k + 1]);
      B[0] = bpk(0, c[0]);
      for (int k = 1; k < 4; k++) B[k] = bpk(c[2 * k - 1], c[2 * k]);
      B[4] = bpk(c[7], 0);
      for (int k = 0; k < 5; k++) {
        t.h[a][f][0][0][k] = A[k];
        t.h[a][f][0][1][k] = B[k];
        t.h[a][f][1][0][k] = B[k];
        t.h[a][f][1][1][k] = k ? A[k - 1] : 0u;
        t.vb[a][f][k] = B[k];
      }
      for (int k = 0; k < 4; k++) t.va[a][f][k] = A[k];
    }
  for (int f = 0; f < 32; f++)
    for (int k = 0; k < 2; k++) t.c[f][k] = bpk(bk_chroma[f][2 * k], bk_chroma[f][2 * k + 1]);
  return t;
}
__constant__ BiTaps c_btaps = make_bitaps();

__device__ __forceinline__ int bdot2(uint32_t a, uint32_t b, int c) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a), __builtin_bit_cast(s2, b), c, true);
}
__device__ __forceinline__ int blo(uint32_t v) { return (int16_t)(v & 0xffff); }
__device__ __forceinline__ int bhi(uint32_t v) { return (int16_t)(v >> 16); }
typedef uint32_t bu32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t bu32x2 __attribute__((ext_vector_type(2), aligned(4)));

constexpr int BPF = 12;   // luma prefetch window row pitch, dwords (23 samples + the parity sample)
constexpr int BPC = 6;    // chroma window row pitch, dwords (11 + 1)
constexpr int BBL = 10;   // bilinear row pitch, dwords (20 samples)
constexpr int BHT = 24;   // luma H output, transposed: samples per column (23 rows + 1)
constexpr int BPR = 18;   // predictions with their one-sample ring
// 5.5 KB per wave (7 waves per SIMD): buffers whose lifetimes do not overlap share storage
struct BidirLds {
  union {
    uint32_t pf[2][23][BPF];   // luma prefetch windows per list, from the even column at or before them (to the H phase)
    int16_t pr[2][BPR][BPR];   // 14-bit predictions per list, (y + 1, x + 1), ring: integer samples (BDOF) (V phase on)
  } u1;
  union {
    struct {
      uint32_t bl[2][20][BBL];   // DMVR bilinear pre-MC per list
      uint32_t sad[32];          // DMVR: the 25 costs
    } d;
    struct {
      int16_t ht[2][16][BHT];    // luma H pass output per list, column-major
      uint32_t hc[4][11][4];     // chroma H pass output per (component, list), pairs of columns
    } f;
    int16_t t[3][16][16];        // BDOF: (gx0 + gx1) >> 1, (gy0 + gy1) >> 1, (p1 >> 4) - (p0 >> 4)
  } u2;
  uint32_t pc[4][11][BPC];     // chroma windows per (component, list) (to the H phase)
};

template <int W, int H>
__device__ __forceinline__ void bidir_block(const McParams &P, const McJob &J, int32_t *dmvr_out, BidirLds &S) {
  const int lane = threadIdx.x;
  const int bd = P.bd, maxv = (1 << bd) - 1, headRoom = max(2, IF_INTERNAL_PREC - bd);
  const bool dmvr = (J.flags & MC_DMVR) != 0;
  const int alt = (J.flags & MC_ALT_HPEL) ? 1 : 0;   // cu.imv == IMV_HPEL: the final MC only
  const int mx0 = J.mv[0][0], my0 = J.mv[0][1], mx1 = J.mv[1][0], my1 = J.mv[1][1];
  const DPlane RL0 = P.ref.get(J.slot[0], 0), RL1 = P.ref.get(J.slot[1], 0);
  // the four chroma planes, read uniformly (a per-lane slot / component would make the plane-table read a
  // per-lane load in front of the sample loads)
  const DPlane CPL[4] = {P.ref.get(J.slot[0], 1), P.ref.get(J.slot[1], 1), P.ref.get(J.slot[0], 2), P.ref.get(J.slot[1], 2)};
  // prefetch windows: integer MV - 3 (luma) / - 1 (chroma)
  const int px0 = J.x + (mx0 >> 4) - 3, py0 = J.y + (my0 >> 4) - 3, px1 = J.x + (mx1 >> 4) - 3, py1 = J.y + (my1 >> 4) - 3;
  const int cx0 = (J.x >> 1) + (mx0 >> 5) - 1, cy0 = (J.y >> 1) + (my0 >> 5) - 1;
  const int cx1 = (J.x >> 1) + (mx1 >> 5) - 1, cy1 = (J.y >> 1) + (my1 >> 5) - 1;
  const int16_t *pfs = (const int16_t *)&S.u1.pf[0][0][0];   // [l * 23 * 24 + row * 24 + col]
  const int16_t *pcs = (const int16_t *)&S.pc[0][0][0];   // [k * 11 * 12 + row * 12 + col]

  // ---- 1. gather
  {
    constexpr int NCH = W == 16 ? 3 : 2, RL = H + 7, NL = 2 * RL * NCH;   // 16-byte chunks
    constexpr int NCC = W == 16 ? 3 : 2, RC = H / 2 + 3, NC = 4 * RC * NCC; // 8-byte chunks
    constexpr int IL = (NL + 63) / 64, IC = (NC + 63) / 64;
    bu32x4 vl[IL];
    bu32x2 vc[IC];
#pragma unroll
    for (int k = 0; k < IL; k++) {
      const int it = lane + 64 * k;
      if (it < NL) {
        const int l = it >= RL * NCH, rem = it - (l ? RL * NCH : 0), r = rem / NCH, ch = rem - r * NCH;
        const DPlane &R = l ? RL1 : RL0;
        const int y = clampi((l ? py1 : py0) + r, 0, R.h - 1), c0 = ((l ? px1 : px0) & ~1) + 8 * ch;
        const int16_t *row = R.p + (size_t)y * R.stride;
        if (c0 >= 0 && c0 + 8 <= R.w) {
          vl[k] = *(const bu32x4 *)(row + c0);
        } else {
          int v[8];
#pragma unroll
          for (int e = 0; e < 8; e++) v[e] = row[clampi(c0 + e, 0, R.w - 1)];
          vl[k] = bu32x4{bpk(v[0], v[1]), bpk(v[2], v[3]), bpk(v[4], v[5]), bpk(v[6], v[7])};
        }
      }
    }
#pragma unroll
    for (int k = 0; k < IC; k++) {
      const int it = lane + 64 * k;
      if (it < NC) {
        const int kk = it / (RC * NCC), rem = it - kk * (RC * NCC), r = rem / NCC, ch = rem - r * NCC;
        const int l = kk & 1;
        const int16_t *rp = kk == 0 ? CPL[0].p : kk == 1 ? CPL[1].p : kk == 2 ? CPL[2].p : CPL[3].p;
        const DPlane R{const_cast<int16_t *>(rp), CPL[0].stride, CPL[0].w, CPL[0].h};   // Cb and Cr share the geometry
        const int y = clampi((l ? cy1 : cy0) + r, 0, R.h - 1), c0 = ((l ? cx1 : cx0) & ~1) + 4 * ch;
        const int16_t *row = R.p + (size_t)y * R.stride;
        if (c0 >= 0 && c0 + 4 <= R.w) {
          vc[k] = *(const bu32x2 *)(row + c0);
        } else {
          int v[4];
#pragma unroll
          for (int e = 0; e < 4; e++) v[e] = row[clampi(c0 + e, 0, R.w - 1)];
          vc[k] = bu32x2{bpk(v[0], v[1]), bpk(v[2], v[3])};
        }
      }
    }
#pragma unroll
    for (int k = 0; k < IL; k++) {
      const int it = lane + 64 * k;
      if (it < NL) {
        const int l = it >= RL * NCH, rem = it - (l ? RL * NCH : 0), r = rem / NCH, ch = rem - r * NCH;
        uint32_t *d = &S.u1.pf[l][r][4 * ch];
        d[0] = vl[k].x; d[1] = vl[k].y; d[2] = vl[k].z; d[3] = vl[k].w;
      }
    }
#pragma unroll
    for (int k = 0; k < IC; k++) {
      const int it = lane + 64 * k;
      if (it < NC) {
        const int kk = it / (RC * NCC), rem = it - kk * (RC * NCC), r = rem / NCC, ch = rem - r * NCC;
        uint32_t *d = &S.pc[kk][r][2 * ch];
        d[0] = vc[k].x; d[1] = vc[k].y;
      }
    }
  }
  __syncthreads();

  // ---- 2. DMVR search (xinitMC, xBIPMVRefine, xDMVRSubPixelErrorSurface)
  int dx = 0, dy = 0;
  bool bdof = (J.flags & MC_BDOF) != 0;
#ifndef BIDIR_ABL
#define BIDIR_ABL 0   // diagnostics ablations (results wrong): 1 no DMVR search, 2 no BDOF, 4 no chroma
#endif
  if ((BIDIR_ABL & 2)) bdof = false;
  if (dmvr && !(BIDIR_ABL & 1)) {
    {
      // bilinear (InterpolationFilter::filter with m_bilinearFilterPrec4, IF_INTERNAL_PREC_BILINEAR 10): the
      // separable form below reproduces the reference's copy / H-only / V-only branches exactly (every
      // intermediate is non-negative and exact: (16 s + 2^(sh-1)) >> sh == s << (10 - bd))
      const int shB = bd - 6, offB = 1 << (shB - 1);
      constexpr int BW = W + 4, BH = H + 4, NPB = BW / 2, NB = 2 * BH * NPB;
#pragma unroll
      for (int k = 0; k < (NB + 63) / 64; k++) {
        const int it = lane + 64 * k;
        if (it < NB) {
          const int l = it >= BH * NPB, rem = it - (l ? BH * NPB : 0), r = rem / NPB, pp = rem - r * NPB;
          const int fx = (l ? mx1 : mx0) & 15, fy = (l ? my1 : my0) & 15;
          const int par = (l ? px1 : px0) & 1;
          const int16_t *s = pfs + l * (23 * 24) + (r + 1) * 24 + par + 1 + 2 * pp;   // the search window: one row / column in
          const int a0 = s[0], a1 = s[1], a2 = s[2], b0 = s[24], b1 = s[25], b2 = s[26];
          const int t00 = (a0 * (16 - fx) + a1 * fx + offB) >> shB, t01 = (a1 * (16 - fx) + a2 * fx + offB) >> shB;
          const int t10 = (b0 * (16 - fx) + b1 * fx + offB) >> shB, t11 = (b1 * (16 - fx) + b2 * fx + offB) >> shB;
          const int v0 = (t00 * (16 - fy) + t10 * fy + 8) >> 4, v1 = (t01 * (16 - fy) + t11 * fy + 8) >> 4;
          S.u2.d.bl[l][r][pp] = bpk(v0, v1);
        }
      }
    }
    __syncthreads();
    {
      // 25-point SAD over rows 0, 2, 4, .. (xGetSAD with subShift 1): lane (sampled row ri, vertical offset oy)
      constexpr int NR = H / 2, NPB = (W + 4) / 2;
      const int ri = lane % NR, oyi = lane / NR;
      uint32_t acc[5] = {0, 0, 0, 0, 0};
      if (oyi < 5) {
        const int oy = oyi - 2;
        uint32_t A[NPB], B[NPB];
#pragma unroll
        for (int k = 0; k < NPB; k++) { A[k] = S.u2.d.bl[0][2 + oy + 2 * ri][k]; B[k] = S.u2.d.bl[1][2 - oy + 2 * ri][k]; }
#pragma unroll
        for (int oxi = 0; oxi < 5; oxi++) {
          const int sA = oxi, sB = 4 - oxi;   // 2 + ox, 2 - ox: the same parity
          uint32_t c = 0;
#pragma unroll
          for (int k = 0; k < W / 2; k++) {
            uint32_t a, b;
            if ((sA & 1) == 0) { a = A[sA / 2 + k]; b = B[sB / 2 + k]; }
            else {
              a = __builtin_amdgcn_alignbyte(A[(sA + 1) / 2 + k], A[(sA - 1) / 2 + k], 2);
              b = __builtin_amdgcn_alignbyte(B[(sB + 1) / 2 + k], B[(sB - 1) / 2 + k], 2);
            }
            c = __builtin_amdgcn_sad_u16(a, b, c);
          }
          acc[oxi] = c;
        }
      }
#pragma unroll
      for (int oxi = 0; oxi < 5; oxi++)
#pragma unroll
        for (int m = 1; m < NR; m <<= 1) acc[oxi] += __shfl_xor(acc[oxi], m);
      if (oyi < 5 && ri == 0)
#pragma unroll
        for (int oxi = 0; oxi < 5; oxi++) S.u2.d.sad[oyi * 5 + oxi] = acc[oxi];
    }
    __syncthreads();
    {
      // xDMVRCost's scan "minCost = sad'[12]; for k: if (sad[k] < minCost)" (sad'[12] = sad[12] - sad[12] / 4)
      // picks the first strict minimum, the centre on a tie: one min-reduction over the keys (cost, 0 for
      // the centre / 1 + k for the others); every lane ends with the same result
      const uint32_t c12 = S.u2.d.sad[12], adj = c12 - (c12 >> 2);
      const bool notZero = adj >= (uint32_t)(W * H);
      const uint32_t cost = lane < 25 ? (lane == 12 ? adj : S.u2.d.sad[lane]) : 0xffffffffu;
      // (a cost is below 2^17: 8 sampled rows x 16 columns of 10-bit differences, so the key fits 32 bits)
      uint32_t key = lane < 25 ? cost << 5 | (uint32_t)(lane == 12 ? 0 : lane + 1) : 0xffffffffu;
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) {
        const uint32_t o = __shfl_xor(key, m);
        key = o < key ? o : key;
      }
      key = __builtin_amdgcn_readfirstlane(key);   // lanes 0..31 hold the minimum
      unsigned long long minCost = adj;
      int tdx = 0, tdy = 0, pos = 12;
      if (notZero) {
        minCost = key >> 5;
        pos = (key & 31) ? (int)(key & 31) - 1 : 12;
        tdx = x_search[pos][0]; tdy = x_search[pos][1];
      }
      bdof = minCost < (unsigned long long)(2 * W * H) ? false : ((J.flags & MC_BDOF) != 0);
      tdx <<= 4; tdy <<= 4;
      if (notZero && abs(tdx) != 32 && abs(tdy) != 32) {
        auto sadAt = [&](int q) -> unsigned long long { return q == 12 ? adj : S.u2.d.sad[q]; };
        unsigned long long sb[5] = {sadAt(pos), sadAt(pos - 1), sadAt(pos - 5), sadAt(pos + 1), sadAt(pos + 5)};
        int d[2] = {0, 0};
        subpel_surface(sb, d);
        tdx += d[0]; tdy += d[1];
      }
      dx = __builtin_amdgcn_readfirstlane(tdx);
      dy = __builtin_amdgcn_readfirstlane(tdy);
      bdof = __builtin_amdgcn_readfirstlane((int)bdof) != 0 && !(BIDIR_ABL & 2);
      if (lane == 0 && J.aux >= 0) { dmvr_out[2 * J.aux] = dx; dmvr_out[2 * J.aux + 1] = dy; }
    }
  }

  // ---- 3. final MC (xFinalPaddedMCForDMVR / xPredInterBlk with bioApplied): the refined MV of each list,
  // its fractions and its window's offset inside the staged prefetch window
  const int MVLIM = (1 << 17) - 1;
  const int rx0 = clampi(mx0 + dx, -MVLIM - 1, MVLIM), ry0 = clampi(my0 + dy, -MVLIM - 1, MVLIM);
  const int rx1 = clampi(mx1 - dx, -MVLIM - 1, MVLIM), ry1 = clampi(my1 - dy, -MVLIM - 1, MVLIM);
  const int sx0 = (rx0 >> 4) - (mx0 >> 4), sy0 = (ry0 >> 4) - (my0 >> 4), sx1 = (rx1 >> 4) - (mx1 >> 4), sy1 = (ry1 >> 4) - (my1 >> 4);
  const int csx0 = (rx0 >> 5) - (mx0 >> 5), csy0 = (ry0 >> 5) - (my0 >> 5), csx1 = (rx1 >> 5) - (mx1 >> 5), csy1 = (ry1 >> 5) - (my1 >> 5);
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);
  constexpr int NRG = 2 * (W + 2) + 2 * H, IRG = (2 * NRG + 63) / 64;   // ring positions per list
  auto ring_pos = [](int it, int &l, int &x, int &y) {
    l = it >= NRG;
    const int q = it - (l ? NRG : 0);
    if (q < W + 2) { x = q - 1; y = -1; }
    else if (q < 2 * (W + 2)) { x = q - (W + 2) - 1; y = H; }
    else { const int k2 = q - 2 * (W + 2); y = k2 >> 1; x = (k2 & 1) ? W : -1; }
  };
  int ringv[IRG];
  {
    // luma H: lane item (list, window row r, column quad q): outputs 4q..4q+3 of row r
    constexpr int NQ = W / 4, RL = H + 7, NHL = 2 * RL * NQ;
#pragma unroll
    for (int k = 0; k < (NHL + 63) / 64; k++) {
      const int it = lane + 64 * k;
      if (it < NHL) {
        const int l = it >= RL * NQ, rem = it - (l ? RL * NQ : 0), r = rem / NQ, q = rem - r * NQ;
        const int sx = l ? sx1 : sx0, sy = l ? sy1 : sy0, ppar = (l ? px1 : px0) & 1, fx = (l ? rx1 : rx0) & 15;
        const int rr = clampi(r + sy, 0, H + 6);   // xPad: rows beyond the prefetch window repeat its edge
        const int s0 = ppar + sx + 4 * q, par = s0 & 1;
        const int16_t *row = pfs + l * (23 * 24) + rr * 24;
        uint32_t wv[6];
        if (sx + 4 * q >= 0 && sx + 4 * q + 10 <= W + 6) {
          const uint32_t *d = (const uint32_t *)row + ((s0 - par) >> 1);
#pragma unroll
          for (int e = 0; e < 6; e++) wv[e] = d[e];
        } else {   // the window's columns clamped to the prefetch window (DMVR only)
#pragma unroll
          for (int e = 0; e < 6; e++)
            wv[e] = bpk(row[ppar + clampi(sx + 4 * q - par + 2 * e, 0, W + 6)], row[ppar + clampi(sx + 4 * q - par + 2 * e + 1, 0, W + 6)]);
        }
        const uint32_t *T = c_btaps.h[alt][fx][par][0];
        int a = 0, b = 0, c = 0, e4 = 0;
#pragma unroll
        for (int m = 0; m < 5; m++) {
          a = bdot2(wv[m], T[m], a);
          b = bdot2(wv[m], T[5 + m], b);
          c = bdot2(wv[m + 1], T[m], c);
          e4 = bdot2(wv[m + 1], T[5 + m], e4);
        }
        int16_t *o = &S.u2.f.ht[l][4 * q][r];
        o[0] = (int16_t)((a + off1) >> sh1);
        o[BHT] = (int16_t)((b + off1) >> sh1);
        o[2 * BHT] = (int16_t)((c + off1) >> sh1);
        o[3 * BHT] = (int16_t)((e4 + off1) >> sh1);
      }
    }
    if (bdof) {
      // integer-sample ring (xPredInterBlk :812-846): the nearest integer position of the refined MV,
      // << headRoom, - IF_INTERNAL_OFFS, at (x, y) in -1..W x -1..H outside the block; read here, written
      // to the prediction buffers (which take the prefetch windows' storage) in the V phase
#pragma unroll
      for (int k = 0; k < IRG; k++) {
        const int it = lane + 64 * k;
        if (it < 2 * NRG) {
          int l, x, y;
          ring_pos(it, l, x, y);
          const int sx = l ? sx1 : sx0, sy = l ? sy1 : sy0, ppar = (l ? px1 : px0) & 1;
          const int xo = ((l ? rx1 : rx0) & 15) >= 8 ? 1 : 0, yo = ((l ? ry1 : ry0) & 15) >= 8 ? 1 : 0;
          const int v = pfs[l * (23 * 24) + clampi(y + yo + 3 + sy, 0, H + 6) * 24 + ppar + clampi(x + xo + 3 + sx, 0, W + 6)];
          ringv[k] = (v << headRoom) - IF_INTERNAL_OFFS;
        }
      }
    }
    // chroma H: item ((component, list) kk, window row r, column pair p)
    constexpr int NP = W / 4, RC = H / 2 + 3, NHC = (BIDIR_ABL & 4) ? 0 : 4 * RC * NP;
#pragma unroll
    for (int k = 0; k < (NHC + 63) / 64; k++) {
      const int it = lane + 64 * k;
      if (it < NHC) {
        const int kk = it / (RC * NP), rem = it - kk * (RC * NP), r = rem / NP, p = rem - r * NP;
        const int l = kk & 1;
        const int csx = l ? csx1 : csx0, csy = l ? csy1 : csy0, cpar = (l ? cx1 : cx0) & 1, cfx = (l ? rx1 : rx0) & 31;
        const int16_t *row = pcs + kk * (11 * 12) + clampi(r + csy, 0, H / 2 + 2) * 12 + cpar;
        int sm[5];
#pragma unroll
        for (int e = 0; e < 5; e++) sm[e] = row[clampi(csx + 2 * p + e, 0, W / 2 + 2)];
        const uint32_t t01 = c_btaps.c[cfx][0], t23 = c_btaps.c[cfx][1];
        const int h0 = bdot2(bpk(sm[2], sm[3]), t23, bdot2(bpk(sm[0], sm[1]), t01, 0));
        const int h1 = bdot2(bpk(sm[3], sm[4]), t23, bdot2(bpk(sm[1], sm[2]), t01, 0));
        S.u2.f.hc[kk][r][p] = bpk((h0 + off1) >> sh1, (h1 + off1) >> sh1);
      }
    }
  }
  __syncthreads();

  // one output row piece: to the prediction plane, or (MC_RECON, fused_inter_cu) clip(pred + resi) into the
  // picture (AreaBuf::reconstruct, Buffer.cpp:590); v[] already clipped to the sample range
  auto store = [&](int comp, int x, int y, int *v, int n) {
    if (J.flags & MC_RECON) {
      if (J.flags & (MC_RESI << comp)) {
        const int16_t *rs = P.resi[comp].p + (size_t)y * P.resi[comp].stride + x;
        if (n == 4) {
          const uint2 q = *(const uint2 *)rs;
          v[0] += blo(q.x); v[1] += bhi(q.x); v[2] += blo(q.y); v[3] += bhi(q.y);
        } else {
          const uint32_t q = *(const uint32_t *)rs;
          v[0] += blo(q); v[1] += bhi(q);
        }
        for (int e = 0; e < n; e++) v[e] = clampi(v[e], 0, maxv);
      }
      int16_t *d = P.reco[comp].p + (size_t)y * P.reco[comp].stride + x;
      if (n == 4) *(uint2 *)d = make_uint2(bpk(v[0], v[1]), bpk(v[2], v[3]));
      else *(uint32_t *)d = bpk(v[0], v[1]);
    } else {
      int16_t *d = P.out[comp].p + (size_t)y * P.out[comp].stride + x;
      if (n == 4) *(uint2 *)d = make_uint2(bpk(v[0], v[1]), bpk(v[2], v[3]));
      else *(uint32_t *)d = bpk(v[0], v[1]);
    }
  };
  const int shAvg = headRoom + 1, offAvg = (1 << (shAvg - 1)) + 2 * IF_INTERNAL_OFFS;
  {
    // luma V (not the last stage: sum >> IF_FILTER_PREC, 14 bits kept): item (list, column x, rows 4g..4g+3)
    // from the column's aligned vertical pairs; odd output rows through the B pairs
    if (bdof) {
#pragma unroll
      for (int k = 0; k < IRG; k++) {
        const int it = lane + 64 * k;
        if (it < 2 * NRG) {
          int l, x, y;
          ring_pos(it, l, x, y);
          S.u1.pr[l][y + 1][x + 1] = (int16_t)ringv[k];
        }
      }
    }
    constexpr int NG = H / 4, NVL = 2 * W * NG;
#pragma unroll
    for (int k = 0; k < (NVL + 63) / 64; k++) {
      const int it = lane + 64 * k;
      if (it < NVL) {
        const int l = it >= W * NG, rem = it - (l ? W * NG : 0), x = rem / NG, g = rem - x * NG;
        const int fy = (l ? ry1 : ry0) & 15;
        const uint32_t *col = (const uint32_t *)&S.u2.f.ht[l][x][4 * g];
        uint32_t D[6];
#pragma unroll
        for (int e = 0; e < 6; e++) D[e] = col[e];
        const uint32_t *VA = c_btaps.va[alt][fy], *VB = c_btaps.vb[alt][fy];
        int o0 = 0, o1 = 0, o2 = 0, o3 = 0;
#pragma unroll
        for (int m = 0; m < 4; m++) { o0 = bdot2(D[m], VA[m], o0); o2 = bdot2(D[m + 1], VA[m], o2); }
#pragma unroll
        for (int m = 0; m < 5; m++) { o1 = bdot2(D[m], VB[m], o1); o3 = bdot2(D[m + 1], VB[m], o3); }
        S.u1.pr[l][4 * g + 1][x + 1] = (int16_t)(o0 >> IF_FILTER_PREC);
        S.u1.pr[l][4 * g + 2][x + 1] = (int16_t)(o1 >> IF_FILTER_PREC);
        S.u1.pr[l][4 * g + 3][x + 1] = (int16_t)(o2 >> IF_FILTER_PREC);
        S.u1.pr[l][4 * g + 4][x + 1] = (int16_t)(o3 >> IF_FILTER_PREC);
      }
    }
    // chroma V of both lists and their average (addAvg): item (component, row y, column pair p)
    constexpr int NP = W / 4, NVC = (BIDIR_ABL & 4) ? 0 : 2 * (H / 2) * NP;
    if (lane < NVC) {
      const int comp = lane / ((H / 2) * NP), rem = lane - comp * ((H / 2) * NP), y = rem / NP, p = rem - y * NP;
      int s[2][2];
#pragma unroll
      for (int l = 0; l < 2; l++) {
        const uint32_t *hc = &S.u2.f.hc[comp * 2 + l][y][p];
        const uint32_t r0 = hc[0], r1 = hc[4], r2 = hc[8], r3 = hc[12];
        const int cfy = (l ? ry1 : ry0) & 31;
        const uint32_t t01 = c_btaps.c[cfy][0], t23 = c_btaps.c[cfy][1];
        s[l][0] = bdot2(__builtin_amdgcn_perm(r3, r2, 0x05040100u), t23, bdot2(__builtin_amdgcn_perm(r1, r0, 0x05040100u), t01, 0)) >> IF_FILTER_PREC;
        s[l][1] = bdot2(__builtin_amdgcn_perm(r3, r2, 0x07060302u), t23, bdot2(__builtin_amdgcn_perm(r1, r0, 0x07060302u), t01, 0)) >> IF_FILTER_PREC;
      }
      int v[2];
#pragma unroll
      for (int e = 0; e < 2; e++) v[e] = clampi((s[0][e] + s[1][e] + offAvg) >> shAvg, 0, maxv);
      store(1 + comp, (J.x >> 1) + 2 * p, (J.y >> 1) + y, v, 2);
    }
  }
  __syncthreads();

  // ---- luma output: lane (row y, quad q) owns samples (4q .. 4q + 3, y), row ry = y & 3 of the 4x4 unit
  // (y >> 2, q)
  constexpr int NQ = W / 4;
  const int y = lane / NQ, q = lane - y * NQ, x0 = 4 * q;
  if (!bdof) {
    if (y < H) {
      int v[4];
#pragma unroll
      for (int e = 0; e < 4; e++) v[e] = clampi((S.u1.pr[0][y + 1][x0 + e + 1] + S.u1.pr[1][y + 1][x0 + e + 1] + offAvg) >> shAvg, 0, maxv);
      store(0, J.x + x0, J.y + y, v, 4);
    }
    return;
  }
  // ---- 4. BDOF: gradients (gradFilterCore, shift 6) of the lane's samples, the window terms to LDS
  int dgx[4], dgy[4], ps[4];
  if (y < H) {
    int gx[2][4], gy[2][4], pv[2][4];
#pragma unroll
    for (int l = 0; l < 2; l++) {
      const int16_t *c = &S.u1.pr[l][y + 1][x0];
      int m[6];
#pragma unroll
      for (int e = 0; e < 6; e++) m[e] = c[e];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        pv[l][e] = m[e + 1];
        gx[l][e] = (m[e + 2] >> 6) - (m[e] >> 6);
        gy[l][e] = (c[BPR + e + 1] >> 6) - (c[-BPR + e + 1] >> 6);
      }
    }
    int tg[3][4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      tg[0][e] = (gx[0][e] + gx[1][e]) >> 1;
      tg[1][e] = (gy[0][e] + gy[1][e]) >> 1;
      tg[2][e] = (pv[1][e] >> 4) - (pv[0][e] >> 4);
      dgx[e] = gx[0][e] - gx[1][e];
      dgy[e] = gy[0][e] - gy[1][e];
      ps[e] = pv[0][e] + pv[1][e];
    }
#pragma unroll
    for (int t = 0; t < 3; t++) {
      uint32_t *d = (uint32_t *)&S.u2.t[t][y][x0];
      d[0] = bpk(tg[t][0], tg[t][1]);
      d[1] = bpk(tg[t][2], tg[t][3]);
    }
  }
  __syncthreads();
  // the unit's 6x6 window sums (calcBIOSumsCore): this lane's window rows (ry 0: -1, 0; 1: 1; 2: 2; 3: 3, 4),
  // positions outside the block at the nearest sample inside (the reference pads gradients and predictions)
  int sGX = 0, sGY = 0, sDIX = 0, sDIY = 0, sSGG = 0;
  if (y < H) {
    const int ry = y & 3, uy0 = y - ry;
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int wy = ry == 0 ? t - 1 : (ry == 3 ? 3 + t : ry);
      if (t == 1 && ry != 0 && ry != 3) break;
      const int Y = clampi(uy0 + wy, 0, H - 1);
#pragma unroll
      for (int e = -1; e < 5; e++) {
        const int X = clampi(x0 + e, 0, W - 1);
        const int tGX = S.u2.t[0][Y][X], tGY = S.u2.t[1][Y][X], tDI = S.u2.t[2][Y][X];
        sGX += abs(tGX);
        sGY += abs(tGY);
        sDIX += tGX < 0 ? -tDI : (tGX == 0 ? 0 : tDI);
        sDIY += tGY < 0 ? -tDI : (tGY == 0 ? 0 : tDI);
        sSGG += tGY < 0 ? -tGX : (tGY == 0 ? 0 : tGX);
      }
    }
  }
  // the four lanes of a unit (rows ry = 0..3: lanes NQ apart)
#pragma unroll
  for (int m = NQ; m < 4 * NQ; m <<= 1) {
    sGX += __shfl_xor(sGX, m);
    sGY += __shfl_xor(sGY, m);
    sDIX += __shfl_xor(sDIX, m);
    sDIY += __shfl_xor(sDIY, m);
    sSGG += __shfl_xor(sSGG, m);
  }
  if (y < H) {
    const int limit = 15;   // applyBiOptFlow :1338-1351
    int vx = sGX == 0 ? 0 : (sDIX << 2) >> (31 - __clz(sGX));
    vx = clampi(vx, -limit, limit);
    const int mains = sSGG >> 12, secs = sSGG & 4095;
    const int tmpData = ((vx * mains) * (1 << 12) + vx * secs) >> 1;
    int vy = sGY == 0 ? 0 : ((sDIY << 2) - tmpData) >> (31 - __clz(sGY));
    vy = clampi(vy, -limit, limit);
    const int shiftNum = IF_INTERNAL_PREC + 1 - bd, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int b = vx * dgx[e] + vy * dgy[e];
      v[e] = clampi((int16_t)((ps[e] + b + offset) >> shiftNum), 0, maxv);
    }
    store(0, J.x + x0, J.y + y, v, 4);
  }
}

// A job of one of the batch's pictures per workgroup (picture p: blocks [job0[p], job0[p + 1]))
__global__ __launch_bounds__(64) void k_mc_bidir(ExtBatch B) {
  __shared__ BidirLds S;
  // XCD runs of 32 jobs (xcd_run_swizzle): neighbouring jobs' reference windows share an L2
#if BIDIR_XCD_RUN > 0
  const int j = xcd_run_swizzle((int)blockIdx.x, (int)gridDim.x, BIDIR_XCD_RUN);
#else
  const int j = blockIdx.x;
#endif
  if (j >= B.job0[B.npic]) return;
  int p = 0;
#pragma unroll
  for (int q = 1; q < MC_MAXPIC; q++)
    if (q < B.npic && j >= B.job0[q]) p = q;
  const McParams &P = B.pic[p];   // (p uniform: scalar-offset reads of the kernel argument)
  int32_t *dmvr_out = B.dmvr[p];
  const McJob J = load_uniform((const McJob *)B.jobs[p] + (j - B.job0[p]));
  // block sizes: DMVR sub-blocks and xSubPuBio tiles of PUs with w, h >= 8 and w * h >= 128 (the host checks
  // multiples of 8): 16x16, 16x8, 8x16; 8x8 is not produced by the reference's conditions but handled
  if (J.w == 16 && J.h == 16) bidir_block<16, 16>(P, J, dmvr_out, S);
  else if (J.w == 16) bidir_block<16, 8>(P, J, dmvr_out, S);
  else if (J.h == 16) bidir_block<8, 16>(P, J, dmvr_out, S);
  else bidir_block<8, 8>(P, J, dmvr_out, S);
}

}  // namespace

void launch_mc_bidir(ExtBatch &b, hipStream_t s) {
  b.job0[0] = 0;
  for (int p = 0; p < MC_MAXPIC; p++) b.job0[p + 1] = b.job0[p] + (p < b.npic ? b.njobs[p] : 0);
  const int n = b.job0[b.npic];
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mc_bidir, dim3(n), dim3(BIDIR_WG), 0, s, b);
}
