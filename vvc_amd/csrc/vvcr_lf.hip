// vvcr_lf.hip — in-loop filters for gfx950: SAO and ALF / CC-ALF (deblocking: vvcr_dbk.hip).
//
// SAO (SampleAdaptiveOffset::offsetBlock, SampleAdaptiveOffset.cpp:293): one lane per 8 horizontally
// adjacent samples of one component; every sample of the picture is written (copy where SAO is off),
// reading the deblocked picture and writing the SAO picture (ping-pong, so neighbours are pre-SAO).
//
// ALF (AdaptiveLoopFilter::deriveClassificationBlk :873, filterBlk<7x7/5x5> :1085, filterBlkCcAlf :1328):
// one workgroup per 64x16 luma region and its 32x8 chroma, all three planes staged in LDS with their
// halos (classification + 7x7 luma filter, 5x5 chroma filter + CC-ALF from the staged luma).
// Reads the SAO picture, writes the final picture. Coordinates are clamped to the picture
// (equivalent to PelUnitBuf::extendBorderPel(3) on the ALF input, AdaptiveLoopFilter.cpp:411).
#include "vvcr_internal.h"

#ifdef VVCR_ALF_PROF
// Diagnostics build only (tools/alf_prof.py): per-workgroup phase stamps (s_memrealtime, 100 MHz) of k_alf.
__device__ unsigned long long g_alfprof[1 << 15][6];
extern "C" int vvcr_alf_prof_read(unsigned long long *dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_alfprof), (size_t)n * 6 * 8);
}
#define ALF_STAMP(k) do { if (threadIdx.x == 0) stamp[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define ALF_STAMP(k) do { } while (0)
#endif
namespace {

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
typedef short short2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// One lane per 8 horizontally adjacent samples (a 16-byte vector) of one component, a wave per row, four
// rows per workgroup. The lane's row and both neighbour rows are loaded as vectors, with the samples
// left / right of them, all before the CTB's parameters are known; the 8 samples lie in one CTB (CTB
// widths are multiples of 8). The edge-offset classes read their neighbours from these registers.
__global__ __launch_bounds__(256) void k_sao(SaoParams P) {
  const int comp = blockIdx.z;               // one launch for the three planes
  const DPlane &S = P.src[comp];
  const DPlane &D = P.dst[comp];
  const int W = S.w, H = S.h;
  const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 8;
  const int y = (comp ? P.y0 >> 1 : P.y0) + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x0 >= W || y >= H || y >= (comp ? P.y1 >> 1 : P.y1)) return;
  const int cs = comp ? P.ctu >> 1 : P.ctu;
  const int maxv = (1 << P.bd) - 1;
  const int ya = max(y - 1, 0), yb = min(y + 1, H - 1);
  const int16_t *rc = S.p + (size_t)y * S.stride, *ra = S.p + (size_t)ya * S.stride, *rb = S.p + (size_t)yb * S.stride;
  const int xl = max(x0 - 1, 0), xr = min(x0 + 8, W - 1);
  // rows as [x0 - 1 .. x0 + 8] (plane rows are 64-sample pitched: the vector stays inside the row)
  const uint4 vc = *(const uint4 *)(rc + x0), va = *(const uint4 *)(ra + x0), vb = *(const uint4 *)(rb + x0);
  int C[10], A[10], B[10];
  C[0] = rc[xl]; C[9] = rc[xr]; A[0] = ra[xl]; A[9] = ra[xr]; B[0] = rb[xl]; B[9] = rb[xr];
  const int ctb = (y / cs) * P.wc + x0 / cs;
  const int32_t *prm = P.sao + ((size_t)ctb * 3 + comp) * 35;
  // tiles / slices not filtered across: the CTB's neighbour availability (deriveLoopFilterBoundaryAvailibility,
  // SampleAdaptiveOffset.cpp:668-718); offsetBlock (:293-547) modifies a sample only when both samples its class
  // compares it with lie in available CTBs
  const int nbm = P.nb ? P.nb[ctb] : 0xff;
  const int bx0 = (x0 / cs) * cs, by0 = (y / cs) * cs;
  const int on = prm[0], type = prm[1];
  const int e0 = prm[3], e1 = prm[4], e2 = prm[5], e3 = prm[6], e4 = prm[7];
  {
    const uint32_t wc[4] = {vc.x, vc.y, vc.z, vc.w}, wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      C[1 + 2 * k] = (int16_t)(wc[k] & 0xffff); C[2 + 2 * k] = (int16_t)(wc[k] >> 16);
      A[1 + 2 * k] = (int16_t)(wa[k] & 0xffff); A[2 + 2 * k] = (int16_t)(wa[k] >> 16);
      B[1 + 2 * k] = (int16_t)(wb[k] & 0xffff); B[2 + 2 * k] = (int16_t)(wb[k] >> 16);
    }
  }
  int v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = C[1 + k];
  if (on) {
    if (type == 4) {   // band offset
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = clip3(0, maxv, v[k] + prm[3 + (v[k] >> (P.bd - 5))]);
    } else {
      // neighbours per EO class: 0 horizontal, 1 vertical, 2 135 degrees, 3 45 degrees
      const int dax = type == 1 ? 0 : (type == 3 ? 1 : -1), day = type == 0 ? 0 : -1;
      const bool rowsIn = day == 0 || (y - 1 >= 0 && y + 1 < H);
      // the CTB offsets of row y + day / y - day
      const int oya = y + day < by0 ? -1 : (y + day >= by0 + cs ? 1 : 0), oyb = y - day < by0 ? -1 : (y - day >= by0 + cs ? 1 : 0);
      auto avail = [&](int ox, int oy) {   // bit of neighbour CTB (ox, oy): L R A B AL AR BL BR (vvcr_host.h LFNB_*)
        const int bit = oy == 0 ? (ox < 0 ? 0 : 1) : (ox == 0 ? (oy < 0 ? 2 : 3) : (oy < 0 ? (ox < 0 ? 4 : 5) : (ox < 0 ? 6 : 7)));
        return (ox == 0 && oy == 0) || ((nbm >> bit) & 1);
      };
      // virtual boundaries (SampleAdaptiveOffset::isProcessDisabled, SampleAdaptiveOffset.cpp:96-116): no
      // edge offset on the samples either side of one the class compares across (horizontal class: the
      // vertical boundaries, vertical class: the horizontal ones, diagonal classes: both)
      bool vbRow = false;
      const int vsh = comp ? 1 : 0;
#pragma unroll
      for (int i = 0; i < 3; i++)
        if (type != 0 && i < P.nvb[1]) { const int v = P.vb[1][i] >> vsh; vbRow |= y == v || y == v - 1; }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int x = x0 + k;
        bool vbCol = false;
#pragma unroll
        for (int i = 0; i < 3; i++)
          if (type != 1 && i < P.nvb[0]) { const int v = P.vb[0][i] >> vsh; vbCol |= x == v || x == v - 1; }
        const int a = type == 0 ? C[k] : (type == 1 ? A[1 + k] : (type == 2 ? A[k] : A[2 + k]));
        const int b = type == 0 ? C[2 + k] : (type == 1 ? B[1 + k] : (type == 2 ? B[2 + k] : B[k]));
        const int oxa = x + dax < bx0 ? -1 : (x + dax >= bx0 + cs ? 1 : 0), oxb = x - dax < bx0 ? -1 : (x - dax >= bx0 + cs ? 1 : 0);
        const bool in = rowsIn && x + dax >= 0 && x + dax < W && x - dax >= 0 && x - dax < W && x < W && avail(oxa, oya) && avail(oxb, oyb);
        const int s0 = v[k], ei = 2 + sgn(s0 - a) + sgn(s0 - b);
        const int off = ei == 0 ? e0 : (ei == 1 ? e1 : (ei == 2 ? e2 : (ei == 3 ? e3 : e4)));
        if (in && !vbRow && !vbCol) v[k] = clip3(0, maxv, s0 + off);
      }
    }
  }
  int16_t *out = D.p + (size_t)y * D.stride + x0;
  if (x0 + 8 <= W) {
    *(uint4 *)out = make_uint4((uint32_t)(uint16_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)(uint16_t)v[2] | ((uint32_t)v[3] << 16),
                               (uint32_t)(uint16_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)(uint16_t)v[6] | ((uint32_t)v[7] << 16));
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (x0 + k < W) out[k] = (int16_t)v[k];
  }
}

__device__ __forceinline__ int at(const DPlane &p, int x, int y) {
  x = x < 0 ? 0 : (x >= p.w ? p.w - 1 : x);
  y = y < 0 ? 0 : (y >= p.h ? p.h - 1 : y);
  return p.p[(size_t)y * p.stride + x];
}
// min / max (one v_med3_i32 each), not clip3's compare-and-select
__device__ __forceinline__ int clip_alf(int c, int ref, int v0, int v1) {
  return min(max(v0 - ref, -c), c) + min(max(v1 - ref, -c), c);
}

// Rows of the diamond's taps at distance 1..3 below (r1, r3, r5) / above (r2, r4, r6) row y, padded at
// the ALF virtual boundary (AdaptiveLoopFilter.cpp filterBlk); all selects (conditional assignments
// through references were lowered to scratch stores).
__device__ __forceinline__ void alf_rows(int y, int vbH, int vbPos, bool luma, int &r1, int &r2, int &r3, int &r4, int &r5, int &r6) {
  const int yVb = y & (vbH - 1);
  const bool up = yVb < vbPos && yVb >= vbPos - (luma ? 4 : 2);     // rows above the boundary
  const bool dn = yVb >= vbPos && yVb <= vbPos + (luma ? 3 : 1);    // rows below it
  const bool e1 = up ? yVb == vbPos - 1 : (dn && yVb == vbPos);
  const bool e2 = up ? yVb >= vbPos - 2 : (dn && yVb <= vbPos + 1);
  const bool e3 = up ? yVb >= vbPos - 3 : (dn && yVb <= vbPos + 2);
  const int a1 = e1 ? y : y + 1, b1 = e1 ? y : y - 1;
  const int a3 = e2 ? a1 : y + 2, b3 = e2 ? b1 : y - 2;
  const int a5 = e3 ? a3 : y + 3, b5 = e3 ? b3 : y - 3;
  r1 = a1; r2 = b1; r3 = a3; r4 = b3; r5 = a5; r6 = b5;
}

__constant__ int8_t c_perm7[4][13] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12},
                                      {9, 4, 10, 8, 1, 5, 11, 7, 3, 0, 2, 6, 12},
                                      {0, 3, 2, 1, 8, 7, 6, 5, 4, 9, 10, 11, 12},
                                      {9, 8, 10, 4, 3, 7, 11, 5, 1, 0, 2, 6, 12}};

// ALF of one region: 64x16 luma samples and the co-located 32x8 Cb and Cr samples, one 256-lane
// workgroup. The luma tile with its 3-sample halo and both chroma tiles with their 2-sample halo are staged
// in LDS once, by 16-byte loads of aligned 8-sample chunks (picture-clamped coordinates); then
//   luma: four lanes classify each 4x4 block (one subsampled row pair each, reduced by shuffles), then
//         each lane filters one column of one 4x4 block (7x7 diamond, packed 16-bit arithmetic);
//   chroma: one lane per chroma position filters Cb and Cr (5x5 diamond) and adds the CC-ALF correction,
//         whose luma taps (the same for both components) come from the staged luma tile.
// Work is dispatched in XCD-contiguous runs of regions (xcd_swizzle), so the halo rows and columns a
// region shares with its neighbours are fetched from HBM once per XCD, and the chroma work of a region
// reads the luma its own workgroup staged (before r04 the chroma work was dispatched after all luma
// tiles and re-read the luma from HBM: 3.2x the algorithmic bytes).
// diagnostics only (timing ablations, wrong output): skip the classification sums / the luma taps / chroma
#ifndef ALF_ABL_CLASS
#define ALF_ABL_CLASS 0
#endif
#ifndef ALF_ABL_LUMA
#define ALF_ABL_LUMA 0
#endif
#ifndef ALF_ABL_CHROMA
#define ALF_ABL_CHROMA 0
#endif
#ifndef ALF_ROWS
#define ALF_ROWS 16   // region height (16 or 32; at most the CTU size, so a region lies in one CTB)
#endif
constexpr int ALF_TW = 64, ALF_TH = ALF_ROWS, ALF_HALO = 3;
constexpr int ALF_LX = 8;                            // staged luma columns left of the tile (one chunk)
constexpr int ALF_SW = ALF_TW + 2 * ALF_LX;          // LDS row pitch (80): chunks [X0 - 8, X0 + 72)
constexpr int ALF_SH = ALF_TH + 2 * ALF_HALO;        // 22 rows
constexpr int ALF_LCH = ALF_SW / 8;                  // luma chunks per row (10)
constexpr int ALF_CW = ALF_TW / 2, ALF_CHH = ALF_TH / 2;   // chroma region 32 x 8
constexpr int ALF_CSW = ALF_CW + 16, ALF_CSH = ALF_CHH + 4; // chroma LDS: chunks [cx0 - 8, cx0 + 40), rows cy0 - 2 .. cy0 + 9
constexpr int ALF_CCH = ALF_CSW / 8;                 // chroma chunks per row (6)
constexpr int ALF_LQ = (ALF_SH * ALF_LCH + 255) / 256;   // staged luma chunks per lane
static_assert(2 * ALF_CSH * ALF_CCH <= 256, "one chroma chunk per lane");

// 8 samples of row y from column x0 (a multiple of 8), clamped to columns [xl, xh) and rows [yl, yh): the
// picture, or the CTB's sides that border tiles / slices not filtered across (one vector load when inside)
__device__ __forceinline__ uint4 alf_chunk(const DPlane &S, int x0, int y, int xl, int xh, int yl, int yh) {
  const int16_t *row = S.p + (size_t)clip3(yl, yh - 1, y) * S.stride;
  if (x0 >= xl && x0 + 8 <= xh) return *(const uint4 *)(row + x0);
  int v[8];
#pragma unroll
  for (int e = 0; e < 8; e++) v[e] = row[clip3(xl, xh - 1, x0 + e)];
  return make_uint4((uint32_t)(uint16_t)v[0] | (uint32_t)v[1] << 16, (uint32_t)(uint16_t)v[2] | (uint32_t)v[3] << 16,
                    (uint32_t)(uint16_t)v[4] | (uint32_t)v[5] << 16, (uint32_t)(uint16_t)v[6] | (uint32_t)v[7] << 16);
}

// Uniform loads of a per-CTB control byte / short through the scalar cache (the containing aligned dword,
// constant address space: s_load). A vector load here would share the in-order vmcnt counter with the
// sample chunks in flight, so waiting for the control value would wait for the HBM loads too.
typedef const __attribute__((address_space(4))) uint32_t *cdword_t;
__device__ __forceinline__ int ldc_u8(const uint8_t *base, int i) {
  const uintptr_t a = (uintptr_t)(base + i);
  const uint32_t w = *(cdword_t)(a & ~(uintptr_t)3);
  return (int)((w >> ((a & 3) * 8)) & 0xff);
}
__device__ __forceinline__ int ldc_i16(const int16_t *base, int i) {
  const uintptr_t a = (uintptr_t)(base + i);
  const uint32_t w = *(cdword_t)(a & ~(uintptr_t)3);
  return (int)(int16_t)(w >> ((a & 2) * 8));
}

// The sub-rectangle between virtual boundaries that contains position p (luma samples; chroma: c = 1):
// [lo, hi]. With loop filtering across virtual boundaries disabled, VTM filters every such sub-rectangle of a
// CTB from a copy extended by edge replication (AdaptiveLoopFilter::ALFProcess :458-483), i.e. a tap
// outside it reads the nearest sample inside: a coordinate clamp.
__device__ __forceinline__ void vb_span(const AlfParams &P, int d, int c, int p, int &lo, int &hi) {
  lo = -(1 << 20);
  hi = 1 << 20;
#pragma unroll
  for (int i = 0; i < 3; i++)
    if (i < P.nvb[d]) {
      const int v = P.vb[d][i] >> c;
      if (v <= p) lo = max(lo, v);
      else hi = min(hi, v - 1);
    }
}

template <bool VB>
__device__ __forceinline__ void alf_region(const AlfParams &P, int tx, int ty, unsigned long long *stamp) {
  const DPlane &S = P.src[0];
  const DPlane &D = P.dst[0];
  __shared__ __attribute__((aligned(16))) int16_t t[ALF_SH * ALF_SW];
  __shared__ __attribute__((aligned(16))) int16_t tc[2][ALF_CSH * ALF_CSW];
  // the CTB's filter set per class, packed for the tap arithmetic: (c, c), (l, l), (-l, -l)
  __shared__ uint2 s_cc[25 * 13];   // .x (c, c)  .y (l, l): one 8-byte LDS read per tap (ds_read_b64)
  __shared__ int8_t s_perm[4 * 13];
  // the CTB's chroma filters (per component: (c, c), (l, l) per tap pair) and CC-ALF filters
  __shared__ uint2 s_ch[2][6];
  __shared__ int32_t s_cc8[2][8];
  const int X0 = tx * ALF_TW, Y0 = P.y0 + ty * ALF_TH;
  const int cx0 = X0 >> 1, cy0 = Y0 >> 1;
  const int tid = threadIdx.x;
  const int W = S.w, H = S.h;
  // every staging load in flight first (one memory round trip): a luma chunk per lane (220 of them) and a
  // chroma chunk for 144 lanes; then the CTB's controls (a 64x16 tile lies in one CTB, so they are
  // uniform: scalar loads) and the filters they select (the luma set's 25 classes of coefficients / clips,
  // both chroma filters, both CC-ALF filters), staged in LDS with the samples
  // the sample bounds: the picture, or with tiles / slices not filtered across the CTB's clipped sides
  // (AdaptiveLoopFilter::isCrossedByVirtualBoundaries :121-170: the CTB is filtered from a copy extended by
  // edge replication there, as at the picture's edges)
  int xl = 0, xh = W, yl = 0, yh = H;
  const int ctu = 1 << P.ctu_log2, bx = X0 & ~(ctu - 1), by = Y0 & ~(ctu - 1);
  // raster-slice corner padding (AdaptiveLoopFilter.cpp:172-198 with AreaBuf::padBorderPel): the rows above
  // the CTB take their samples left of it from its first column, the rows below it those right of it from its
  // last column
  int pf = 0;
  if (P.nb) {
    const int k = (Y0 >> P.ctu_log2) * P.wc + (X0 >> P.ctu_log2);
    const int m = ldc_u8(P.nb, k);
    if (P.pad) pf = ldc_u8(P.pad, k);
    if (!(m & 1)) xl = bx;
    if (!(m & 2)) xh = min(W, bx + ctu);
    if (!(m & 4)) yl = by;
    if (!(m & 8)) yh = min(H, by + ctu);
  }
  auto row_xl = [&](int y, int sh) { return (pf & 1) && y < (by >> sh) ? max(xl >> sh, bx >> sh) : xl >> sh; };
  auto row_xh = [&](int y, int sh) { return (pf & 2) && y >= ((by + ctu) >> sh) ? min(xh >> sh, (bx + ctu) >> sh) : xh >> sh; };
  uint4 lv[ALF_LQ] = {}, cv = {};
#pragma unroll
  for (int q = 0; q < ALF_LQ; q++) {
    const int i = tid + 256 * q, lr = i / ALF_LCH, lc = i - lr * ALF_LCH, y = Y0 - ALF_HALO + lr;
    if (i < ALF_SH * ALF_LCH) lv[q] = alf_chunk(S, X0 - ALF_LX + 8 * lc, y, row_xl(y, 0), row_xh(y, 0), yl, yh);
  }
  const int ccomp = tid / (ALF_CSH * ALF_CCH), ci = tid - ccomp * (ALF_CSH * ALF_CCH);
  const int cr = ci / ALF_CCH, cc = ci - cr * ALF_CCH;
  {
    // Cb and Cr share stride and size: select the base pointer per lane from the two uniform descriptors
    // (a lane-indexed P.src[1 + ccomp] is a per-lane load of the descriptor, one more memory round trip)
    DPlane cs = P.src[1];
    cs.p = ccomp ? P.src[2].p : P.src[1].p;
    const int y = cy0 - 2 + cr;
    if (ccomp < 2) cv = alf_chunk(cs, cx0 - 8 + 8 * cc, y, row_xl(y, 1), row_xh(y, 1), yl >> 1, yh >> 1);
  }
  const int ctbT = (Y0 >> P.ctu_log2) * P.wc + (X0 >> P.ctu_log2);
  const int n = P.nctb;
  // every per-CTB control of the region in one round trip (all independent, uniform), then every filter
  // it selects in a second one, both while the sample chunks are in flight
  // (unconditional: a load under a condition is waited for inside it, together with the chunks)
  const int ctbE = ldc_u8(P.ctb_en, ctbT), set0 = ldc_i16(P.ctb_set, ctbT);
  const int eCb = ldc_u8(P.ctb_en, n + ctbT), eCr = ldc_u8(P.ctb_en, 2 * n + ctbT);
  const int altCb = ldc_u8(P.ctb_alt, n + ctbT), altCr = ldc_u8(P.ctb_alt, 2 * n + ctbT);
  const int fCb = ldc_u8(P.cc_ctl, ctbT), fCr = ldc_u8(P.cc_ctl, n + ctbT);
  const bool ctbOn = P.en[0] && ctbE;
  const int onCb = P.en[1] && eCb, onCr = P.en[2] && eCr;
  const int ccCb = P.en[3] ? fCb : 0, ccCr = P.en[4] ? fCr : 0;
  const int set = ctbOn ? set0 : 0;
  constexpr int NC = (25 * 13 + 255) / 256;
  int16_t cfv[NC], clv[NC];
  {
    const int16_t *cf = P.luma_coef + set * 25 * 13, *cl = P.luma_clip + set * 25 * 13;
#pragma unroll
    for (int q = 0; q < NC; q++) {
      const int i = min(tid + 256 * q, 25 * 13 - 1);
      cfv[q] = cf[i];
      clv[q] = cl[i];
    }
  }
  // chroma filter taps and CC-ALF taps: lane & 15 = component (bit 3) and tap (bits 0..2)
  const int ck = (tid >> 3) & 1, ctt = tid & 7;
  const int calt = min(ck ? altCr : altCb, 7), cf_ = ck ? ccCr : ccCb;
  const int chc = P.chroma_coef[calt * 7 + min(ctt, 6)], chl = P.chroma_clip[calt * 7 + min(ctt, 6)];
  const int ccv = P.cc_coef[(ck * 4 + max(cf_ - 1, 0)) * 8 + ctt];
#pragma unroll
  for (int q = 0; q < ALF_LQ; q++) {
    const int i = tid + 256 * q, lr = i / ALF_LCH, lc = i - lr * ALF_LCH;
    if (i < ALF_SH * ALF_LCH) *(uint4 *)&t[lr * ALF_SW + 8 * lc] = lv[q];
  }
  if (ccomp < 2) *(uint4 *)&tc[ccomp][cr * ALF_CSW + 8 * cc] = cv;
  if (ctbOn) {
#pragma unroll
    for (int q = 0; q < NC; q++) {
      const int i = tid + 256 * q;
      if (i < 25 * 13) {
        const uint32_t c = (uint16_t)cfv[q], l = (uint16_t)clv[q];
        s_cc[i] = make_uint2(c | c << 16, l | l << 16);
      }
    }
    if (tid < 4 * 13) s_perm[tid] = (&c_perm7[0][0])[tid];
  }
  if (tid < 16) {
    const uint32_t c = (uint16_t)chc, l = (uint16_t)chl;
    if (ctt < 6) s_ch[ck][ctt] = make_uint2(c | c << 16, l | l << 16);
    s_cc8[ck][ctt] = ccv;
  }
  __syncthreads();
  ALF_STAMP(1);
  // sample (x, y) in picture coordinates -> LDS (valid for x in [X0 - 8, X0 + 72), y in [Y0 - 3, Y0 + 19));
  // with virtual boundaries (VB: the picture has some) clamped to the sub-rectangle [vxl, vxh] x [vyl, vyh]
  // of the sample being classified / filtered
  int vxl = 0, vxh = 0, vyl = 0, vyh = 0;
#define VCX(x) (VB ? min(max((x), vxl), vxh) : (x))
#define VCY(y) (VB ? min(max((y), vyl), vyh) : (y))
#define T(x, y) ((int)t[(VCY(y) - Y0 + ALF_HALO) * ALF_SW + VCX(x) - X0 + ALF_LX])
  const int vbH = 1 << P.ctu_log2, vbPos = P.vb_luma;
  // Classification and filtering of a 4x4 block run on the same four lanes: lane (block b, ii) classifies
  // the block's subsampled row pair ii, the four partial sums are reduced across the lane quad (DPP), every
  // lane of the quad derives the class, and then filters the block's column ii (no class table in LDS,
  // no barrier between the two).
  for (int b = tid >> 2; b < (ALF_TW / 4) * (ALF_TH / 4); b += 64) {
    // --- classification (deriveClassificationBlk): block b, subsampled row pair ii
    const int ii = tid & 3;
    const int bx = X0 + (b & 15) * 4, by = Y0 + (b >> 4) * 4;
    if (VB) {   // a 4x4 block lies in one sub-rectangle (virtual boundaries are multiples of 8)
      vb_span(P, 0, 0, bx, vxl, vxh);
      vb_span(P, 1, 0, by, vyl, vyh);
    }
    const bool on = bx < W && by < H && ctbOn;
    int sumV = 0, sumH = 0, sumD0 = 0, sumD1 = 0;
    const int yv = by & (vbH - 1);
    const int i0 = (yv == vbPos) ? 1 : 0, i1 = (yv == vbPos - 4) ? 3 : 4;
    if (!ALF_ABL_CLASS && on && ii >= i0 && ii < i1) {
      const int ay = by - 2 + ii * 2;
      int rA = ay - 1, rB = ay + 1, rB2 = ay + 2;
      if (ay > 0 && (ay & (vbH - 1)) == vbPos - 2) rB2 = ay + 1;
      else if (ay > 0 && (ay & (vbH - 1)) == vbPos) rA = ay;
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        const int ax = bx - 2 + jj * 2;
        // |2 c - n1 - n2| as one v_sad_u16 each (all terms are non-negative and below 2^16)
        const uint32_t a = T(ax, ay) << 1, bb = T(ax + 1, ay + 1) << 1;
        auto sad = [](uint32_t c, int n1, int n2, int acc) { return (int)__builtin_amdgcn_sad_u16(c, (uint32_t)(n1 + n2), (uint32_t)acc); };
        sumV = sad(a, T(ax, rA), T(ax, rB), sad(bb, T(ax + 1, ay), T(ax + 1, rB2), sumV));
        sumH = sad(a, T(ax + 1, ay), T(ax - 1, ay), sad(bb, T(ax + 2, rB), T(ax, rB), sumH));
        sumD0 = sad(a, T(ax - 1, rA), T(ax + 1, rB), sad(bb, T(ax, ay), T(ax + 2, rB2), sumD0));
        sumD1 = sad(a, T(ax - 1, rB), T(ax + 1, rA), sad(bb, T(ax, rB2), T(ax + 2, ay), sumD1));
      }
    }
    // quad sums: DPP quad_perm [1,0,3,2] then [2,3,0,1] (VALU only; a shuffle is an LDS instruction)
    auto quad_sum = [](int v) {
      v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);
      return v + __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);
    };
    sumV = quad_sum(sumV); sumH = quad_sum(sumH); sumD0 = quad_sum(sumD0); sumD1 = quad_sum(sumD1);
    const int x = bx + ii;
    if (bx >= W || by >= H) continue;
    int16_t *dst = D.p + x;
    if (!on) {
      for (int y = by; y < by + 4 && y < H; y++) dst[(size_t)y * D.stride] = (int16_t)T(x, y);
      continue;
    }
    int classIdx, tr;
    {
      const int shift = P.bd + 4;
      const int act = clip3(0, 15, ((sumV + sumH) * ((yv == vbPos - 4 || yv == vbPos) ? 96 : 64)) >> shift);
      // c_th / c_transpose as packed immediates (a lane-indexed __constant__ table is a vector load)
      classIdx = (int)((0x4333333332222210ull >> (4 * act)) & 15);   // th[16] = {0,1,2,2,2,2,2,3,...,3,4}
      int hv1, hv0, d1, d0, dirHV, dirD, mainDir, secDir;
      if (sumV > sumH) { hv1 = sumV; hv0 = sumH; dirHV = 1; } else { hv1 = sumH; hv0 = sumV; dirHV = 3; }
      if (sumD0 > sumD1) { d1 = sumD0; d0 = sumD1; dirD = 0; } else { d1 = sumD1; d0 = sumD0; dirD = 2; }
      int hvd1, hvd0;
      if ((uint32_t)d1 * (uint32_t)hv0 > (uint32_t)hv1 * (uint32_t)d0) { hvd1 = d1; hvd0 = d0; mainDir = dirD; secDir = dirHV; }
      else { hvd1 = hv1; hvd0 = hv0; mainDir = dirHV; secDir = dirD; }
      int strength = 0;
      if (hvd1 > 2 * hvd0) strength = 1;
      if (hvd1 * 2 > 9 * hvd0) strength = 2;
      if (strength) classIdx += (((mainDir & 1) << 1) + strength) * 5;
      tr = (0xDE84 >> (2 * (mainDir * 2 + (secDir >> 1)))) & 3;        // transpose[8] = {0,1,0,2,2,3,1,3}
    }
    {
      {
        const uint2 *cc = s_cc + classIdx * 13;
        // packed 16-bit arithmetic: the two samples of a tap pair as one int16x2 (differences to the centre
        // fit 16 bits, clips <= 1 << bd), clipped with packed min / max, then one dot2 with the coefficient
        // pair (c, c): exactly c * clip(a - cur) + c * clip(b - cur)
        short2_t fcp[12], clp[12], cln[12];
#pragma unroll
        for (int k = 0; k < 12; k++) {
          const int pk = s_perm[tr * 13 + k];
          const uint2 e = cc[pk];
          fcp[k] = __builtin_bit_cast(short2_t, e.x);
          clp[k] = __builtin_bit_cast(short2_t, e.y);
          cln[k] = (short2_t){0, 0} - clp[k];
        }
        const int maxv = (1 << P.bd) - 1;
        const int yb = by & (vbH - 1);
        if (!VB && yb != vbPos - 4 && yb != vbPos) {
          // no row of this 4x4 block (one per wave: wave-uniform) touches the virtual boundary: every tap at a
          // constant LDS offset from the block's column (immediate ds_read offsets, no row arithmetic)
          // based at the window's top-left sample: every tap offset non-negative (ds_read offsets are unsigned)
          const int16_t *c0 = &t[(by - Y0) * ALF_SW + (x - X0) + ALF_LX - 3];
#define TT(dx, dy) ((int)c0[((dy) + 3) * ALF_SW + (dx) + 3])
#pragma unroll
          for (int dy = 0; dy < 4; dy++) {
            if (by + dy >= H) break;
            const int cur = TT(0, dy);
            const short2_t cc2 = {(short)cur, (short)cur};
            int sum = 0;
            auto tap = [&](int k, int a, int b) {
              short2_t d = (short2_t){(short)a, (short)b} - cc2;
              d = __builtin_elementwise_min(__builtin_elementwise_max(d, cln[k]), clp[k]);
              sum = __builtin_amdgcn_sdot2(d, fcp[k], sum, true);
            };
#if !ALF_ABL_LUMA
            tap(0, TT(0, dy + 3), TT(0, dy - 3));
            tap(1, TT(1, dy + 2), TT(-1, dy - 2));
            tap(2, TT(0, dy + 2), TT(0, dy - 2));
            tap(3, TT(-1, dy + 2), TT(1, dy - 2));
            tap(4, TT(2, dy + 1), TT(-2, dy - 1));
            tap(5, TT(1, dy + 1), TT(-1, dy - 1));
            tap(6, TT(0, dy + 1), TT(0, dy - 1));
            tap(7, TT(-1, dy + 1), TT(1, dy - 1));
            tap(8, TT(-2, dy + 1), TT(2, dy - 1));
            tap(9, TT(3, dy), TT(-3, dy));
            tap(10, TT(2, dy), TT(-2, dy));
            tap(11, TT(1, dy), TT(-1, dy));
#endif
            sum = (sum + 64) >> 7;
            dst[(size_t)(by + dy) * D.stride] = (int16_t)clip3(0, maxv, sum + cur);
          }
#undef TT
        } else
#pragma unroll
        for (int dy = 0; dy < 4; dy++) {
          const int y = by + dy;
          if (y >= H) break;
          int r1, r2, r3, r4, r5, r6;
          alf_rows(y, vbH, vbPos, true, r1, r2, r3, r4, r5, r6);
          const int yVb = y & (vbH - 1);
          const bool nearVB = (yVb == vbPos - 1) || (yVb == vbPos);
          const int cur = T(x, y);
          const short2_t cc2 = {(short)cur, (short)cur};
          int sum = 0;
          auto tap = [&](int k, int a, int b) {
            short2_t d = (short2_t){(short)a, (short)b} - cc2;
            d = __builtin_elementwise_min(__builtin_elementwise_max(d, cln[k]), clp[k]);
            sum = __builtin_amdgcn_sdot2(d, fcp[k], sum, true);
          };
          tap(0, T(x, r5), T(x, r6));
          tap(1, T(x + 1, r3), T(x - 1, r4));
          tap(2, T(x, r3), T(x, r4));
          tap(3, T(x - 1, r3), T(x + 1, r4));
          tap(4, T(x + 2, r1), T(x - 2, r2));
          tap(5, T(x + 1, r1), T(x - 1, r2));
          tap(6, T(x, r1), T(x, r2));
          tap(7, T(x - 1, r1), T(x + 1, r2));
          tap(8, T(x - 2, r1), T(x + 2, r2));
          tap(9, T(x + 3, y), T(x - 3, y));
          tap(10, T(x + 2, y), T(x - 2, y));
          tap(11, T(x + 1, y), T(x - 1, y));
          sum = nearVB ? (sum + 64) >> 10 : (sum + 64) >> 7;
          dst[(size_t)y * D.stride] = (int16_t)clip3(0, maxv, sum + cur);
        }
      }
    }
  }
  ALF_STAMP(2);
  ALF_STAMP(3);
  // --- chroma (filterBlk<ALF_FILTER_5> per component + filterBlkCcAlf): lane = one chroma position
  for (int ci = tid; ci < ALF_CW * ALF_CHH; ci += 256) {
    const int x = cx0 + (ci & (ALF_CW - 1)), y = cy0 + ci / ALF_CW;
    const DPlane &C1 = P.src[1];
    if (!ALF_ABL_CHROMA && x < C1.w && y < C1.h && y < (P.y1 >> 1)) {
      int cxl = 0, cxh = 0, cyl = 0, cyh = 0;
      if (VB) {   // the chroma sample's sub-rectangle, and the luma one of the CC-ALF taps
        vb_span(P, 0, 1, x, cxl, cxh);
        vb_span(P, 1, 1, y, cyl, cyh);
        vb_span(P, 0, 0, 2 * x, vxl, vxh);
        vb_span(P, 1, 0, 2 * y, vyl, vyh);
      }
#define TC(k, xx, yy) ((int)tc[k][((VB ? min(max((yy), cyl), cyh) : (yy)) - cy0 + 2) * ALF_CSW + (VB ? min(max((xx), cxl), cxh) : (xx)) - cx0 + 8])
      const int maxv = (1 << P.bd) - 1;
      const int vbHc = 1 << (P.ctu_log2 - 1), vbPosC = P.vb_chroma;
      int r1, r2, r3, r4, r5, r6;
      alf_rows(y, vbHc, vbPosC, false, r1, r2, r3, r4, r5, r6);
      (void)r5; (void)r6;
      const int lx = x * 2, ly = y * 2;
      const int pos = ly & ((1 << P.ctu_log2) - 1);
      int o1 = 1, o2 = -1, o3 = 2;
      if (pos == P.vb_luma - 2 || pos == P.vb_luma + 1) o3 = o1;
      else if (pos == P.vb_luma - 1 || pos == P.vb_luma) { o1 = 0; o2 = 0; o3 = 0; }
      const int yVb = y & (vbHc - 1);
      const bool nearVB = (yVb == vbPosC - 1) || (yVb == vbPosC);
      // CC-ALF luma taps (clamped to the picture like the staged tile: AdaptiveLoopFilter.cpp:411)
      // (the staged tile holds picture-clamped samples at every position: no clamps here)
      auto L = [&](int xx, int yy) { return T(xx, yy); };
      int sl[8] = {};
      if (ccCb || ccCr) {
        sl[0] = L(lx, ly);
        sl[1] = L(lx, ly + o2); sl[2] = L(lx - 1, ly); sl[3] = L(lx + 1, ly);
        sl[4] = L(lx - 1, ly + o1); sl[5] = L(lx, ly + o1); sl[6] = L(lx + 1, ly + o1);
        sl[7] = L(lx, ly + o3);
      }
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int comp = 1 + k;
        const DPlane &Sc = P.src[comp];
        auto A = [&](int xx, int yy) { return TC(k, xx, yy); };
        const int cur = TC(k, x, y);
        const bool on = k ? onCr : onCb;
        const int ccf = k ? ccCr : ccCb;
        int v = cur;
        if (on) {
          const int q[12] = {A(x, r3), A(x, r4), A(x + 1, r1), A(x - 1, r2), A(x, r1), A(x, r2),
                             A(x - 1, r1), A(x + 1, r2), A(x + 2, y), A(x - 2, y), A(x + 1, y), A(x - 1, y)};
          // packed like the luma taps: the pair's differences to the centre clipped as int16x2, one dot2
          const short2_t cc2 = {(short)cur, (short)cur};
          int sum = 0;
#pragma unroll
          for (int tt = 0; tt < 6; tt++) {
            const uint2 e = s_ch[k][tt];
            const short2_t l2 = __builtin_bit_cast(short2_t, e.y);
            short2_t d = (short2_t){(short)q[2 * tt], (short)q[2 * tt + 1]} - cc2;
            d = __builtin_elementwise_min(__builtin_elementwise_max(d, (short2_t){0, 0} - l2), l2);
            sum = __builtin_amdgcn_sdot2(d, __builtin_bit_cast(short2_t, e.x), sum, true);
          }
          sum = nearVB ? (sum + 64) >> 10 : (sum + 64) >> 7;
          v = clip3(0, maxv, sum + cur);
        }
        if (ccf) {
          const int c0 = sl[0];
          int sum = 0;
#pragma unroll
          for (int tt = 0; tt < 7; tt++) sum += s_cc8[k][tt] * (sl[1 + tt] - c0);
          sum = (sum + 64) >> 7;
          const int off = (1 << P.bd) >> 1;
          sum = clip3(0, maxv, sum + off) - off;
          v = clip3(0, maxv, sum + v);
        }
        const DPlane &Dc = P.dst[comp];
        Dc.p[(size_t)y * Dc.stride + x] = (int16_t)v;
      }
#undef TC
    }
  }
#undef T
#undef VCX
#undef VCY
}

// One launch, one workgroup per region; regions in XCD-contiguous runs (raster order within a run).
#ifndef ALF_WAVES_PER_EU
#define ALF_WAVES_PER_EU 1   // no cap (72 VGPRs, seven workgroups per CU); 8 (64 VGPRs) spills one VGPR, same speed
#endif
template <bool VB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ALF_WAVES_PER_EU))) void k_alf(AlfParams P, int gx, int gy) {
#ifdef ALF_NO_SWIZZLE
  const int b = (int)blockIdx.x;
#elif defined(ALF_XCD_RUN)
  const int b = xcd_run_swizzle((int)blockIdx.x, (int)gridDim.x, ALF_XCD_RUN);
#else
  const int b = xcd_swizzle(blockIdx.x, gridDim.x);
#endif
  unsigned long long stamp[6] = {0, 0, 0, 0, 0, 0};
  ALF_STAMP(0);
  alf_region<VB>(P, b % gx, b / gx, stamp);
  ALF_STAMP(4);
#ifdef VVCR_ALF_PROF
  if (threadIdx.x == 0 && blockIdx.x < (1u << 15)) {
    for (int k = 0; k < 5; k++) g_alfprof[blockIdx.x][k] = stamp[k];
    g_alfprof[blockIdx.x][5] = (unsigned long long)b;
  }
#endif
}

}  // namespace

void launch_sao(const SaoParams &p, hipStream_t s) {
  const int W = p.src[0].w;   // luma bounds; chroma blocks beyond their rows exit
  if (p.y1 <= p.y0) return;
  dim3 grid(((W + 7) / 8 + 63) / 64, (p.y1 - p.y0 + 3) / 4, 3);
  hipLaunchKernelGGL(k_sao, grid, dim3(256), 0, s, p);
}

// Clear (copy == 0) or copy the three planes of a picture in one launch (the per-picture residual
// clear and the SAO-only copy-back would otherwise be three runtime fill / copy dispatches each).
__global__ __launch_bounds__(256) void k_planes3(Planes3 P) {
  const int c = blockIdx.z;
  const DPlane &D = P.dst[c];
  const int y = (c ? P.y0 >> 1 : P.y0) + blockIdx.y, x = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (y >= D.h || x >= D.w || y >= (c ? P.y1 >> 1 : P.y1)) return;
  // 8 samples (16 B) per lane: planes are 128-B pitched, so the vector stays inside the row
  uint4 *d = (uint4 *)(D.p + (size_t)y * D.stride + x);
  *d = P.copy ? *(const uint4 *)(P.src[c].p + (size_t)y * P.src[c].stride + x) : make_uint4(0, 0, 0, 0);
}

void launch_planes3(const Planes3 &p, hipStream_t s) {
  const int W = p.dst[0].w;
  if (p.y1 <= p.y0) return;
  dim3 grid(((W + 7) / 8 + 255) / 256, p.y1 - p.y0, 3);
  hipLaunchKernelGGL(k_planes3, grid, dim3(256), 0, s, p);
}

void launch_alf(const AlfParams &p, hipStream_t s) {
  if (p.y1 <= p.y0) return;
  const int gx = (p.src[0].w + ALF_TW - 1) / ALF_TW, gy = (p.y1 - p.y0 + ALF_TH - 1) / ALF_TH;
  // pictures with virtual boundaries (loop filters not across them) take the clamping instantiation
  if (p.nvb[0] + p.nvb[1]) hipLaunchKernelGGL(k_alf<true>, dim3(gx * gy), dim3(256), 0, s, p, gx, gy);
  else hipLaunchKernelGGL(k_alf<false>, dim3(gx * gy), dim3(256), 0, s, p, gx, gy);
}
