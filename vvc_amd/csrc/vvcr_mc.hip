// vvcr_mc.hip — motion-compensated prediction of plain (translational) inter CUs for gfx950: k_mc.
//
// k_mc: one lane per cell (luma 4 columns x 8 rows, chroma 4 x 4 of one component) of a McJob, no LDS and
// no barriers, one wave per workgroup (details at the kernel's section below). The lane reads its
// reference windows straight from the planes as aligned dword runs of sample pairs; a job whose windows
// may leave the picture goes to the k_mc<edge> instantiation, which clamps rows and shifts / replicates the
// dwords of a row crossing the left / right edge (equivalent to VTM's edge-replicated 288-sample margin,
// Picture::extendPicBorder Picture.cpp:737, plus clipMv Mv.cpp:54: every filter phase sums to 64, so a
// clamped run of equal samples filters to the same value whatever the phase). DMVR / BDOF jobs are
// k_mc_bidir's (vvcr_mc_ext.hip), affine ones k_mc_affine's (vvcr_mc_affine.hip).
//
// Filtering is InterpolationFilter::filter<N,isVertical,isFirst,isLast> (InterpolationFilter.cpp:548-650)
// as the H-then-V pass of xPredInterBlk (InterPrediction.cpp:784-803) for EVERY fraction: a zero fraction
// takes the identity phase {.., 64, ..}, whose intermediate is exact (16 s - 8192 fits int16), and the
// 2-D roundings then equal the copy / H-only / V-only branches (((64 t + off2) >> sh2) == t;
// ((16 X - 2^19) >> 6) == ((X - 2^15) >> 2); (16 X + 2^9) >> 10 == (X + 32) >> 6). One code path, no
// divergence on fractions.
//
// Arithmetic is packed: samples are int16 pairs in dwords and each tap pair is one v_dot2c_i32_i16. An
// output whose first tap sits on an even sample uses the pair-aligned coefficients A = (c0,c1)(c2,c3)..,
// one starting on an odd sample the shifted set B = (0,c0)(c1,c2)..(c_{N-1},0) over the same aligned
// pairs, so every read is an aligned dword. The H outputs of consecutive rows are packed into vertical
// pairs as they arrive, so the V pass runs on aligned pairs the same way. Results combine like
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

// The weighted combinations of the two lists, reduced to one per-sample form
//   clip(((a * w0 + b * w1 + k) >> s) + o)
// with per-cell constants (a, b: the lists' 14-bit intermediates with IF_INTERNAL_OFFS removed; uni WP
// has b == a, w1 == 0): WeightPrediction::addWeightUni (WeightPrediction.cpp:280-378) and addWeightBi
// (:157-222), AreaBuf::addWeightedAvg (BCW, Buffer.cpp:350) and the GEO blend of xWeightedGeoBlk
// (InterpolationFilter.cpp:997), whose weight w0 = w(x, y), w1 = 8 - w0 varies per sample: its mask index
// (Rom.cpp:778-801, computed in place) is linear in the sample position, so a cell carries its value at
// the cell origin and the steps per column / row.
struct Comb {
  int w0, w1, k, s, o;
  int gb, gdx, gdy;   // GEO: mask index at the cell origin, per column, per row
  bool geo;
};
__device__ __forceinline__ Comb comb_setup(const WpTable &WT, const McJob &J, int comp, int bd, int cx, int cy) {
  Comb C;
  const int cs = comp ? 1 : 0;
  const bool l0 = J.flags & MC_L0, l1 = J.flags & MC_L1, bi = l0 && l1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  C.geo = false;
  C.gb = C.gdx = C.gdy = 0;
  C.o = 0;
  if (J.flags & MC_WP) {
    if (!bi) {
      const int l = l0 ? 0 : 1, r = l0 ? (J.ridx & 15) : (J.ridx >> 4);
      const int w = WT.w[l][r][comp], sh = WT.d[l][r][comp] + headRoom;
      C.w0 = w; C.w1 = 0; C.k = w * IF_INTERNAL_OFFS + (1 << (sh - 1)); C.s = sh; C.o = WT.o[l][r][comp];
    } else {
      const int r0 = J.ridx & 15, r1 = J.ridx >> 4;
      const int sh = WT.d[0][r0][comp] + 1 + headRoom;
      const int off = WT.o[0][r0][comp] + WT.o[1][r1][comp];
      C.w0 = WT.w[0][r0][comp]; C.w1 = WT.w[1][r1][comp];
      C.k = (C.w0 + C.w1) * IF_INTERNAL_OFFS + (1 << (sh - 1)) + off * (1 << (sh - 1));
      C.s = sh;
    }
    return C;
  }
  C.k = (1 << (headRoom + 2)) + (IF_INTERNAL_OFFS << 3);
  C.s = headRoom + 3;
  if (J.flags & MC_GEO) {
    const int angle = J.aux & 31, offX = (J.aux >> 8) & 255, offY = (J.aux >> 16) & 255;
    const int lx = ((J.x >> cs) + cx - (J.pu_x >> cs)) << cs, ly = ((J.y >> cs) + cy - (J.pu_y >> cs)) << cs;
    const int mir = c_geo_angle2mirror[angle];
    const int X = mir == 1 ? GEO_WEIGHT_MASK_SIZE - 1 - offX - lx : offX + lx;
    const int Y = mir == 2 ? GEO_WEIGHT_MASK_SIZE - 1 - offY - ly : offY + ly;
    const int b = c_geo_mask_angle[c_geo_angle2mask[angle]];
    const int dX = c_geo_dis[b], dY = c_geo_dis[(b + 8) & 31];
    const int rho = (dX << 8) + (dY << 8);
    C.geo = true;
    C.gb = (((X + GEO_MASK_OFFSET) << 1) + 1) * dX + (((Y + GEO_MASK_OFFSET) << 1) + 1) * dY - rho;
    C.gdx = ((mir == 1 ? -2 : 2) * dX) << cs;
    C.gdy = ((mir == 2 ? -2 : 2) * dY) << cs;
    C.w0 = C.w1 = 0;
    return C;
  }
  const int w1 = c_bcw_w1[J.bcw];   // BCW (bcw == 2: the equal weights, used only through addAvg)
  C.w0 = 8 - w1; C.w1 = w1;
  return C;
}
// one sample at column q / row o of the cell
__device__ __forceinline__ int comb_apply(const Comb &C, int q, int o, int a, int b, int maxv) {
  int w0 = C.w0, w1 = C.w1;
  if (C.geo) {
    w0 = clampi((32 + C.gb + q * C.gdx + o * C.gdy + 4) >> 3, 0, 8);
    w1 = 8 - w0;
  }
  return clampi(((a * w0 + b * w1 + C.k) >> C.s) + C.o, 0, maxv);
}

// ------------------------------------------------------------------------------------------------
// k_mc: one lane per cell, no LDS and no barriers. A luma cell is 4 columns x 8 rows of one job, a chroma
// cell 4 columns x 4 rows of one component; the lane filters every list of its job and combines them.
//
// H pass, one reference row at a time: the lane loads the dwords of sample pairs that hold the row's
// 11 (luma) / 7 (chroma) window samples, starting at the even column at or before the window origin, so
// the first tap may sit on the low or the high half of the first dword (parity par, per lane). Two
// per-lane tap sets absorb the parity instead of realigning the samples: T0 for outputs 0 and 2, T1 for
// outputs 1 and 3 (output 2 / 3 = output 0 / 1 one dword on), each N/2 + 1 packed pairs:
//   par 0: T0 = A = (c0,c1)(c2,c3).. + zero pair, T1 = B = (0,c0)(c1,c2)..(cN-1,0)
//   par 1: T0 = B, T1 = zero pair + A
// so four outputs cost 2 (N/2 + 1) v_dot2 on aligned dwords. The H intermediate is kept as sum >> sh1
// (IF_INTERNAL_OFFS not subtracted: every phase sums to 64, so the V pass subtracts 64 * IF_INTERNAL_OFFS
// once; the values fit int16), and consecutive rows of a column are packed into vertical pairs as they
// arrive: V output o = sum_m dot2(pair(o + 2m), A_m). Same roundings as filter<N,isVertical,isFirst,isLast>
// (InterpolationFilter.cpp:548-650) in the H-then-V order of xPredInterBlk (InterPrediction.cpp:784-803)
// for every fraction (the identity phase reproduces the copy / 1-D branches exactly, see the file header).
// Rows are clamped to the picture; a lane whose window leaves the picture horizontally gathers its row
// samples one by one with clamped columns (the edge-replicated margin, Picture.cpp:737).
// ------------------------------------------------------------------------------------------------
struct CellTaps {
  // luma H: set x frac x par x (T0, T1); sets: 0 8-tap, 1 6-tap of 4x4 blocks, 2 / 3 the same with the
  // alternative half-sample filter at frac 8 (it takes precedence over the 4x4 set, InterpolationFilter.cpp:778)
  uint32_t lh[4][16][2][2][5];
  uint32_t lv[4][16][4];         // luma V: A pairs
  uint32_t ch[32][2][2][3];      // chroma H: frac x par x (T0, T1)
  uint32_t cv[32][2];            // chroma V
};
constexpr int8_t k_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
constexpr int8_t k_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
constexpr int8_t k_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
constexpr int8_t k_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
template <int N>
constexpr void cell_hset(const int8_t *c, uint32_t (&t)[2][2][N / 2 + 1]) {
  uint32_t A[N / 2 + 1] = {}, B[N / 2 + 1] = {};
  for (int k = 0; k < N / 2; k++) A[k] = pk(c[2 * k], c[2 * k + 1]);
  B[0] = pk(0, c[0]);
  for (int k = 1; k < N / 2; k++) B[k] = pk(c[2 * k - 1], c[2 * k]);
  B[N / 2] = pk(c[N - 1], 0);
  for (int k = 0; k <= N / 2; k++) {
    t[0][0][k] = A[k];                  // par 0: T0 = A (+ zero pair)
    t[0][1][k] = B[k];                  //        T1 = B
    t[1][0][k] = B[k];                  // par 1: T0 = B
    t[1][1][k] = k ? A[k - 1] : 0u;     //        T1 = zero pair + A
  }
}
constexpr CellTaps make_cell_taps() {
  CellTaps t{};
  for (int set = 0; set < 4; set++)
    for (int f = 0; f < 16; f++) {
      const int8_t *c = (set >= 2 && f == 8) ? k_alt_hpel : ((set & 1) ? k_luma4x4[f] : k_luma[f]);
      cell_hset<8>(c, t.lh[set][f]);
      for (int k = 0; k < 4; k++) t.lv[set][f][k] = pk(c[2 * k], c[2 * k + 1]);
    }
  for (int f = 0; f < 32; f++) {
    cell_hset<4>(k_chroma[f], t.ch[f]);
    for (int k = 0; k < 2; k++) t.cv[f][k] = pk(k_chroma[f][2 * k], k_chroma[f][2 * k + 1]);
  }
  return t;
}
__constant__ CellTaps c_ctaps = make_cell_taps();

// Lanes per workgroup. k_mc shares nothing within a workgroup (no LDS, no barrier), and a workgroup's slot
// is freed only when its slowest wave ends: one wave per workgroup lets every wave slot refill as soon as its
// wave ends (with four, the luma waves' spread of lifetimes left CUs half empty, r04 per-wave trace).
#ifndef MC_WG
#define MC_WG 64
#endif
#ifndef MC_WAVES_PER_EU
#define MC_WAVES_PER_EU 4
#endif
#ifndef MC_XCD_RUN
#define MC_XCD_RUN 32
#endif
static_assert(MC_WG == 64, "k_mc: one wave per workgroup (wave64)");
// MC_RING: reference rows in flight per lane in a continuous ring (0: the r05 form, groups of MC_ROWS_AHEAD rows)
#ifndef MC_RING
#define MC_RING 2
#endif
// the residual row of an output is loaded this many H rows before the row that completes it: with the ring,
// at least MC_RING, so that it is older than the row loads in flight when the store waits for it (a load
// younger than them would make that wait drain the ring)
#ifndef MC_RESI_AHEAD
#define MC_RESI_AHEAD (MC_RING > 0 ? MC_RING : 0)
#endif
#ifndef MC_ROWS_AHEAD
#define MC_ROWS_AHEAD 4
#endif
// Dword-aligned loads of 2 / 4 / 6 dwords (multi-dword global loads need dword alignment only).
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));

// The ND dwords of sample pairs of one reference row from the even column dc: one 16-byte (+ 8-byte) load
// when the span lies inside the row; else the same loads at the row's first / last 2 ND samples, the
// dwords shifted into place by selects and the columns beyond the edge filled with the edge sample
// (dc is even, so a dword is either wholly inside or wholly outside the row). Rows are >= 2 ND samples
// wide (vvcr_create: width >= 16).
template <int ND>
__device__ __forceinline__ void load_nd(const int16_t *q, uint32_t (&w)[ND]) {
#ifdef MC_ABL_LOADS   // diagnostics ablation: no reference loads (results wrong)
#pragma unroll
  for (int k = 0; k < ND; k++) w[k] = (uint32_t)(uintptr_t)q * (k + 3);
  return;
#endif
  const u32x4a v = *(const u32x4a *)q;
  w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  if (ND == 6) {
    const u32x2a u = *(const u32x2a *)(q + 8);
    w[4 % ND] = u.x; w[5 % ND] = u.y;
  }
}
// Edge windows: the loads start at a column inside the row (cb), and dword k of the span is loaded dword
// k + sh (sh < 0: the span starts left of the row, > 0: right; dc is even, so a dword is either wholly
// inside or wholly outside the row), the others are the edge sample repeated. Branch-free per row.
struct EdgeMap {
  int cb, sh;
  bool left;
};
template <int ND>
__device__ __forceinline__ EdgeMap edge_map(int dc, int pw) {
  EdgeMap e;
  if (dc < 0) { e.cb = 0; e.sh = max(dc >> 1, -ND); e.left = true; }
  else if (dc + 2 * ND > pw) { e.cb = pw - 2 * ND; e.sh = min((dc - e.cb) >> 1, ND); e.left = false; }
  else { e.cb = dc; e.sh = 0; e.left = false; }
  return e;
}
template <int ND>
__device__ __forceinline__ void edge_dwords(const int16_t *row, const EdgeMap &e, uint32_t (&w)[ND]) {
  uint32_t D[ND];
  load_nd<ND>(row + e.cb, D);
  const uint32_t s = e.left ? (D[0] & 0xffffu) : (D[ND - 1] >> 16), fill = s | s << 16;
#pragma unroll
  for (int k = 0; k < ND; k++) {
    uint32_t v = fill;
#pragma unroll
    for (int t = 0; t < ND; t++) v = (k + e.sh == t) ? D[t] : v;
    w[k] = v;
  }
}

// One list of a cell: R x 4 outputs of the N-tap separable filter from the reference plane R, window
// origin (ox, oy) (first tap), fractions fx / fy, tap set ts (luma); emit(o, v) receives output row o,
// v[c] = (V sum + off2) >> sh2 before any clamp, as soon as its last H row is filtered.
template <int N, int R, bool EDGE, class Emit, class Pre>
__device__ __forceinline__ void cell_filter(const DPlane &Rp, int ox, int oy, int fx, int fy, int ts, int sh1, int off2, int sh2,
                                            Emit &&emit, Pre &&pre) {
  constexpr int ND = N / 2 + 2, NT = N / 2 + 1, NV = N / 2, ROWS = R + N - 1;
  const int par = ox & 1, dc = ox - par;
  uint32_t T0[NT], T1[NT], TV[NV];
  if (N == 8) {
    const uint32_t *h = c_ctaps.lh[ts][fx][par][0];
#pragma unroll
    for (int k = 0; k < NT; k++) { T0[k] = h[k]; T1[k] = h[NT + k]; }
#pragma unroll
    for (int k = 0; k < NV; k++) TV[k] = c_ctaps.lv[ts][fy][k];
  } else {
    const uint32_t *h = c_ctaps.ch[fx][par][0];
#pragma unroll
    for (int k = 0; k < NT; k++) { T0[k] = h[k]; T1[k] = h[NT + k]; }
#pragma unroll
    for (int k = 0; k < NV; k++) TV[k] = c_ctaps.cv[fy][k];
  }
  uint32_t Pv[4][ROWS - 1];   // vertical pairs (H row r, H row r + 1) per column
  int prev[4] = {0, 0, 0, 0};
  // one H row: 2 (N/2 + 1) dot2 for the four columns, the vertical pairs with the row before, and the V
  // outputs whose last pair this row completes (output o reads pairs o, o + 2, .., o + N - 2), so that a
  // pair lives only as long as an output still needs it
  auto hrow = [&](int r, const uint32_t (&w)[ND]) {
    int a, b, c, d;
#ifdef MC_ABL_FILTER   // diagnostics ablation: no H filter arithmetic (results wrong)
    a = w[0] ^ T0[0]; b = w[1] ^ T1[0]; c = w[2]; d = w[3];
#else
    a = dot2(w[0], T0[0], 0);
    b = dot2(w[0], T1[0], 0);
    c = dot2(w[1], T0[0], 0);
    d = dot2(w[1], T1[0], 0);
#pragma unroll
    for (int k = 1; k < NT; k++) {
      a = dot2(w[k], T0[k], a);
      b = dot2(w[k], T1[k], b);
      c = dot2(w[k + 1], T0[k], c);
      d = dot2(w[k + 1], T1[k], d);
    }
#endif
    const int hs[4] = {a >> sh1, b >> sh1, c >> sh1, d >> sh1};
    if (r > 0) {
#pragma unroll
      for (int q = 0; q < 4; q++) Pv[q][r - 1] = __builtin_amdgcn_perm((uint32_t)hs[q], (uint32_t)prev[q], 0x05040100u);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) prev[q] = hs[q];
    const int o = r - (N - 1);
    if (o >= 0) {
      int v[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        int acc;
#ifdef MC_ABL_FILTER
        acc = off2 + (Pv[q][o] ^ Pv[q][o + N - 2] ^ TV[0]);
#else
        acc = dot2(Pv[q][o], TV[0], off2);
#pragma unroll
        for (int m = 1; m < NV; m++) acc = dot2(Pv[q][o + 2 * m], TV[m], acc);
#endif
        v[q] = acc >> sh2;
      }
      emit(o, v);
    }
  };
  if constexpr (!EDGE && MC_RING > 0) {
    // k_mc: the host routed every job whose windows may leave the picture to k_mc<edge> (mc_job_edge), so
    // the window is inside: vector loads. The rows stream through a ring of MC_RING loads in flight: row
    // r + MC_RING is issued right after row r's dwords are taken, before row r is filtered, so the next
    // rows' memory round trips overlap this row's arithmetic (r05 issued four rows, filtered them, then
    // issued the next four: a wave then lived ~9 dependent round trips, 13-15 us even on an idle chip,
    // r06 per-wave trace profiles/r06_mcprof_*)
    const int16_t *row = Rp.p + (size_t)oy * Rp.stride + dc;
    constexpr int K = MC_RING < ROWS ? MC_RING : ROWS;
    uint32_t ring[K][ND];
#pragma unroll
    for (int r = 0; r < K; r++) load_nd<ND>(row + (size_t)r * Rp.stride, ring[r]);
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      pre(r);
      uint32_t w[ND];
#pragma unroll
      for (int k = 0; k < ND; k++) w[k] = ring[r % K][k];
      if (r + K < ROWS) load_nd<ND>(row + (size_t)(r + K) * Rp.stride, ring[r % K]);
      hrow(r, w);
      __builtin_amdgcn_sched_barrier(0);   // keeps the order: the load of row r + K before row r's arithmetic
    }
  } else if constexpr (!EDGE) {
    const int16_t *row = Rp.p + (size_t)oy * Rp.stride + dc;
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      pre(r);
      uint32_t w[ND];
      load_nd<ND>(row, w);
      hrow(r, w);
      row += Rp.stride;
      // at most MC_ROWS_AHEAD rows of loads in flight: more would only raise the register count (and lower the
      // occupancy that hides the load latency)
      if (r % MC_ROWS_AHEAD == MC_ROWS_AHEAD - 1) __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    // k_mc<edge>: rows clamped, edge columns replicated (Picture::extendPicBorder)
    const EdgeMap e = edge_map<ND>(dc, Rp.w);
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      pre(r);
      const int16_t *row = Rp.p + (size_t)clampi(oy + r, 0, Rp.h - 1) * Rp.stride;
      uint32_t w[ND];
      edge_dwords<ND>(row, e, w);
      hrow(r, w);
    }
  }
}

// The window of list l of job J for the cell at (x, y) of component comp (picture coordinates of that
// component): origin of the first tap, fractions, reference plane.
struct CellWin {
  DPlane R;
  int ox, oy, fx, fy;
};
__device__ __forceinline__ CellWin cell_win(const RefPlanes &ref, const McJob &J, int comp, int l, int x, int y) {
  CellWin W;
  const int cs = comp ? 1 : 0, fb = 4 + cs, half = comp ? 1 : 3;
  const int slot = l ? J.slot[1] : J.slot[0];
  // comp is a per-lane value in the chroma cells: the plane geometry by selects between static fields
  // (Cb and Cr share it), never a lane-indexed read of the kernel argument
  W.R.p = const_cast<int16_t *>(ref.p[slot * 3 + comp]);
  W.R.stride = comp ? ref.stride[1] : ref.stride[0];
  W.R.w = comp ? ref.w[1] : ref.w[0];
  W.R.h = comp ? ref.h[1] : ref.h[0];
  const int mvx = l ? J.mv[1][0] : J.mv[0][0], mvy = l ? J.mv[1][1] : J.mv[0][1], mask = (1 << fb) - 1;
  W.fx = mvx & mask;
  W.fy = mvy & mask;
  W.ox = x + (mvx >> fb) - half;
  W.oy = y + (mvy >> fb) - half;
  return W;
}

// One cell: every list of the job, combined (AreaBuf::addAvg / addWeightedAvg, WP, GEO blend, or the uni
// rounding), stored as rows of up to 4 samples. (x, y): the cell origin in the component plane; nc / nr:
// the valid columns / rows of the cell (blocks narrower or shorter than a cell). Q: the job's picture.
template <int N, int R, bool EDGE>
__device__ __forceinline__ void mc_cell(const McBatch &B, const McPic &Q, const WpTable &WT, const McJob &J, int comp, int x, int y,
                                        int nc, int nr) {
  const bool l0 = J.flags & MC_L0, l1 = J.flags & MC_L1, bi = l0 && l1;
  const int bd = B.bd, maxv = (1 << bd) - 1, headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int sh1 = IF_FILTER_PREC - headRoom;
  const bool rnd = !bi && !(J.flags & MC_KEEP14) && !(J.flags & MC_WP);
  // V pass: (sum - 64 * IF_INTERNAL_OFFS + off2) >> sh2 with the reference's off2 / sh2 (the H offset folded in)
  const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
  const int off2 = (rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0) - (IF_INTERNAL_OFFS << IF_FILTER_PREC);
  const int ts = (N == 8) ? ((J.w == 4 && J.h == 4) ? 1 : 0) | ((J.flags & MC_ALT_HPEL) ? 2 : 0) : 0;
  // destination: the prediction planes, or with MC_RECON the picture itself (the reconstruction
  // clip(pred + resi) of AreaBuf::reconstruct, Buffer.cpp:590, fused: no prediction plane round trip)
  const bool recon = (J.flags & MC_RECON) != 0, addResi = (J.flags & (MC_RESI << comp)) != 0;
  const DPlane &O0 = recon ? Q.reco[0] : Q.out[0], &O1 = recon ? Q.reco[1] : Q.out[1], &O2 = recon ? Q.reco[2] : Q.out[2];
  const int ostride = comp ? O1.stride : O0.stride;
  int16_t *dst = (comp == 0 ? O0.p : comp == 1 ? O1.p : O2.p) + (size_t)y * ostride + x;
  const int rstride = comp ? Q.resi[1].stride : Q.resi[0].stride;
  const int16_t *rsrc = (comp == 0 ? Q.resi[0].p : comp == 1 ? Q.resi[1].p : Q.resi[2].p) + (size_t)y * rstride + x;
  const int cx = x - (comp ? J.x >> 1 : J.x), cy = y - (comp ? J.y >> 1 : J.y);   // cell origin in the block
  const bool wide = nc == 4 && (x & 3) == 0;
  // one output row of 4 samples: 8-byte store, or 2-sample aligned pieces (chroma of blocks at odd
  // multiples of 4 luma columns, or 2 wide)
  // MC_RESI: the residual row of output o is loaded MC_RESI_AHEAD H rows before the row that completes o
  // (the last list's pre hook), so the store does not wait for a memory round trip of its own
  uint32_t rres[R][2];
  // (at row 0 also every output row the look-ahead already passed: MC_RESI_AHEAD may exceed N - 1)
  auto pre = [&](int r) {
    const int hi = r - (N - 1) + MC_RESI_AHEAD, lo = r == 0 ? 0 : hi;
#pragma unroll
    for (int o = lo; o <= hi; o++) {
      if (o < 0 || o >= R || !addResi || o >= nr) continue;
      const int16_t *rr = rsrc + (size_t)o * rstride;
      rres[o][1] = 0;
      if (wide) { const uint2 v = *(const uint2 *)rr; rres[o][0] = v.x; rres[o][1] = v.y; }
      else { rres[o][0] = ((const uint32_t *)rr)[0]; if (nc == 4) rres[o][1] = ((const uint32_t *)rr)[1]; }
    }
  };
  auto store = [&](int o, int (&a)[4]) {
    if (o >= nr) return;
#ifdef MC_ABL_STORE   // diagnostics ablation: no stores unless the value is impossible (results wrong)
    if (a[0] != -12345) return;
#endif
    int16_t *q = dst + (size_t)o * ostride;
    if (addResi) {
      const uint32_t r0 = rres[o][0], r1 = rres[o][1];
      a[0] = clampi(a[0] + lo16(r0), 0, maxv); a[1] = clampi(a[1] + hi16(r0), 0, maxv);
      a[2] = clampi(a[2] + lo16(r1), 0, maxv); a[3] = clampi(a[3] + hi16(r1), 0, maxv);
    }
    if (wide) *(uint2 *)q = make_uint2(pk(a[0], a[1]), pk(a[2], a[3]));
    else {
      ((uint32_t *)q)[0] = pk(a[0], a[1]);
      if (nc == 4) ((uint32_t *)q)[1] = pk(a[2], a[3]);
    }
  };
  // bi: list 0 first, its rows kept as packed 14-bit pairs; then the last list (list 1, or the only list of
  // a uni job) through ONE filter body whose emit combines: uni and bi share it (separate bodies per case
  // tripled k_mc's code, and its instruction footprint, not its VALU count, stretched the waves, r04).
  // (r05: list 0's rows in LDS instead of registers, bi cells split over two lanes, 4- and 16-row luma cells:
  // each measured slower, profiles/r05_mc_*; removed.)
  const bool avg = bi && !(J.flags & (MC_WP | MC_GEO)) && J.bcw == 2;
  uint32_t p0[R][2];
  if (bi) {
    const CellWin W0 = cell_win(B.ref, J, comp, 0, x, y);
    cell_filter<N, R, EDGE>(W0.R, W0.ox, W0.oy, W0.fx, W0.fy, ts, sh1, off2, sh2, [&](int o, const int (&v)[4]) {
      p0[o][0] = pk(v[0], v[1]);
      p0[o][1] = pk(v[2], v[3]);
    }, [](int) {});
  }
  const Comb CB = comb_setup(WT, J, comp, bd, cx, cy);
  const CellWin W = cell_win(B.ref, J, comp, (bi || !l0) ? 1 : 0, x, y);
  cell_filter<N, R, EDGE>(W.R, W.ox, W.oy, W.fx, W.fy, ts, sh1, off2, sh2, [&](int o, const int (&v)[4]) {
    int a[4];
    if (rnd) {
#pragma unroll
      for (int q = 0; q < 4; q++) a[q] = clampi(v[q], 0, maxv);
    } else if (avg) {   // AreaBuf::addAvg (Buffer.cpp:447)
      const uint32_t q0 = p0[o][0], q1 = p0[o][1];
      const int u[4] = {lo16(q0), hi16(q0), lo16(q1), hi16(q1)};
      const int shiftNum = headRoom + 1, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
#pragma unroll
      for (int q = 0; q < 4; q++) a[q] = clampi((u[q] + v[q] + offset) >> shiftNum, 0, maxv);
    } else {   // uni WP, bi WP / GEO / BCW
      const uint32_t q0 = bi ? p0[o][0] : 0u, q1 = bi ? p0[o][1] : 0u;
      const int u[4] = {bi ? lo16(q0) : v[0], bi ? hi16(q0) : v[1], bi ? lo16(q1) : v[2], bi ? hi16(q1) : v[3]};
#pragma unroll
      for (int q = 0; q < 4; q++) a[q] = comb_apply(CB, q, o, u[q], v[q], maxv);
    }
    store(o, a);
  }, pre);
}

// A job record through two 16-byte loads (per lane: the lanes of a wave hold different jobs).
__device__ __forceinline__ McJob load_job(const McJob *p) {
  const uint4 *q = (const uint4 *)p;
  const uint4 a = q[0], b = q[1];
  uint32_t raw[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  McJob J;
  __builtin_memcpy(&J, raw, sizeof(J));
  return J;
}

// Grid (frame-batched: the plain MC of B.npic pictures in one launch): the luma blocks of picture 0, of
// picture 1, ..., then the chroma blocks likewise (the longer luma waves first); within a picture, the cells
// of its classes as in its class table, MC_WG lanes per workgroup. The picture and the class of a wave are
// wave-uniform (a picture's class ranges are whole waves).
__device__ __forceinline__ void mc_body(const McBatch &B, int b
#ifdef VVCR_MC_PROF
                                        , unsigned long long &tag
#endif
) {
  const int nbL = B.lblk0[B.npic];
  const bool luma = b < nbL;
  const int bb = luma ? b : b - nbL;
  // the block's picture by a scan over static fields (uniform compares, no indexed kernel-argument read)
  int p = 0;
#pragma unroll
  for (int q = 1; q < MC_MAXPIC; q++)
    if (q < B.npic && bb >= (luma ? B.lblk0[q] : B.cblk0[q])) p = q;
  p = __builtin_amdgcn_readfirstlane(p);
  const McPic &Q = B.pic[p];   // (p uniform: a scalar-offset read of the kernel argument)
  // the class table through the constant address space: scalar loads, whatever the compiler proves
  const __attribute__((address_space(4))) McClassTable &ct = *(const __attribute__((address_space(4))) McClassTable *)(uintptr_t)Q.ct;
  const int g = (bb - (luma ? B.lblk0[p] : B.cblk0[p])) * MC_WG + (int)threadIdx.x;
  const int gw = __builtin_amdgcn_readfirstlane(g & ~63);   // the wave's first cell: selects the class
  // the class of the wave by a scan over static fields (wave-uniform selects; a class index used to read
  // the kernel argument would make it a per-lane indexed copy)
  int w = ct.w[0], h = ct.h[0], c0 = luma ? ct.lcell0[0] : ct.ccell0[0], jbase = ct.job0[0], jend = ct.job0[1], ed = ct.edge[0];
#pragma unroll
  for (int q = 1; q < MC_MAXCLS; q++)
    if (q < ct.n && gw >= (luma ? ct.lcell0[q] : ct.ccell0[q])) {
      w = ct.w[q]; h = ct.h[q]; c0 = luma ? ct.lcell0[q] : ct.ccell0[q]; jbase = ct.job0[q]; jend = ct.job0[q + 1]; ed = ct.edge[q];
    }
  const int i = g - c0;
  const int per = luma ? mc_luma_cells(w, h) : mc_chroma_cells(w, h);   // a power of two
  const int jn = i >> (__ffs(per) - 1), s = i & (per - 1);
#ifdef VVCR_MC_PROF
  tag = (unsigned long long)luma << 63 | (unsigned long long)(w & 255) << 8 | (h & 255) | (unsigned long long)p << 48;
#endif
  if (jn >= jend - jbase) return;   // padding of the class's cell range (whole waves)
  const McJob J = load_job(Q.jobs + jbase + jn);
#ifdef MC_ABL_EXIT   // diagnostics ablation: the job record only (results wrong)
  if (J.flags == 0xffff) Q.out[0].p[jn] = 1;
  return;
#endif
#ifdef VVCR_MC_PROF
  tag |= (unsigned long long)__builtin_popcountll(__ballot((J.flags & (MC_L0 | MC_L1)) == (MC_L0 | MC_L1))) << 16 |
         (unsigned long long)__builtin_popcountll(__ballot(J.flags & MC_RECON)) << 24 |
         (unsigned long long)__builtin_popcountll(__ballot(J.flags & (MC_WP | MC_GEO))) << 32 |
         (unsigned long long)__builtin_popcountll(__ballot(1)) << 40;
#endif
  const WpTable &WT = *Q.wpd;
  // the path is a class property (wave-uniform): edge classes take the clamped gathers, the others none
  if (luma) {
    const int ncx = w >> 2, cx = s & (ncx - 1), cy = s >> (__ffs(ncx) - 1);
    if (ed) mc_cell<8, 8, true>(B, Q, WT, J, 0, J.x + 4 * cx, J.y + 8 * cy, 4, min(8, h - 8 * cy));
    else mc_cell<8, 8, false>(B, Q, WT, J, 0, J.x + 4 * cx, J.y + 8 * cy, 4, min(8, h - 8 * cy));
  } else {
    const int cw = w >> 1, chh = h >> 1;
    const bool tall = mc_tall_chroma(h);   // class-uniform: 8-row chroma cells (mc_chroma_cells)
    const int ncx = (cw + 3) >> 2, ncy = tall ? chh >> 3 : (chh + 3) >> 2, nper = ncx * ncy;
    const int comp = 1 + (s >= nper), t = s - (comp - 1) * nper;
    const int cx = t & (ncx - 1), cy = t >> (__ffs(ncx) - 1);   // ncx is a power of two
    const int ox = (J.x >> 1) + 4 * cx, nc = min(4, cw - 4 * cx);
    if (ed) {
      if (tall) mc_cell<4, 8, true>(B, Q, WT, J, comp, ox, (J.y >> 1) + 8 * cy, nc, 8);
      else mc_cell<4, 4, true>(B, Q, WT, J, comp, ox, (J.y >> 1) + 4 * cy, nc, min(4, chh - 4 * cy));
    } else {
      if (tall) mc_cell<4, 8, false>(B, Q, WT, J, comp, ox, (J.y >> 1) + 8 * cy, nc, 8);
      else mc_cell<4, 4, false>(B, Q, WT, J, comp, ox, (J.y >> 1) + 4 * cy, nc, min(4, chh - 4 * cy));
    }
  }
}
__global__ __launch_bounds__(MC_WG) __attribute__((amdgpu_waves_per_eu(MC_WAVES_PER_EU))) void k_mc(McBatch B) {
#ifdef VVCR_MC_PROF
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // XCC_ID
  unsigned long long tag = 0;
#define MC_BODY(b) mc_body(B, b, tag)
#else
#define MC_BODY(b) mc_body(B, b)
#endif
  // (A persistent grid walking the blocks was slower, 47.3 vs 41.4 us, and doubled the kernel's code:
  // removed, r04.)
  // Block order: XCD runs of MC_XCD_RUN (32) consecutive blocks, the XCDs taking turns every run. Whole-grid
  // XCD-contiguous runs (r03, xcd_swizzle) cluster heavy regions on a few XCDs (4K B pictures, fused: QP27
  // 34.6 us, 67 MB read); dispatch order spreads the work but fetches every shared reference window into
  // several L2s (35.2 us, 151 MB); runs of 32: 30.0 us, 78 MB (runs of 4 / 8 / 16 / 64 / 128: 32.5 / 31.0
  // / 30.3 / 30.7 / 30.8 us; r04)
#if MC_XCD_RUN > 0
  MC_BODY(xcd_run_swizzle((int)blockIdx.x, (int)gridDim.x, MC_XCD_RUN));
#else
  MC_BODY((int)blockIdx.x);
#endif
#undef MC_BODY
#ifdef VVCR_MC_PROF
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const int wv = blockIdx.x * (MC_WG / 64) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && wv < (1 << 16)) {
    g_mcprof[wv][0] = t0; g_mcprof[wv][1] = t1; g_mcprof[wv][2] = (unsigned long long)hw | (unsigned long long)xcc << 32; g_mcprof[wv][3] = tag;
  }
#endif
}

}  // namespace

void launch_mc_batch(McBatch &b, const McClassTable *const *hct, hipStream_t s) {
  int lb = 0, cb = 0;
  for (int p = 0; p < b.npic; p++) {
    const McClassTable &ct = *hct[p];
    b.lblk0[p] = lb;
    b.cblk0[p] = cb;
    if (ct.n > 0) {
      lb += (ct.lcell0[ct.n] + MC_WG - 1) / MC_WG;
      cb += (ct.ccell0[ct.n] + MC_WG - 1) / MC_WG;
    }
  }
  for (int p = b.npic; p <= MC_MAXPIC; p++) { b.lblk0[p] = lb; b.cblk0[p] = cb; }
  if (lb + cb > 0) hipLaunchKernelGGL(k_mc, dim3(lb + cb), dim3(MC_WG), 0, s, b);
}
