// vvcr_intra.hip — intra prediction and reconstruction for gfx950, one 64-lane workgroup per step.
//
// Per step: reference samples from the reconstructed picture with the reference's availability and
// substitution rules (IntraPrediction::xFillReferenceSamples IntraPrediction.cpp:913-1149; ISP:
// initIntraPatternChTypeISP :798), [1 2 1] smoothing (:1152), the mode parameters of
// initPredIntraParams (:351-443), then planar / DC (:289-350), angular with 4-tap cubic / Gaussian or
// 2-tap chroma interpolation and PDPC (:458-642, predIntraAng :213-261), BDPCM (:644), MIP
// (MatrixIntraPrediction.cpp:62-374) or CCLM (xGetLumaRecPixels :1316, xGetLMParameters :1654), the
// CIIP blend (geneWeightedPred :681), and reconstruction clip(pred + resi) into the picture.
#include "vvcr_intra.h"
#include "vvcr_gen_tables.h"
#include "vvcr_tables.h"

#ifdef VVCR_INTRA_PROF
// Diagnostics build only (tools/intra_prof.py): per-step phase timestamps (s_memtime) of k_intra.
__device__ unsigned long long g_iprof[1 << 17][8];
__device__ unsigned int g_iprof_n;
extern "C" int vvcr_intra_prof_read(unsigned long long *dst, int max) {
  unsigned int n = 0;
  (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_iprof_n), sizeof(n));
  n = n < (unsigned)max ? n : (unsigned)max;
  (void)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_iprof), (size_t)n * 8 * 8);
  unsigned int z = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_iprof_n), &z, sizeof(z));
  return (int)n;
}
// phase stamps of run_step (shader cycles), kept in registers: ps[i] after waiting for the phase's memory
#define IPROF(i) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); ps[i] = __builtin_readcyclecounter(); } while (0)
#else
#define IPROF(i) do { } while (0)
#endif
#if defined(VVCR_INTRA_PROF) && defined(VVCR_IPROF_PRE)   // diagnostics: stamps between the wait and the fill
#define PPROF(i) IPROF(i)
#define IPROF_POST(i) do { } while (0)
#else
#define PPROF(i) do { } while (0)
#define IPROF_POST(i) IPROF(i)
#endif

#ifdef VVCR_DIAG_DUMP
__device__ int32_t g_dbg[1024];
extern "C" int vvcr_diag_dump(int32_t *dst) { return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dbg), sizeof(g_dbg)); }
#endif
namespace {

__constant__ int8_t i_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;

constexpr int PLANAR = 0, DC = 1, HOR = 18, DIA = 34, VER = 50, VDIA = 66, LM = 67, MDLM_L = 68, MDLM_T = 69;
constexpr int RB = 160;                      // reference buffer length (2*64 + mrl + 1, rounded)
constexpr int EXT = 64;                      // negative-index room of the angular main reference
// Residual rectangles of up to RESL samples (32x32, and every ISP CU up to 32x32) are staged in LDS;
// larger ones (64-sample sides, rare in intra pictures) are read from HBM (L2-warm) by the
// reconstruction. This keeps a 4-wave workgroup within half of the CU's 160 KB of LDS, so two CTU
// workgroups — e.g. of two concurrently decoded intra pictures — share a CU.
constexpr int RESL = 1024;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int ilog2(int v) { return v <= 0 ? -1 : 31 - __clz(v); }

struct Ctx {
  const IntraParams *P;
  int ch;        // 0 luma map, 1 chroma map
  int seq;
};

// Plane pointers reach the kernels through LDS / structs as generic pointers; loads and stores through
// them would be FLAT instructions, which count on lgkmcnt too, so every LDS wait would also wait for
// them. Accesses go through these global-address-space casts instead.
template <class T> __device__ __forceinline__ const __attribute__((address_space(1))) T *gp(const T *p) {
  return (const __attribute__((address_space(1))) T *)p;
}
template <class T> __device__ __forceinline__ __attribute__((address_space(1))) T *gpw(T *p) {
  return (__attribute__((address_space(1))) T *)p;
}
__device__ __forceinline__ int pel(const DPlane &D, int x, int y) { return *gp(&D.p[(size_t)y * D.stride + x]); }

// Reconstructed samples are handed between steps of one launch (k_intra is persistent): every store of
// them is a 4-byte sc1 store and every load of them a 4-byte sc1 load (bypasses the CU's L1), the
// producing wave drains its stores (s_waitcnt vmcnt(0)) before its one-lane sc1 flag store, and the
// consumer loads only after its sc1 polls of those flags matched (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row of the sc1 hand-off table; one workgroup per CU).
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ uint32_t ld_sc1(const int16_t *p) {   // p 4-byte aligned
#ifdef VVCR_PROF_PLAIN_LOADS   // diagnostics only: latency of plain loads (not a valid hand-off)
  return *(const uint32_t *)p;
#else
  return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
__device__ __forceinline__ void st_sc1(int16_t *p, uint32_t v) {   // p 4-byte aligned
  __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one reconstructed sample (x any) / the sample pair (x even, x + 1)
__device__ __forceinline__ int pel_rc(const DPlane &D, int x, int y) {
  const uint32_t v = ld_sc1(D.p + (size_t)y * D.stride + (x & ~1));
  return (int)(int16_t)((x & 1) ? (v >> 16) : (v & 0xffff));
}
__device__ __forceinline__ uint32_t pair_rc(const DPlane &D, int x, int y) { return ld_sc1(D.p + (size_t)y * D.stride + x); }

__device__ __forceinline__ int wave_sum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ------------------------------------------------------------------------------------------------
// CTU-resident reconstruction. A workgroup of NW waves owns one CTU at a time: the CTU's samples (luma
// and both chroma planes) live in an LDS tile, each wave runs one step at a time, and steps of the
// same CTU hand over through LDS (a done byte per step). Only samples outside the CTU — the left /
// above / above-right neighbours' borders — are read from HBM, through the sc1 hand-off below, and
// only steps that such a read depends on (IJ_PUBLISH) drain their HBM stores and raise a global flag.
// ------------------------------------------------------------------------------------------------
constexpr int NW = kIntraWaves;              // waves per workgroup
constexpr int TPL = 130, TPC = 66;           // LDS tile pitches (odd dword count: column walks hit distinct banks)
constexpr int TILE_Y = 0, TILE_CB = 128 * TPL, TILE_CR = TILE_CB + 64 * TPC, TILE_N = TILE_CR + 64 * TPC;

struct WaveScratch {
  int16_t refU[2][RB];          // unfiltered top / left (index 0 = corner)
  int16_t refF[2][RB];          // filtered
  int16_t mainA[EXT + RB + 64]; // angular main reference (with negative indices)
  int16_t sideA[EXT + RB + 64];
  int16_t aux[64 * 64 / 4];     // MIP reduced pred / CCLM down-sampled luma
  int16_t tmpl[2][132];         // CCLM down-sampled luma: top row / left column
  int32_t lmp[4];
  int32_t red[8];               // MIP reduced boundary
  int16_t resL[RESL];           // residual of the step (rectangles of <= RESL samples), prefetched at entry
  int16_t ispPrev[64];          // ISP: last row / column of the previous region
};

__shared__ int16_t s_tile[TILE_N];
__shared__ WaveScratch s_ws[NW];
__shared__ uint8_t s_ldone[kIntraMaxStepsPerCtu];
__shared__ __attribute__((aligned(4))) int8_t s_cubic[32][4];   // the 4-tap DCT-IF (chroma) filter the luma angular prediction uses

// Wave-level ordering of LDS traffic between the lanes of one wave (the steps of one workgroup run on
// different waves, so the step body never uses a workgroup barrier). A wavefront-scope fence is not
// enough: it is dropped before instruction scheduling, which may then hoist a lane's LDS read above
// another lane's write of the same word when the two do not alias within one thread. An asm statement
// with a memory clobber is a scheduling barrier for memory operations; the LDS itself executes one
// wave's DS instructions in order, so no wait is needed.
__device__ __forceinline__ void wsync() {
#ifdef VVCR_DIAG_WSYNC_BARRIER
  __syncthreads();
#else
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#endif
}

// Area of the current CTU in luma samples (chroma: halved); scalars only, so that nothing of it is
// indexed dynamically (a private array would be promoted to per-lane LDS or scratch).
struct TileGeo {
  int x0, y0, w, h;
  __device__ __forceinline__ int cx0(int comp) const { return comp ? x0 >> 1 : x0; }
  __device__ __forceinline__ int cy0(int comp) const { return comp ? y0 >> 1 : y0; }
  __device__ __forceinline__ int cw(int comp) const { return comp ? w >> 1 : w; }
  __device__ __forceinline__ int ch(int comp) const { return comp ? h >> 1 : h; }
};
__device__ __forceinline__ int tile_base(int comp) { return comp == 0 ? TILE_Y : (comp == 1 ? TILE_CB : TILE_CR); }
__device__ __forceinline__ int tile_pitch(int comp) { return comp ? TPC : TPL; }

// Reconstructed samples of one component: inside the current CTU from the LDS tile, elsewhere from HBM.
struct Src {
  const int16_t *g;
  int gs, base, ts, x0, y0, w, h;
  __device__ __forceinline__ bool inside(int x, int y) const {
    return (unsigned)(x - x0) < (unsigned)w && (unsigned)(y - y0) < (unsigned)h;
  }
  __device__ __forceinline__ uint32_t pair(int x, int y) const {   // x even
    if (inside(x, y)) return *(const uint32_t *)&s_tile[base + (y - y0) * ts + x - x0];
    return ld_sc1(g + (size_t)y * gs + x);
  }  __device__ __forceinline__ int pel(int x, int y) const {
    const uint32_t v = pair(x & ~1, y);
    return (int)(int16_t)((x & 1) ? (v >> 16) : (v & 0xffff));
  }
};
__device__ __forceinline__ Src src_of(const IntraParams &P, int comp, const TileGeo &G) {
  Src s;
  s.g = P.reco[comp].p; s.gs = P.reco[comp].stride;
  s.base = tile_base(comp); s.ts = tile_pitch(comp);
  s.x0 = G.cx0(comp); s.y0 = G.cy0(comp); s.w = G.cw(comp); s.h = G.ch(comp);
  return s;
}

// Batched sample reads: every HBM load of the batch is issued before the first wait. (Reading through
// Src::pel one sample at a time makes each LDS read wait for the previous sample's HBM load, because
// both results would share a destination register.) Samples with need[k] false read nothing (0).
template <int N>
__device__ __forceinline__ void gather(const Src &s, const int (&x)[N], const int (&y)[N], const bool (&need)[N], int (&out)[N]) {
  bool in[N];
  uint32_t gv[N], lv[N];
#pragma unroll
  for (int k = 0; k < N; k++) in[k] = s.inside(x[k], y[k]);
#pragma unroll
  for (int k = 0; k < N; k++) {
#ifdef VVCR_DIAG_NO_GLOBAL_REFS
    gv[k] = 0u;
#else
    gv[k] = (need[k] && !in[k]) ? ld_sc1(s.g + (size_t)y[k] * s.gs + (x[k] & ~1)) : 0u;
#endif
  }
#pragma unroll
  for (int k = 0; k < N; k++)
    lv[k] = (need[k] && in[k]) ? *(const uint32_t *)&s_tile[s.base + (y[k] - s.y0) * s.ts + ((x[k] & ~1) - s.x0)] : 0u;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint32_t v = in[k] ? lv[k] : gv[k];
    out[k] = (int)(int16_t)((x[k] & 1) ? (v >> 16) : (v & 0xffff));
  }
}

// xFillReferenceSamples for area (fx, fy, fw, fh) of component plane D; top[0..predSize+mrl],
// left[0..predHSize+mrl]; index 0 = corner line.
//
// The reference walks the reference units sequentially (IntraPrediction.cpp:913-1149): units are
// numbered in scan order 0 = bottom-most below-left ... totalLeft = corner ... top-right; a missing unit
// gets the last sample (in scan order) of the nearest earlier available unit, the units before the first
// available one get its first sample, and with no unit available every sample is 1 << (bd - 1). The
// availability mask (lo: units 0..63, hi: unit 64) comes resolved from the host, so every lane handles
// its own samples: available ones are copied, then missing ones read their source from the lines.
__device__ __forceinline__ void fill_refs(const Src &src, const DPlane &D, int ch, int fx, int fy, int predSize, int predHSize,
                                          int mrl, int bd, uint64_t lo, bool hi, int16_t *top, int16_t *left, int lane,
                                          unsigned long long *ps, int vnb = 0, int nul = 0, int nut = 0) {
  (void)ps;
#ifdef VVCR_ABL_FILL
  return;
#endif
#if defined(VVCR_INTRA_PROF) && defined(VVCR_IPROF_FILL)   // diagnostics: stamps inside the fill (ps[5], ps[6])
#define FPROF(i) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); ps[i] = __builtin_readcyclecounter(); } while (0)
#else
#define FPROF(i) do { } while (0)
#endif
  FPROF(5);
  const int lu = ch ? 1 : 2;   // log2 of the unit size
  const int totalLeft = (predHSize + (1 << lu) - 1) >> lu;
  const int ox = fx - 1 - mrl, oy = fy - 1 - mrl;   // corner sample of the reference line
  const int nT = predSize + mrl, nL = predHSize + mrl;   // last index of each line
  if (lo == 0 && !hi) {
    const int16_t dc = (int16_t)(1 << (bd - 1));
    for (int j = lane; j <= nT; j += 64) top[j] = dc;
    for (int i = lane; i <= nL; i += 64) left[i] = dc;
    wsync();
    return;
  }
  if (vnb & CS_PREFIX) {
    // Availability is the corner plus a run of units from the corner along each line (the usual case):
    // copy the available samples, then every missing run takes one sample (the scan rule below reduces to
    // three sources: the left tail, the corner unit, the top tail).
    const bool cAv = (vnb & CS_CORNER) != 0;
    const int aT = mrl + (nut << lu), aL = mrl + (nul << lu);   // last available index of each line
    auto avT = [&](int j) { return j <= mrl ? cAv : j <= aT; };
    auto avL = [&](int i) { return i <= mrl ? cAv : i <= aL; };
    if (vnb & CS_INTILE) {   // all available samples in the LDS tile: plain LDS reads
      const int b = src.base + (oy - src.y0) * src.ts + (ox - src.x0);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const int j = lane + 64 * r;
        if (j <= nT && avT(j)) top[j] = s_tile[b + j];
        if (j <= nL && avL(j)) left[j] = s_tile[b + j * src.ts];
      }
      FPROF(6);
    } else {
      int gx[6], gy[6], gvv[6];
      bool need[6];
      const int cy = max(oy, 0), cx = max(ox, 0);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const int j = lane + 64 * r;
        gx[r] = min(max(ox + j, 0), D.w - 1); gy[r] = cy; need[r] = j <= nT && avT(j);
        gx[3 + r] = cx; gy[3 + r] = min(max(oy + j, 0), D.h - 1); need[3 + r] = j <= nL && avL(j);
      }
      gather(src, gx, gy, need, gvv);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const int j = lane + 64 * r;
        if (need[r]) top[j] = (int16_t)gvv[r];
        if (need[3 + r]) left[j] = (int16_t)gvv[3 + r];
      }
    }
    wsync();
    if (!cAv || aT < nT || aL < nL) {
      // sources (IntraPrediction.cpp:913-1149 scan: bottom-left -> corner -> top-right): a missing unit
      // takes the last available sample before it in scan order, else the first available one
      const int16_t firstAv = nul ? left[aL] : (cAv ? left[mrl] : top[mrl + 1]);
      const int16_t sCorner = nul ? left[mrl + 1] : top[mrl + 1];
      const int16_t sTop = nut ? top[aT] : (cAv ? top[mrl] : left[mrl + 1]);
      wsync();
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const int j = lane + 64 * r;
        if (j <= nT && !avT(j)) top[j] = j <= mrl ? sCorner : sTop;
        if (j <= nL && !avL(j)) left[j] = j <= mrl ? sCorner : firstAv;
      }
      wsync();
    }
    return;
  }
  // unit of top sample j / left sample i
  auto unitT = [&](int j) { return j <= mrl ? totalLeft : totalLeft + 1 + ((j - 1 - mrl) >> lu); };
  auto unitL = [&](int i) { return i <= mrl ? totalLeft : totalLeft - 1 - ((i - 1 - mrl) >> lu); };
  auto unitAv = [&](int u) { return u < 64 ? ((lo >> u) & 1) != 0 : hi; };
  int16_t tv[3], lv[3];
  {
    // only available samples are loaded: a sample outside the CTU costs an HBM round trip (sc1), and
    // the unavailable ones (above-right / below-left beyond the decoded area) are mostly outside it
    const int cy = max(oy, 0), cx = max(ox, 0);
    int gx[6], gy[6], gvv[6];
    bool need[6];
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const int j = lane + 64 * r;
      gx[r] = min(max(ox + j, 0), D.w - 1); gy[r] = cy; need[r] = j <= nT && unitAv(unitT(j));
      gx[3 + r] = cx; gy[3 + r] = min(max(oy + j, 0), D.h - 1); need[3 + r] = j <= nL && unitAv(unitL(j));
    }
    gather(src, gx, gy, need, gvv);
#pragma unroll
    for (int r = 0; r < 3; r++) { tv[r] = (int16_t)gvv[r]; lv[r] = (int16_t)gvv[3 + r]; }
  }
  bool missing = false;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    if (j <= nT) { if (unitAv(unitT(j))) top[j] = tv[r]; else missing = true; }
    if (j <= nL) { if (unitAv(unitL(j))) left[j] = lv[r]; else missing = true; }
  }
  if (__ballot(missing) == 0) { wsync(); return; }
  wsync();
  // missing units: the scan-order last sample of the nearest earlier available unit, else the first
  // sample of the first available unit (both are copied samples)
  const int firstAv = lo ? __builtin_ctzll(lo) : 64;
  auto source = [&](int u) -> int16_t {
    const uint64_t below = u < 64 ? (lo & ((1ull << u) - 1)) : lo;
    if (below) {
      const int q = 63 - __builtin_clzll(below);   // scan-last sample of unit q
      if (q < totalLeft) return left[((totalLeft - q - 1) << lu) + mrl + 1];
      if (q == totalLeft) return top[mrl];
      return top[((q - totalLeft) << lu) + mrl];
    }
    const int q = firstAv;                          // scan-first sample of unit q
    if (q < totalLeft) return left[((totalLeft - q) << lu) + mrl];
    if (q == totalLeft) return left[mrl];
    return top[((q - totalLeft - 1) << lu) + 1 + mrl];
  };
  int16_t sv[6];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    sv[r] = (j <= nT && !unitAv(unitT(j))) ? source(unitT(j)) : 0;
    sv[3 + r] = (j <= nL && !unitAv(unitL(j))) ? source(unitL(j)) : 0;
  }
  wsync();
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    if (j <= nT && !unitAv(unitT(j))) top[j] = sv[r];
    if (j <= nL && !unitAv(unitL(j))) left[j] = sv[3 + r];
  }
  wsync();
}


// isAbove/Left/AboveRight/BelowLeftAvailable counts for CCLM (resolved on the host: nb_bits)
struct NbAvail {
  bool above, left;
  int ar, bl;          // available above-right / below-left units
};
__device__ __forceinline__ NbAvail nb_decode(uint32_t b) {
  NbAvail r;
  r.above = (b & 1) != 0;
  r.left = (b & 2) != 0;
  r.ar = (b >> 2) & 31;
  r.bl = (b >> 7) & 31;
  return r;
}

// Polling interval (s_sleep units of 64 cycles). A polling wave competes with the working waves of its CU
// for instruction issue, so the waits sleep between polls.
#ifndef VVCR_LSLEEP
#define VVCR_LSLEEP 1
#endif
#ifndef VVCR_INTRA_PRIO
#define VVCR_INTRA_PRIO 3
#endif
#ifndef VVCR_GSLEEP
#define VVCR_GSLEEP 2
#endif
// bounded spin on a flag; sets *err and gives up after ~seconds (never expected)
__device__ __forceinline__ void wait_global(const int32_t *f, int32_t *err) {
  for (int it = 1; __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0; it++) {
    __builtin_amdgcn_s_sleep(VVCR_GSLEEP);
    if ((it & 1023) == 0 && __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) break;
    if (it > (1 << 22)) { atomicOr(err, 1); break; }
  }
}
__device__ __forceinline__ void wait_local(int v, int32_t *err) {
  for (int it = 1; __builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_ldone[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0; it++) {
    __builtin_amdgcn_s_sleep(VVCR_LSLEEP);
    if ((it & 1023) == 0 && __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) break;
    if (it > (1 << 24)) { atomicOr(err, 1); break; }
  }
}

// One reconstruction step, run by one wave.
// LMCS chroma residual scale of a block (Reshape::calculateChromaAdjVpduNei, Reshape.cpp:107-198): the
// average of the reconstructed (mapped) luma left of / above the CU at the block's VPDU corner, clipped,
// located among the mapped-domain pivots (getPWLIdxInv :204) and looked up in m_chromaAdjHelpLUT.
__device__ __forceinline__ int chroma_scale(const IntraParams &P, const TileGeo &G, int vx, int vy, int vnb, int lane) {
  const Src SY = src_of(P, 0, G);
  const int W = P.reco[0].w, H = P.reco[0].h;
  const int nn = min(64, P.ctu), lnn = nn == 64 ? 6 : 5;
  int xs[2], ys[2], v[2];
  bool need[2];
  xs[0] = vx - 1; ys[0] = vy + min(lane, H - vy - 1); need[0] = (vnb & CS_LEFT) && lane < nn;
  xs[1] = vx + min(lane, W - vx - 1); ys[1] = vy - 1; need[1] = (vnb & CS_ABOVE) && lane < nn;
  gather(SY, xs, ys, need, v);
  const int sum = wave_sum((need[0] ? v[0] : 0) + (need[1] ? v[1] : 0));
  const int maxv = (1 << P.bd) - 1;
  const int cnt = ((vnb & CS_LEFT) ? 1 : 0) + ((vnb & CS_ABOVE) ? 1 : 0);
  int luma;
  if (cnt == 1) luma = clampi((sum + (1 << (lnn - 1))) >> lnn, 0, maxv);
  else if (cnt == 2) luma = clampi((sum + (1 << lnn)) >> (lnn + 1), 0, maxv);
  else luma = 1 << (P.bd - 1);
  int idx = P.lmcs_min_bin;
  for (; idx <= P.lmcs_max_bin; idx++)
    if (luma < P.lmcs_pivot[idx + 1]) break;
  return P.lmcs_cadj[min(idx, 15)];
}
// AreaBuf::scaleSignal inverse (Buffer.cpp:424-441), CSCALE_FP_PREC = 11
__device__ __forceinline__ int scale_resi(int r, int scale, int bd) {
  const int maxAbs = (1 << bd) - 1;
  r = clampi(r, -maxAbs - 1, maxAbs);
  const int a = r < 0 ? -r : r;
  const int v = (a * scale + (1 << 10)) >> 11;
  return clampi(r < 0 ? -v : v, -32768, 32767);
}

// Step kinds: each gets its own instantiation of run_step, so that a step executes only its own
// path (one generic body made the compiler evaluate and spill the set-up of every path per step).
enum { K_REG = 0, K_ISP = 1, K_MIP = 2, K_LM = 3, K_CIIP = 4, K_BDPCM = 5, K_INTERC = 6 };
__device__ __forceinline__ int step_kind(const IntraJob &J) {
  if (J.xkind == XK_INTER_CHROMA) return K_INTERC;
  if (J.flags & IJ_BDPCM) return K_BDPCM;
  if (J.flags & IJ_CIIP) return K_CIIP;
  if (J.flags & (IJ_ISP_HOR | IJ_ISP_VER)) return K_ISP;
  if (J.flags & IJ_MIP) return K_MIP;
  if (J.comp > 0 && J.mode >= LM) return K_LM;
  return K_REG;
}

// kreg: the region of an ISP step (0 for every other kind). The regions of an ISP CU are iterations of the
// kernel's step loop, not a loop in here: a loop over them made the compiler hoist the set-up of every
// prediction path out of it and spill it (a fixed ~5,400 cycles per ISP step before the first fill).
template <int KIND>
__device__ __forceinline__ void run_step(const IntraParams &P, const IntraJob &J, const TileGeo &G, WaveScratch &S,
                                         const int32_t *dep_start, const int32_t *deps, int gj, int32_t *done,
                                         int32_t *err, int lane, unsigned long long &t_ready, unsigned long long *ps,
                                         const int kreg) {
  if (kreg == 0) IPROF(0);
  const int comp = J.comp, ch = comp ? 1 : 0;
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const DPlane &D = P.reco[comp];
  const Src SD = src_of(P, comp, G);
  const int w = J.w, h = J.h;
  constexpr bool isp = KIND == K_ISP;
  const bool ispVer = isp && (J.flags & IJ_ISP_VER) != 0;
  constexpr bool mip = KIND == K_MIP;
  constexpr bool bdpcm = KIND == K_BDPCM;
  constexpr bool ciip = KIND == K_CIIP;
  constexpr bool lmMode = KIND == K_LM;
  constexpr bool interc = KIND == K_INTERC;
  const int mrl = comp ? 0 : J.mrl;
  const int n = w * h;
  const int lw_ = ilog2(w);   // block sizes are powers of two: shifts instead of divisions
  const int nreg = isp ? J.isp_k : 1;
  const uint64_t avlo = (uint64_t)J.av[0] | (uint64_t)J.av[1] << 32;
  const bool avhi = (J.av[2] & 1) != 0;
  // residual rectangle: the block, or the whole CU for ISP
  const int rx = isp ? J.cx : J.x, ry = isp ? J.cy : J.y, rw = isp ? J.cw : w, rh = isp ? J.ch : h;
  // The residual does not depend on earlier steps: up to RESL samples are loaded into registers before
  // the dependency wait, and stored to LDS after the reference fill; larger rectangles are read from
  // HBM by the reconstruction.
  const DPlane &R = P.resi[comp];
  const int rn = rw * rh;
  const int lrw = ilog2(rw);
  const bool rvec = ((rw | rx) & 3) == 0;   // plane strides are multiples of 64 samples
  const bool rlds = rn <= RESL;
  // The reconstruction takes the residual straight from the prefetch registers when their layout is the
  // block's: one sample per lane (k = lane + 64 b -> rs[b]) for blocks of <= 512 samples, which keeps all
  // 64 lanes busy on small blocks (the chain is latency bound), four consecutive samples per lane
  // (k = 4 (lane + 64 b) -> rv[b]) for larger vector-aligned ones.
  const bool rsreg = !isp && rn <= 512;
  const bool rreg = !isp && !rsreg && rvec && n <= 4 * 64 * 4;
  const bool rvload = rvec && !rsreg;
  uint64_t rv[4] = {0, 0, 0, 0};
  int16_t rs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (kreg > 0) {
    // a later ISP region: its residual is in LDS (stored by region 0) or read from HBM, its
    // dependencies were met before region 0
  } else if (rvload) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int k = min((lane + 64 * b) * 4, rn - 4);
      const int yy = k >> lrw, xx = k & (rw - 1);
      rv[b] = *gp((const uint64_t *)&R.p[(size_t)(ry + yy) * R.stride + rx + xx]);
    }
  } else {
#pragma unroll
    for (int b = 0; b < 8; b++) {
      rs[b] = 0;
      if (64 * b < rn) {   // uniform: small blocks issue one load per lane
        const int k = min(lane + 64 * b, rn - 1);
        const int yy = k >> lrw, xx = k & (rw - 1);
        rs[b] = *gp(&R.p[(size_t)(ry + yy) * R.stride + rx + xx]);
      }
    }
  }
  // MIP: this lane's row of the mode's matrix (output o = lane; <= 64 outputs), loaded before the wait as
  // well (lane-dependent indices into the constant tables are per-lane memory loads)
  int mw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (mip) {
    const int sizeId = (w == 4 && h == 4) ? 0 : ((w == 4 || h == 4 || (w == 8 && h == 8)) ? 1 : 2);
    const int rp = sizeId < 2 ? 4 : 8, o = min(lane, rp * rp - 1), md = J.mode;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (sizeId == 0) mw[i] = i < 4 ? vvcr_tab::mip4x4[md][o][i] : 0;
      else if (sizeId == 1) mw[i] = vvcr_tab::mip8x8[md][o][i];
      else mw[i] = i == 0 ? 0 : vvcr_tab::mip16x16[md][o][i - 1];
    }
  }
  // Wait for the steps this one reads from, newest dependency first (the likeliest to be still
  // running); same-CTU steps through LDS, steps of other CTUs through their global flag. Every lane
  // runs the (uniform) loop and polls the same word — one request per poll — so that no lane-divergent
  // region precedes the step body: the step body's wave syncs do not force reconvergence, and code
  // sunk into a lane-0-only region would run after the other lanes' reads of its results.
  if (kreg == 0) {
    const int k0 = __builtin_amdgcn_readfirstlane(dep_start[gj]), k1 = __builtin_amdgcn_readfirstlane(dep_start[gj + 1]);
    for (int k = k1 - 1; k >= k0; k--) {
      const int v = __builtin_amdgcn_readfirstlane(deps[k]);
      if (v >= 0) wait_local(v, err);
      else wait_global(done + ~v, err);
    }
  }
  wsync();
#ifdef VVCR_INTRA_PROF
  if (kreg == 0) t_ready = __builtin_amdgcn_s_memrealtime();
#else
  (void)t_ready; (void)ps;
#endif
  if (kreg == 0) IPROF(1);
#ifdef VVCR_ABL_ALL
  return;
#endif
  // LMCS chroma residual scale (uniform), after the wait: it reads reconstructed luma of other steps
  const int cscale = (comp > 0 && (J.vnb & CS_SCALE)) ? chroma_scale(P, G, J.vx, J.vy, J.vnb, lane) : 0;
  if (kreg == 0) PPROF(2);
  auto store_resid = [&]() {
    if (!rlds || rreg || rsreg) return;
    if (rvload) {
#pragma unroll
      for (int b = 0; b < 4; b++)
        if ((lane + 64 * b) * 4 < rn) *(uint64_t *)&S.resL[(lane + 64 * b) * 4] = rv[b];
    } else {
#pragma unroll
      for (int b = 0; b < 8; b++)
        if (lane + 64 * b < rn) S.resL[lane + 64 * b] = rs[b];
    }
    for (int k = rvload ? RESL : (lane + 512); k < rn; k += 64) {   // non-vector rectangles above 512 samples
      const int yy = k >> lrw, xx = k & (rw - 1);
      const int16_t *src = &R.p[(size_t)(ry + yy) * R.stride + rx + xx];
      if (rvload) *(uint64_t *)&S.resL[k] = *gp((const uint64_t *)src);
      else S.resL[k] = *gp(src);
    }
  };

  // ---- reference lengths (setReferenceArrayLengths / ISP variants)
  int topLen = 2 * w, leftLen = 2 * h;
  if (isp) { topLen = J.cw + w; leftLen = J.ch + h; }

  // ---- prediction parameters (initPredIntraParams), resolved on the host (IntraJob::pbits ...)
  const int dirMode = ciip ? PLANAR : (int)J.mode;
  const int predMode = J.pred_mode;
  const bool isModeVer = predMode >= DIA;
  const bool applyPDPC = (J.pbits & PB_PDPC) != 0, refFilter = (J.pbits & PB_REFFILT) != 0, interp = (J.pbits & PB_INTERP) != 0;
  const int angle = J.ang, invAngle = J.inv_ang, absAng = angle < 0 ? -angle : angle, angScale = J.pbits >> 4;
  // Direct reference lines: when every reference sample of the step is in the LDS tile and available as
  // the corner plus a run from it along each line (CS_PREFIX: the substitution then only repeats a line's
  // last available sample), the prediction reads the lines in place in the tile (top: a row, left: a
  // column, index clamped at the last available sample) - no copy into refU, no wave sync. Planar's
  // [1 2 1] smoothing is then applied on the fly; other filtered modes take the copy.
  const int lu_ = ch ? 1 : 2;
  const bool direct = (KIND == K_REG || KIND == K_CIIP || KIND == K_BDPCM) && (J.vnb & CS_PREFIX) && (J.vnb & CS_INTILE) &&
                      (J.vnb & CS_CORNER) && J.nul > 0 && J.nut > 0 && (!refFilter || dirMode == PLANAR);
  // ISP: region kreg of the CU (the kernel runs them in order); region k reads the CU-level lines and
  // region k-1
  {
  if (kreg == 0) PPROF(3);
  const int x0 = J.x + (ispVer ? kreg * w : 0), y0 = J.y + (isp && !ispVer ? kreg * h : 0);

  // ---- reference samples
  {
    int16_t *top = S.refU[0], *left = S.refU[1];
    if (!isp) {
      if (!interc && !direct) fill_refs(SD, D, ch, x0, y0, topLen, leftLen, mrl, bd, avlo, avhi, top, left, lane, ps, J.vnb, J.nul, J.nut);
    } else if (kreg == 0) {
      // CU-level fill of the first region (predSize per split direction), kept in refF for the others
      const int fTop = ispVer ? 2 * J.cw : J.cw + w, fLeft = ispVer ? J.ch + h : 2 * J.ch;
      PPROF(4);
      fill_refs(SD, D, 0, J.cx, J.cy, fTop, fLeft, 0, bd, avlo, avhi, top, left, lane, ps, J.vnb, J.nul, J.nut);
      IPROF(7);
      if (nreg > 1)
        for (int i = lane; i < RB; i += 64) { S.refF[0][i] = top[i]; S.refF[1][i] = left[i]; }
      IPROF(8);
    } else {
      // the shift of initIntraPatternChTypeISP (:798-897); ispPrev = last row / column of region k-1
      if (!ispVer) {   // horizontal split: left column shifted, top row from the region above
        const bool la = (J.av[2] >> (8 + kreg)) & 1;
        const int sh = kreg * h;
        const int16_t src0 = S.ispPrev[0];
        for (int i = lane; i <= leftLen; i += 64) left[i] = la ? S.refF[1][i + sh] : src0;
        const int16_t corner = la ? S.refF[1][sh] : src0;
        const int16_t last = S.ispPrev[w - 1];
        for (int i = lane; i <= topLen; i += 64) top[i] = i == 0 ? corner : (i <= w ? S.ispPrev[i - 1] : last);
      } else {         // vertical split: top row shifted, left column from the region to the left
        const bool aa = (J.av[2] >> (8 + kreg)) & 1;
        const int sh = kreg * w;
        const int16_t src0 = S.ispPrev[0];
        for (int i = lane; i <= topLen; i += 64) top[i] = aa ? S.refF[0][i + sh] : src0;
        const int16_t corner = aa ? S.refF[0][sh] : src0;
        const int16_t last = S.ispPrev[h - 1];
        for (int i = lane; i <= leftLen; i += 64) left[i] = i == 0 ? corner : (i <= h ? S.ispPrev[i - 1] : last);
      }
    }
  }
  if (kreg == 0) IPROF_POST(2);
  if (kreg == 0) store_resid();   // read after the wave syncs that follow
  wsync();
  if (kreg == 0) IPROF_POST(3);

  if (refFilter && !direct) {
    const int pS = topLen, pH = leftLen;
    for (int i = lane; i <= pS; i += 64) {
      int v;
      if (i == 0) v = (S.refU[0][0] + S.refU[0][1] + S.refU[1][0] + S.refU[1][1] + 2) >> 2;
      else if (i == pS) v = S.refU[0][pS];
      else v = (S.refU[0][i - 1] + 2 * S.refU[0][i] + S.refU[0][i + 1] + 2) >> 2;
      S.refF[0][i] = (int16_t)v;
    }
    for (int i = lane; i <= pH; i += 64) {
      int v;
      if (i == 0) v = (S.refU[0][0] + S.refU[0][1] + S.refU[1][0] + S.refU[1][1] + 2) >> 2;
      else if (i == pH) v = S.refU[1][pH];
      else v = (S.refU[1][i - 1] + 2 * S.refU[1][i] + S.refU[1][i + 1] + 2) >> 2;
      S.refF[1][i] = (int16_t)v;
    }
    wsync();
  }
  if (kreg == 0) IPROF_POST(4);
#ifdef VVCR_DIAG_DUMP
  if (gj == 0 && kreg == 0) {
    if (lane < 16) { g_dbg[lane] = S.refU[0][lane]; g_dbg[16 + lane] = S.refU[1][lane]; g_dbg[32 + lane] = S.refF[0][lane]; }
    for (int i = lane; i < RB; i += 64) { g_dbg[256 + i] = S.refU[0][i]; g_dbg[512 + i] = S.refF[0][i]; g_dbg[768 + i] = S.refF[1][i]; }
    if (lane == 0) { g_dbg[56] = topLen; g_dbg[57] = leftLen; }
    if (lane == 0) { g_dbg[48] = (int)J.av[0]; g_dbg[49] = (int)J.av[1]; g_dbg[50] = (int)J.av[2]; g_dbg[51] = J.mode;
                     g_dbg[52] = refFilter; g_dbg[53] = predMode; g_dbg[54] = applyPDPC; g_dbg[55] = J.flags; }
  }
#endif
  const int16_t *top = refFilter ? S.refF[0] : S.refU[0];
  const int16_t *left = refFilter ? S.refF[1] : S.refU[1];
  // line views: element j of the top / left reference line (0 = corner), in place or from the copy
  const int dcb = SD.base + (y0 - 1 - mrl - SD.y0) * SD.ts + (x0 - 1 - mrl - SD.x0);   // tile index of the corner
  const int16_t *tp_ = direct ? &s_tile[dcb] : top, *lp_ = direct ? &s_tile[dcb] : left;
  const int lst_ = direct ? SD.ts : 1;
  const int tlast_ = direct ? mrl + (J.nut << lu_) : (1 << 20), llast_ = direct ? mrl + (J.nul << lu_) : (1 << 20);
  const bool ffilt_ = direct && refFilter;   // planar on in-place lines: [1 2 1] on the fly (never at index 0 / the end)
  auto rawT = [&](int j) { return (int)tp_[min(j, tlast_)]; };
  auto rawL = [&](int i) { return (int)lp_[min(i, llast_) * lst_]; };
  auto TOPv = [&](int j) { return ffilt_ ? (rawT(j - 1) + 2 * rawT(j) + rawT(j + 1) + 2) >> 2 : rawT(j); };
  auto LEFTv = [&](int i) { return ffilt_ ? (rawL(i - 1) + 2 * rawL(i) + rawL(i + 1) + 2) >> 2 : rawL(i); };
  // ---- prediction fused with the reconstruction. Each lane takes groups of GS = min(4, w) consecutive
  // samples of a row: pred(xx, yy) gives a sample's prediction in registers, then the CIIP blend
  // (geneWeightedPred), the residual (from the registers prefetched at entry when their layout is the
  // block's, else from LDS / HBM), the LMCS chroma scale and the clip, and the final samples go to the LDS
  // tile once (and to HBM, sc1, when another CTU reads them).
  const DPlane &PP = P.pred[comp];
  const int tb = tile_base(comp), tp = tile_pitch(comp);
  const int ptb = tb + (y0 - G.cy0(comp)) * tp + (x0 - G.cx0(comp));
  const bool publish = (J.flags & IJ_PUBLISH) != 0;
  auto finish = [&](auto pred) {
#ifndef VVCR_ABL_RECON
    // one sample: CIIP blend, residual, LMCS chroma scale, clip; ISP keeps the region's last row / column
    auto recon1 = [&](int xx, int yy, int rr) {
      int pv = pred(xx, yy);
      if (ciip) {
        int ip = pel(PP, x0 + xx, y0 + yy);
        if (comp == 0 && (P.lmcs & 1)) ip = P.lmcs_fwd[ip];   // LMCS: mapped inter prediction (DecCu.cpp:696)
        pv = ((4 - J.ciip_w) * ip + J.ciip_w * pv + 2) >> 2;
      }
      if (cscale) rr = scale_resi(rr, cscale, bd);
      const int v = clampi(pv + rr, 0, maxv);
      if (isp && (ispVer ? xx == w - 1 : yy == h - 1)) S.ispPrev[ispVer ? yy : xx] = (int16_t)v;
      return v;
    };
    // Only a step that another CTU reads writes HBM here (sc1, drained before its flag); the CTU's
    // picture area is written back from the tile once the CTU is done. Every HBM store of a wave delays
    // that wave's later loads (vmcnt counts loads and stores in issue order), so interior steps issue none.
    if (rreg) {
      for (int g = lane, b = 0; (g << 2) < n; g += 64, b++) {
        const int k = g << 2, yy = k >> lw_, xx = k & (w - 1);
        // explicit selects: a runtime index into rv[] would put it in scratch
        const uint64_t r = b == 0 ? rv[0] : (b == 1 ? rv[1] : (b == 2 ? rv[2] : rv[3]));
        int v[4];
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = recon1(xx + e, yy, (int16_t)(r >> (16 * e)));
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const uint32_t pk = (uint32_t)(uint16_t)v[e] | ((uint32_t)v[e + 1] << 16);
          *(uint32_t *)&s_tile[ptb + yy * tp + xx + e] = pk;
          if (publish) st_sc1(D.p + (size_t)(y0 + yy) * D.stride + x0 + xx + e, pk);
        }
      }
    } else {
      for (int k = lane, b = 0; k < n; k += 64, b++) {
        const int yy = k >> lw_, xx = k & (w - 1);
        int rr;
        if (rsreg) {
          rr = b == 0 ? rs[0] : (b == 1 ? rs[1] : (b == 2 ? rs[2] : (b == 3 ? rs[3] : (b == 4 ? rs[4] : (b == 5 ? rs[5] : (b == 6 ? rs[6] : rs[7]))))));
        } else {
          rr = rlds ? S.resL[(y0 - ry + yy) * rw + x0 - rx + xx] : *gp(&R.p[(size_t)(y0 + yy) * R.stride + x0 + xx]);
        }
        const int v = recon1(xx, yy, rr);
        s_tile[ptb + yy * tp + xx] = (int16_t)v;
        if (publish) {   // sample pairs (w and x0 are even): the even lane stores its pair
          const int o = __shfl_xor(v, 1);
          if ((k & 1) == 0) st_sc1(D.p + (size_t)(y0 + yy) * D.stride + x0 + xx, (uint32_t)(uint16_t)v | ((uint32_t)o << 16));
        }
      }
    }
#else
    (void)pred;
#endif
  };

#ifndef VVCR_ABL_PRED
  if (interc) {
    // ---------------- chroma of an inter CU (LMCS chroma residual scaling): the MC prediction
    const DPlane &PI = P.pred[comp];
    finish([&](int xx, int yy) { return pel(PI, x0 + xx, y0 + yy); });
  } else if (lmMode) {
    // ---------------- CCLM (xGetLumaRecPixels + xGetLMParameters)
    const Src SY = src_of(P, 0, G);
    const DPlane &Y = P.reco[0];
    const int lx = 2 * x0, ly = 2 * y0;
    // luma-template availability: luma map in a single tree, chroma map in a separate chroma tree
    const NbAvail lr = nb_decode(J.av[2] >> 16), lm = nb_decode(J.av[3]);
    const int mode = J.mode;
    const int addAR = (mode == MDLM_L || mode == MDLM_T) ? lr.ar * 2 : 0;
    const int addBL = (mode == MDLM_L || mode == MDLM_T) ? lr.bl * 2 : 0;
    const bool firstRowCtu = (ly & (P.ctu - 1)) == 0;
    // luma loads in batches (templates + 256 down-sampled samples first): every load of a batch is
    // issued before the first wait
    const int nT = lr.above ? w + addAR : 0, nLt = lr.left ? h + addBL : 0;
    int ta[6] = {0, 0, 0, 0, 0, 0}, tl[6] = {0, 0, 0, 0, 0, 0};
    // template rows / columns only where they are used (outside the CTU they cost an HBM round trip)
    {
      const int c = lx + 2 * lane;
      const int cl = (lane == 0 && !lr.left) ? c : c - 1;
      const int r = ly + 2 * lane;
      const int Xs[12] = {cl, c, c + 1, cl, c, c + 1, lx - 3, lx - 2, lx - 1, lx - 3, lx - 2, lx - 1};
      const int Ys[12] = {ly - 2, ly - 2, ly - 2, ly - 1, ly - 1, ly - 1, r, r, r, r + 1, r + 1, r + 1};
      int cx[12], cy[12], tv12[12];
      bool need[12];
#pragma unroll
      for (int k = 0; k < 12; k++) {
        cx[k] = clampi(Xs[k], 0, Y.w - 1); cy[k] = clampi(Ys[k], 0, Y.h - 1);
        need[k] = k < 6 ? (lane < nT && (k >= 3 || !firstRowCtu)) : lane < nLt;
      }
      gather(SY, cx, cy, need, tv12);
#pragma unroll
      for (int k = 0; k < 6; k++) { ta[k] = tv12[k]; tl[k] = tv12[6 + k]; }
    }
    auto aux_batch = [&](int k0, bool stores_tmpl) {
      int v[4][6];
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int k = min(k0 + 64 * b, n - 1);
        const int yy = k >> lw_, xx = k & (w - 1);
        const int c = lx + 2 * xx, r = ly + 2 * yy;
        const int cl = (xx == 0 && !lr.left) ? c : c - 1;
        const int Xs[6] = {cl, c, c + 1, cl, c, c + 1}, Ys[6] = {r, r, r, r + 1, r + 1, r + 1};
        const bool need[6] = {true, true, true, true, true, true};
        gather(SY, Xs, Ys, need, v[b]);
      }
      if (stores_tmpl) {
        if (lane < nT)
          S.tmpl[0][lane] = (int16_t)(firstRowCtu ? (ta[4] * 2 + ta[3] + ta[5] + 2) >> 2
                                                : ((ta[1] * 2 + ta[0] + ta[2]) + (ta[4] * 2 + ta[3] + ta[5]) + 4) >> 3);
        if (lane < nLt) S.tmpl[1][lane] = (int16_t)(((tl[1] * 2 + tl[0] + tl[2]) + (tl[4] * 2 + tl[3] + tl[5]) + 4) >> 3);
      }
#pragma unroll
      for (int b = 0; b < 4; b++)
        if (k0 + 64 * b < n)
          S.aux[k0 + 64 * b] = ((v[b][1] * 2 + v[b][2] + v[b][0]) + (v[b][4] * 2 + v[b][5] + v[b][3]) + 4) >> 3;
    };
    aux_batch(lane, true);
    for (int k0 = lane + 256; k0 < n; k0 += 256) aux_batch(k0, false);
    wsync();
    int la_ = 0, lb_ = 1 << (bd - 1), lshift = 0;
    {   // every lane derives the (uniform) model; no lane-divergent region (see the dependency wait)
      bool aboveAv = lm.above, leftAv = lm.left;
      int avAR = lm.ar, avBL = lm.bl;
      const int avA = aboveAv ? w / 2 : 0, avL = leftAv ? h / 2 : 0;   // units of 2 chroma samples
      int topN = 0, leftN = 0;
      if (mode == MDLM_T) {
        leftAv = false;
        avAR = avAR > (h / 2) ? h / 2 : avAR;
        topN = 2 * (avA + avAR);
      } else if (mode == MDLM_L) {
        aboveAv = false;
        avBL = avBL > (w / 2) ? w / 2 : avBL;
        leftN = 2 * (avL + avBL);
      } else {
        topN = w;
        leftN = h;
      }
      const int aboveIs4 = leftAv ? 0 : 1, leftIs4 = aboveAv ? 0 : 1;
      const int sp0 = topN >> (2 + aboveIs4), st0 = max(1, topN >> (1 + aboveIs4));
      const int sp1 = leftN >> (2 + leftIs4), st1 = max(1, leftN >> (1 + leftIs4));
      int sl[4] = {0, 0, 0, 0}, sc[4] = {0, 0, 0, 0};
      int cntT = 0, cntL = 0;
      if (aboveAv) {
        cntT = min(topN, (1 + aboveIs4) << 1);
        for (int pos = sp0, c = 0; c < cntT; pos += st0, c++) { sl[c] = S.tmpl[0][pos]; sc[c] = S.refU[0][1 + pos]; }
      }
      if (leftAv) {
        cntL = min(leftN, (1 + leftIs4) << 1);
        for (int pos = sp1, c = 0; c < cntL; pos += st1, c++) { sl[c + cntT] = S.tmpl[1][pos]; sc[c + cntT] = S.refU[1][1 + pos]; }
      }
      if (cntT + cntL == 2) {
        sl[3] = sl[0]; sc[3] = sc[0];
        sl[2] = sl[1]; sc[2] = sc[1];
        sl[0] = sl[1]; sc[0] = sc[1];
        sl[1] = sl[3]; sc[1] = sc[3];
      }
      int mn[2] = {0, 2}, mx[2] = {1, 3};
      int *a0 = mn, *a1 = mx;
      if (sl[a0[0]] > sl[a0[1]]) { int t = a0[0]; a0[0] = a0[1]; a0[1] = t; }
      if (sl[a1[0]] > sl[a1[1]]) { int t = a1[0]; a1[0] = a1[1]; a1[1] = t; }
      if (sl[a0[0]] > sl[a1[1]]) { int *t = a0; a0 = a1; a1 = t; }
      if (sl[a0[1]] > sl[a1[0]]) { int t = a0[1]; a0[1] = a1[0]; a1[0] = t; }
      const int minL = (sl[a0[0]] + sl[a0[1]] + 1) >> 1, minC = (sc[a0[0]] + sc[a0[1]] + 1) >> 1;
      const int maxL = (sl[a1[0]] + sl[a1[1]] + 1) >> 1, maxC = (sc[a1[0]] + sc[a1[1]] + 1) >> 1;
      if (leftAv || aboveAv) {
        const int diff = maxL - minL;
        if (diff > 0) {
          const int diffC = maxC - minC;
          int x = ilog2(diff);
          const uint8_t divSig[16] = {0, 7, 6, 5, 5, 4, 4, 3, 3, 2, 2, 1, 1, 1, 1, 0};
          const int normDiff = (diff << 4 >> x) & 15;
          const int v = divSig[normDiff] | 8;
          x += normDiff != 0;
          const int y = ilog2(abs(diffC)) + 1;
          const int add = 1 << y >> 1;
          la_ = (diffC * v + add) >> y;
          lshift = 3 + x - y;
          if (lshift < 1) {
            lshift = 1;
            la_ = (la_ == 0) ? 0 : (la_ < 0) ? -15 : 15;
          }
          lb_ = minC - ((la_ * minL) >> lshift);
        } else {
          la_ = 0; lb_ = minC; lshift = 0;
        }
      }
    }
    finish([&](int xx, int yy) { return clampi(((la_ * S.aux[(yy << lw_) + xx]) >> lshift) + lb_, 0, maxv); });
  } else if (mip) {
    // ---------------- MIP
    const int sizeId = (w == 4 && h == 4) ? 0 : ((w == 4 || h == 4 || (w == 8 && h == 8)) ? 1 : 2);
    const int bdry = sizeId == 0 ? 2 : 4, rp = sizeId < 2 ? 4 : 8;
    const bool tr = (J.flags & IJ_MIP_T) != 0;
    // boundaryDownsampling1D of top (w) and left (h): one lane per reduced sample
    if (lane < 2 * bdry) {
      const int side = lane >= bdry, d = lane - side * bdry;
      const int len = side ? h : w;
      const int16_t *src = side ? S.refU[1] : S.refU[0];
      if (bdry < len) {
        const int f = len / bdry, lf = ilog2(f);
        int sum = 0;
        for (int k = 0; k < f; k++) sum += src[1 + d * f + k];
        S.red[lane] = (sum + (1 << (lf - 1))) >> lf;
      } else {
        S.red[lane] = src[1 + d];
      }
    }
    wsync();
    const int inputSize = 2 * bdry;
    int inb[8];
#pragma unroll
    for (int i = 0; i < 8; i++) inb[i] = i < inputSize ? (tr ? S.red[i < bdry ? bdry + i : i - bdry] : S.red[i]) : 0;
    const int inOff = inb[0];
    inb[0] = sizeId < 2 ? ((1 << (bd - 1)) - inOff) : 0;
    int sum = inb[0];
#pragma unroll
    for (int i = 1; i < 8; i++) {
      if (i < inputSize) inb[i] -= inOff;
      sum += inb[i];
    }
    const int offset = 32 - 32 * sum;   // (1 << (MIP_SHIFT_MATRIX - 1)) - MIP_OFFSET_MATRIX * sum
    const int mode = J.mode;
    (void)mode;
    if (lane < rp * rp) {   // rp * rp <= 64: one output per lane, its matrix row prefetched in mw[]
      const int o = lane;
      int acc = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (i >= inputSize) break;
        acc += inb[i] * mw[i];
      }
      const int v = clampi(((acc + offset) >> 6) + inOff, 0, maxv);
      // transposed matrices produce the transposed block
      const int oy = o >> (rp == 8 ? 3 : 2), ox = o & (rp - 1);
      S.aux[tr ? ox * rp + oy : o] = v;
    }
    wsync();
    const int upH = w / rp, upV = h / rp;
    // predictionUpsampling (:252-277): the horizontally upsampled row grid, then vertically
    auto hval = [&](int rr, int cx) -> int {
      if (upH <= 1) return S.aux[rr * rp + cx];
      const int lf = ilog2(upH);
      const int c = cx >> ilog2(upH), pos = cx - c * upH + 1;
      const int before = c == 0 ? (int)S.refU[1][1 + (rr + 1) * upV - 1] : S.aux[rr * rp + c - 1];
      const int behind = S.aux[rr * rp + c];
      return (before * (upH - pos) + behind * pos + (1 << (lf - 1))) >> lf;
    };
    finish([&](int xx, int yy) {
      if (upV <= 1) return hval(yy, xx);
      const int lf = ilog2(upV);
      const int r = yy >> ilog2(upV), pos = yy - r * upV + 1;
      const int before = r == 0 ? (int)S.refU[0][1 + xx] : hval(r - 1, xx);
      const int behind = hval(r, xx);
      return (before * (upV - pos) + behind * pos + (1 << (lf - 1))) >> lf;
    });
  } else {
    // ---------------- planar / DC / angular / BDPCM
    const int lw = ilog2(w), lh = ilog2(h);
    const bool pdpcPD = applyPDPC && !bdpcm && (dirMode == PLANAR || dirMode == DC);
    const int pdScale = (lw - 2 + lh - 2 + 2) >> 2;
    // PDPC of planar / DC (xPredIntraPlanar / DC + the PDPC of predIntraAng)
    auto pdpc = [&](int v, int xx, int yy) {
      if (!pdpcPD) return v;
      const int wT = 32 >> min(31, (yy << 1) >> pdScale);
      const int wL = 32 >> min(31, (xx << 1) >> pdScale);
      return (int)(int16_t)(v + ((wL * (LEFTv(yy + 1) - v) + wT * (TOPv(xx + 1) - v) + 32) >> 6));
    };
    if (bdpcm) {
      const bool hor = J.mode == 1;
      finish([&](int xx, int yy) { return hor ? LEFTv(yy + 1) : TOPv(xx + 1); });
    } else if (dirMode == PLANAR) {
      const int tr = TOPv(w + 1), bl = LEFTv(h + 1);
      finish([&](int xx, int yy) {
        const int lv = LEFTv(yy + 1), tv = TOPv(xx + 1);
        const int hor = (lv << lw) + (xx + 1) * (tr - lv);
        const int ver = (tv << lh) + (yy + 1) * (bl - tv);
        return pdpc(((hor << lh) + (ver << lw) + (1 << (lw + lh))) >> (1 + lw + lh), xx, yy);
      });
    } else if (dirMode == DC) {
      int part = 0;
      if (w >= h) part += lane < w ? TOPv(mrl + 1 + lane) : 0;
      if (w <= h) part += lane < h ? LEFTv(mrl + 1 + lane) : 0;
      const int sum = wave_sum(part);
      const int denom = (w == h) ? (w << 1) : max(w, h);
      const int dc = (sum + (denom >> 1)) >> ilog2(denom);
      finish([&](int xx, int yy) { return pdpc(dc, xx, yy); });
    } else {
      // angular (xPredIntraAng): positive and zero angles read the main / side lines in place, the main
      // one clamped at its end (the reference extends it with its last sample); negative angles build the
      // main reference with its projected side part first
      const int W = isModeVer ? w : h, H = isModeVer ? h : w;   // in the (possibly transposed) frame
      // main / side lines as (pointer, stride, last index), resolved once: in place (tile, or refU / refF)
      // for non-negative angles, the built references for negative ones. (Angular steps never use the
      // on-the-fly smoothing: a smoothed angular step takes the refF copy.)
      const int lastM = (isModeVer ? topLen : leftLen);   // last index of the main line past mrl (mainLen)
      const int16_t *mP = isModeVer ? tp_ : lp_, *sP = isModeVer ? lp_ : tp_;
      int mSt = isModeVer ? 1 : lst_, sSt = isModeVer ? lst_ : 1;
      int mLast = min(isModeVer ? tlast_ : llast_, lastM + mrl), sLast = isModeVer ? llast_ : tlast_;
      if (angle < 0) {
        int16_t *refMain = S.mainA + EXT, *refSide = S.sideA + EXT;
        for (int k = lane; k <= W + 1 + mrl; k += 64) refMain[k] = mP[min(k, mLast) * mSt];
        for (int k = lane; k <= H + 1 + mrl; k += 64) refSide[k] = sP[min(k, sLast) * sSt];
        for (int k = -H + lane; k <= -1; k += 64) refMain[k] = sP[min(min((-k * invAngle + 256) >> 9, H), sLast) * sSt];
        wsync();
        mP = refMain; sP = refSide; mSt = sSt = 1; mLast = sLast = 1 << 20;
      }
      // rM / rS of xPredIntraAng (main / side reference from index mrl on)
      auto rM = [&](int j) { return (int)mP[min(j + mrl, mLast) * mSt]; };
      auto rS = [&](int j) { return (int)sP[min(j + mrl, sLast) * sSt]; };
      const bool integerSlope = (absAng & 31) == 0;
      const int scale0 = (ilog2(W) + ilog2(H) - 2) >> 2;
      finish([&](int ox, int oy) {
        const int xx = isModeVer ? ox : oy, yy = isModeVer ? oy : ox;   // transposed-frame coordinates
        int v;
        if (angle == 0) {
          v = rM(xx + 1);
          if (applyPDPC && xx < min(3 << scale0, W)) {
            const int wL = 32 >> (2 * xx >> scale0);
            v = clampi(v + ((wL * (rS(1 + yy) - rM(0)) + 32) >> 6), 0, maxv);
          }
        } else {
          const int deltaPos = angle * (1 + mrl) + yy * angle;
          const int di = deltaPos >> 5, df = deltaPos & 31;
          if (!integerSlope) {
            if (comp == 0) {
              int f[4];
              if (!interp) {
                const uint32_t cw = *reinterpret_cast<const uint32_t *>(&s_cubic[df][0]);   // df differs per lane: LDS, one read
#pragma unroll
                for (int t = 0; t < 4; t++) f[t] = (int)(int8_t)(cw >> (8 * t));
              } else {
                f[0] = 16 - (df >> 1); f[1] = 32 - (df >> 1); f[2] = 16 + (df >> 1); f[3] = df >> 1;
              }
              const int j0 = di + xx;
              const int sm = f[0] * rM(j0) + f[1] * rM(j0 + 1) + f[2] * rM(j0 + 2) + f[3] * rM(j0 + 3);
              v = clampi((sm + 32) >> 6, 0, maxv);
            } else {
              const int p0 = rM(di + xx + 1), p1 = rM(di + xx + 2);
              v = p0 + ((df * (p1 - p0) + 16) >> 5);
            }
          } else {
            v = rM(xx + di + 1);
          }
          if (applyPDPC && xx < min(3 << angScale, W)) {
            const int invSum = 256 + (xx + 1) * invAngle;
            const int wL = 32 >> (2 * xx >> angScale);
            const int l = rS(yy + (invSum >> 9) + 1);
            v = (int16_t)(v + ((wL * (l - v) + 32) >> 6));
          }
        }
        return v;
      });
    }
  }
#else
  finish([&](int, int) { return 0; });
#endif
#ifndef VVCR_IPROF_FILL
  if (kreg == 0) IPROF(5);
#endif
  wsync();
  }   // regions
#ifndef VVCR_IPROF_FILL
  IPROF(6);
#endif
}

// Persistent: each workgroup takes CTUs (that have steps) in the plan's order (wavefront) from an
// atomic counter; its waves take the CTU's steps in topological order from an LDS counter. A CTU only
// waits for CTUs taken before it (left / above neighbours), and a step only for earlier steps, so every
// wave progresses.
// state[0] = CTU counter, state[16 + i] = global flag of published step i; *err set if a wait times out.
__global__ __launch_bounds__(64 * NW) void k_intra(const IntraParams *__restrict__ Pg, const IntraJob *__restrict__ jobs,
                                                   const int32_t *__restrict__ ctu_list, const int32_t *__restrict__ ctu_start,
                                                   int nctu, const int32_t *__restrict__ dep_start,
                                                   const int32_t *__restrict__ deps, int32_t *state, int32_t *err) {
  __shared__ int s_ctu, s_next;
  __shared__ __attribute__((aligned(16))) uint32_t s_Praw[sizeof(IntraParams) / 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // The intra chain is latency bound and shares its CUs with the B pictures' kernels of other lanes:
  // its waves take issue priority over them.
  __builtin_amdgcn_s_setprio(VVCR_INTRA_PRIO);
  int32_t *done = state + 16;
  WaveScratch &S = s_ws[wid];
  // The parameters live in LDS for the whole launch: every plane pointer / size the step body reads is
  // an LDS read, never a vector-memory load queued behind the wave's HBM traffic.
  static_assert(sizeof(IntraParams) % 4 == 0, "IntraParams copy");
  for (int i = tid; i < (int)(sizeof(IntraParams) / 4); i += 64 * NW) s_Praw[i] = ((const uint32_t *)Pg)[i];
  if (tid < 128) (&s_cubic[0][0])[tid] = (&i_chroma[0][0])[tid];
  const IntraParams &P = *reinterpret_cast<const IntraParams *>(s_Praw);
  for (;;) {
    if (tid == 0) { s_ctu = atomicAdd(&state[0], 1); s_next = 0; }
    __syncthreads();
    const int c = s_ctu;
    if (c >= nctu) break;
    const int cl = P.ctu_log2, ctu = 1 << cl;
    const int wc = (P.reco[0].w + ctu - 1) >> cl;
    const int cy = ctu_list[c] / wc, cx = ctu_list[c] - cy * wc;
    TileGeo G;
    G.x0 = cx << cl; G.y0 = cy << cl;
    G.w = min(ctu, P.reco[0].w - G.x0); G.h = min(ctu, P.reco[0].h - G.y0);
    const int j0 = ctu_start[c], nj = ctu_start[c + 1] - j0;
    // tile <- picture (inter CUs were reconstructed by k_recon_inter; intra areas are overwritten
    // before any step reads them), 4 samples per load
    for (int k = 0; k < 3; k++) {
      const DPlane &D = P.reco[k];
      const int q = G.cw(k) >> 2, tb = tile_base(k), tp = tile_pitch(k), lq = ilog2(q);
      for (int i = tid; i < q * G.ch(k); i += 64 * NW) {
        const int yy = i >> lq, xx = (i & (q - 1)) * 4;
        const uint64_t v = *gp((const uint64_t *)&D.p[(size_t)(G.cy0(k) + yy) * D.stride + G.cx0(k) + xx]);
        *(uint32_t *)&s_tile[tb + yy * tp + xx] = (uint32_t)v;
        *(uint32_t *)&s_tile[tb + yy * tp + xx + 2] = (uint32_t)(v >> 32);
      }
    }
    for (int i = tid; i < nj; i += 64 * NW) s_ldone[i] = 0;
    // Warm the XCD's L2 with the CTU's residual (written by k_resid long before): a step's residual
    // load then hits L2 instead of paying an HBM round trip on the dependency chain. The loaded values
    // only feed an opaque register move, so nothing waits for them here.
    for (int k = 0; k < 3; k++) {
      const DPlane &R = P.resi[k];
      const int q = G.cw(k) >> 3, lq = ilog2(q);   // 8 samples (16 B) per load
      for (int i = tid; i < q * G.ch(k); i += 64 * NW) {
        const int yy = i >> lq, xx = (i & (q - 1)) * 8;
        const uint64_t v = *gp((const uint64_t *)&R.p[(size_t)(G.cy0(k) + yy) * R.stride + G.cx0(k) + xx]);
        asm volatile("" :: "v"(v));
      }
    }
    __syncthreads();
    // One iteration per step, and per region of an ISP step (kreg / nk): the regions are iterations of
    // this loop so that nothing of a region's set-up is loop-invariant (run_step).
    IntraJob J{};
    int lj = 0, gj = 0, kreg = 0, nk = 0;
    unsigned long long t_ready = 0, ps[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#ifdef VVCR_INTRA_PROF
    unsigned long long t0 = 0;
#endif
    for (;;) {
      if (kreg == nk) {
        // uniform control flow only (no lane-0 regions anywhere around the step body): every lane adds,
        // lane 0 adds 1, and lane 0's result is the step
        lj = __builtin_amdgcn_readfirstlane(atomicAdd(&s_next, lane == 0 ? 1 : 0));
        if (lj >= nj) break;
        gj = j0 + lj;
        J = jobs[gj];
        kreg = 0;
        nk = (J.flags & (IJ_ISP_HOR | IJ_ISP_VER)) ? J.isp_k : 1;
        t_ready = 0;
#ifdef VVCR_INTRA_PROF
        for (int q = 0; q < 10; q++) ps[q] = 0;
        t0 = __builtin_amdgcn_s_memrealtime();
#endif
      }
      switch (step_kind(J)) {
        case K_REG: run_step<K_REG>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
        case K_ISP: run_step<K_ISP>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, kreg); break;
        case K_MIP: run_step<K_MIP>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
        case K_LM: run_step<K_LM>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
        case K_CIIP: run_step<K_CIIP>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
        case K_BDPCM: run_step<K_BDPCM>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
        default: run_step<K_INTERC>(P, J, G, S, dep_start, deps, gj, done, err, lane, t_ready, ps, 0); break;
      }
      if (++kreg < nk) continue;   // the step's next region
      // hand-off: LDS stores of this wave complete before its done byte; a step read by another CTU
      // also drains its HBM stores (sc1) before its global flag
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __hip_atomic_store(&s_ldone[lj], (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (J.flags & IJ_PUBLISH) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&done[gj], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#ifdef VVCR_INTRA_PROF
      if (lane == 0) {
        const unsigned int slot = atomicAdd(&g_iprof_n, 1u);
        if (slot < (1u << 17)) {
          unsigned int xcc;
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
          g_iprof[slot][0] = t0;
          g_iprof[slot][1] = t_ready;
          g_iprof[slot][2] = __builtin_amdgcn_s_memrealtime();
          g_iprof[slot][3] = (ps[1] - ps[0]) | (ps[2] - ps[0]) << 16 | (ps[3] - ps[0]) << 32 | (ps[4] - ps[0]) << 48;
          g_iprof[slot][4] = (ps[5] - ps[0]) | (ps[6] - ps[0]) << 16 | (ps[7] - ps[0]) << 32 | (ps[8] - ps[0]) << 48;
          g_iprof[slot][5] = (unsigned long long)J.comp | (unsigned long long)J.w << 8 | (unsigned long long)J.h << 16 |
                             (unsigned long long)J.flags << 24 | (unsigned long long)J.mode << 32 | (unsigned long long)(xcc & 15) << 40 |
                             (unsigned long long)J.vnb << 48;
          g_iprof[slot][6] = (unsigned long long)gj | (unsigned long long)blockIdx.x << 32;
          g_iprof[slot][7] = (unsigned long long)(uint16_t)J.x | (unsigned long long)(uint16_t)J.y << 16 | (unsigned long long)c << 32;
        }
      }
#endif
    }
    __syncthreads();   // every step of the CTU finished
    // tile -> picture (the final reconstruction of the CTU; published samples are rewritten with the
    // same values), 4 samples per store, before the tile is reused
    for (int k = 0; k < 3; k++) {
      const DPlane &D = P.reco[k];
      const int q = G.cw(k) >> 2, tb = tile_base(k), tp = tile_pitch(k), lq = ilog2(q);
      for (int i = tid; i < q * G.ch(k); i += 64 * NW) {
        const int yy = i >> lq, xx = (i & (q - 1)) * 4;
        const uint64_t v = (uint64_t)*(const uint32_t *)&s_tile[tb + yy * tp + xx] |
                           (uint64_t)*(const uint32_t *)&s_tile[tb + yy * tp + xx + 2] << 32;
        *gpw((uint64_t *)&D.p[(size_t)(G.cy0(k) + yy) * D.stride + G.cx0(k) + xx]) = v;
      }
    }
    __syncthreads();
  }
}

// One wave per inter tile (<= 16x16 luma, sides 4 / 8 / 16), four tiles per workgroup: four luma samples per lane (8-byte loads of
// the prediction and the residual), two chroma samples per lane (Cb on lanes 0..31, Cr on 32..63); all
// loads are issued before the first use.
__global__ __launch_bounds__(256) void k_recon_inter(IntraParams P, const ReconTile *__restrict__ tiles, int n) {
  const int t = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // a tile per wave
  if (t >= n) return;
  const ReconTile T = load_uniform(tiles + t);
  const int lane = threadIdx.x & 63, maxv = (1 << P.bd) - 1;
  const int w = T.w, h = T.h, lq = ilog2(w) - 2;
  const bool doY = (T.comps & 1) && lane < ((w >> 2) * h);
  const int yy = lane >> lq, xx = (lane & ((1 << lq) - 1)) * 4;
  const int cw = w >> 1, chh = h >> 1, cq = ilog2(cw) - 1, comp = 1 + (lane >> 5), cl = lane & 31;
  const bool doC = (T.comps & 2) && cl < ((cw >> 1) * chh);
  const int cy = cl >> cq, cx = (cl & ((1 << cq) - 1)) * 2;
  uint2 py = {}, ry = {};
  uint32_t pc = 0, rc = 0;
  const DPlane &DY = P.reco[0], &PY = P.pred[0], &RY = P.resi[0];
  const DPlane &DC = P.reco[comp], &PC = P.pred[comp], &RC = P.resi[comp];
  const size_t oy = (size_t)(T.y + yy) * PY.stride + T.x + xx;
  const size_t oc = (size_t)((T.y >> 1) + cy) * PC.stride + (T.x >> 1) + cx;
  if (doY) { py = *(const uint2 *)&PY.p[oy]; ry = *(const uint2 *)&RY.p[oy]; }
  if (doC) { pc = *(const uint32_t *)&PC.p[oc]; rc = *(const uint32_t *)&RC.p[oc]; }
  if (doY) {
    int pv[4] = {(int16_t)(py.x & 0xffff), (int16_t)(py.x >> 16), (int16_t)(py.y & 0xffff), (int16_t)(py.y >> 16)};
    const int rv[4] = {(int16_t)(ry.x & 0xffff), (int16_t)(ry.x >> 16), (int16_t)(ry.y & 0xffff), (int16_t)(ry.y >> 16)};
    if (P.lmcs & 1) {   // LMCS forward map of the prediction (DecCu.cpp:742,765)
#pragma unroll
      for (int e = 0; e < 4; e++) pv[e] = P.lmcs_fwd[pv[e]];
    }
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; e++) v[e] = clampi(pv[e] + rv[e], 0, maxv);
    *(uint2 *)(&DY.p[(size_t)(T.y + yy) * DY.stride + T.x + xx]) =
        make_uint2((uint32_t)(uint16_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)(uint16_t)v[2] | ((uint32_t)v[3] << 16));
  }
  if (doC) {
    const int v0 = clampi((int)(int16_t)(pc & 0xffff) + (int)(int16_t)(rc & 0xffff), 0, maxv);
    const int v1 = clampi((int)(int16_t)(pc >> 16) + (int)(int16_t)(rc >> 16), 0, maxv);
    *(uint32_t *)(&DC.p[(size_t)((T.y >> 1) + cy) * DC.stride + (T.x >> 1) + cx]) = (uint32_t)(uint16_t)v0 | ((uint32_t)v1 << 16);
  }
}

// LMCS inverse luma mapping of the whole reconstructed picture (DecLib.cpp:574 rspSignal(invLUT)), in place,
// 8 samples per lane
__global__ void k_lmcs_inverse(DPlane L, const int16_t *__restrict__ inv, int y0) {
  const int q = L.w >> 3, y = y0 + blockIdx.y, qx = blockIdx.x * blockDim.x + threadIdx.x;
  if (qx >= q) return;
  int16_t *row = L.p + (size_t)y * L.stride + qx * 8;
#pragma unroll
  for (int k = 0; k < 8; k++) row[k] = inv[row[k]];
}
}  // namespace

void launch_lmcs_inverse(const DPlane &luma, const int16_t *inv_lut, int y0, int y1, hipStream_t s) {
  if (y1 <= y0) return;
  const int q = luma.w >> 3;
  hipLaunchKernelGGL(k_lmcs_inverse, dim3((q + 63) / 64, y1 - y0), dim3(64), 0, s, luma, inv_lut, y0);
}

void launch_recon_inter(const IntraParams &p, const ReconTile *tiles, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_recon_inter, dim3((n + 3) / 4), dim3(256), 0, s, p, tiles, n);
}

void launch_intra(const IntraParams *p_dev, const IntraJob *jobs, int n, const int32_t *ctu_list, const int32_t *ctu_start,
                  int nctu, const int32_t *dep_start, const int32_t *deps, int32_t *state, int32_t *err, int n_wg,
                  hipStream_t s) {
  if (n <= 0 || nctu <= 0) return;
  VVCR_CHECK_HIP(hipMemsetAsync(state, 0, (16 + (size_t)n) * sizeof(int32_t), s));
  // n_wg persistent workgroups (the caller sizes it to the wavefront), never more than the CTUs
  hipLaunchKernelGGL(k_intra, dim3(std::min(nctu, n_wg)), dim3(64 * NW), 0, s, p_dev, jobs, ctu_list, ctu_start, nctu,
                     dep_start, deps, state, err);
}
