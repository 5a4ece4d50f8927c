// vvcr_rdo.hip — the encoder's RDO inner loop for gfx950 (BASELINE config 5):
// batched SAD + Hadamard SATD of (original, prediction) block pairs and batched forward transforms.
//
// Distortion (RdCost::xGetSAD RdCost.cpp:503, RdCost::xGetHADs :2800): a block is cut into the
// Hadamard tiles xGetHADs chooses for its shape (16x8, 8x16, 8x4, 4x8, 8x8, 4x4, 2x2; :2818-2911). One
// tile = TH lanes (one tile row per lane, TW differences in registers): the row WHT runs in registers,
// the column WHT across the tile's lanes with xor-shuffles (the sum of |coefficients| does not depend
// on the order or sign of the Walsh-Hadamard basis, so the fast transform equals the reference's
// butterflies), the tile normalisation is the kernel's own ((s+1)>>1, (s+2)>>2, or
// (int)(s / sqrt(w*h) * 2) in double precision for rectangles), and the tile leader adds the tile's
// SATD and SAD to its block with one integer atomic each (order-independent, so deterministic).
// Tiles are sorted by kind on the host and each kind is one launch of its template instantiation.
//
// Forward transform (TrQuant::xT TrQuant.cpp:749-824): blocks grouped by size and transform types on
// the host, one launch per group, the matrices, residuals and first-pass outputs staged in LDS; each 1-D pass is the integer matrix product the partial
// butterflies compute (fastForwardDCT2_B* / DST7 / DCT8, TrQuant_EMT.cpp), with xT's shifts and
// zero-out; DCT2 up to 32 points ignores the output cut-off exactly as the reference does (:131-607).
#include "vvcr_internal.h"
#include "vvcr_gen_tables.h"
#include <cstdlib>

namespace {

template <int TW, int TH>
__global__ __launch_bounds__(256) void k_rd_tiles(const int16_t *__restrict__ org, const int16_t *__restrict__ cur,
                                                  const RdTile *__restrict__ tiles, int ntiles,
                                                  const RdBlockDev *__restrict__ blocks, uint32_t *sad, uint32_t *satd) {
  static_assert(TH <= 64 && (64 % TH) == 0, "tile rows map to lanes of one wave");
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gl / TH, row = gl % TH;
  const bool valid = t < ntiles;
  const RdTile T = valid ? tiles[t] : RdTile{0, 0, 0};
  const RdBlockDev B = blocks[valid ? T.block : 0];
  int d[TW];
  int s_abs = 0;
  if (valid) {
    const int16_t *o = org + B.org_off + (int64_t)(T.y + row) * B.org_stride + T.x;
    const int16_t *c = cur + B.cur_off + (int64_t)(T.y + row) * B.cur_stride + T.x;
#pragma unroll
    for (int i = 0; i < TW; i++) {
      d[i] = o[i] - c[i];
      s_abs += abs(d[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < TW; i++) d[i] = 0;
  }
  // row WHT in registers
#pragma unroll
  for (int len = 1; len < TW; len <<= 1)
#pragma unroll
    for (int i = 0; i < TW; i += 2 * len)
#pragma unroll
      for (int j = i; j < i + len; j++) {
        const int a = d[j], b = d[j + len];
        d[j] = a + b;
        d[j + len] = a - b;
      }
  // column WHT across the TH lanes of the tile
#pragma unroll
  for (int len = 1; len < TH; len <<= 1) {
    const bool hi = (row & len) != 0;
#pragma unroll
    for (int i = 0; i < TW; i++) {
      const int p = __shfl_xor(d[i], len);
      d[i] = hi ? p - d[i] : d[i] + p;
    }
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < TW; i++) s += abs(d[i]);
#pragma unroll
  for (int len = 1; len < TH; len <<= 1) {
    s += __shfl_xor(s, len);
    s_abs += __shfl_xor(s_abs, len);
  }
  if (valid && row == 0) {
    uint32_t v;
    if (TW == 2 && TH == 2) v = (uint32_t)s;
    else if (TW == 4 && TH == 4) v = (uint32_t)((s + 1) >> 1);
    else if (TW == 8 && TH == 8) v = (uint32_t)((s + 2) >> 2);
    else v = (uint32_t)(int)((double)s / sqrt((double)(TW * TH)) * 2.0);
    atomicAdd(&satd[T.block], v);
    atomicAdd(&sad[T.block], (uint32_t)s_abs);
  }
}

__device__ __forceinline__ int tr_coef(int type, int N, int k, int n) {
  if (type == 0) return vvcr_tab::dct2_64[k * (64 / N)][n];
  if (type == 1) {
    switch (N) {
      case 4: return vvcr_tab::dst7_4[k][n];
      case 8: return vvcr_tab::dst7_8[k][n];
      case 16: return vvcr_tab::dst7_16[k][n];
      default: return vvcr_tab::dst7_32[k][n];
    }
  }
  switch (N) {
    case 4: return vvcr_tab::dct8_4[k][n];
    case 8: return vvcr_tab::dct8_8[k][n];
    case 16: return vvcr_tab::dct8_16[k][n];
    default: return vvcr_tab::dct8_32[k][n];
  }
}

// Forward transform of one size class: a workgroup stages the class's two matrices in LDS once and then
// transforms NB blocks at a time (NB * W * H >= 256 samples per pass keeps the 256 lanes busy). The
// products (residual <= 11 bits or first-pass outputs <= 17 bits, times matrix entries <= 8 bits) and
// sums fit the 32-bit integer path the reference's TCoeff butterflies use, so v_mad_i32_i24 + int32
// accumulation reproduces them exactly.
template <int W, int H>
__global__ __launch_bounds__(256) void k_fwd_sz(const int16_t *__restrict__ resi, int32_t *__restrict__ coef,
                                                const FwdBlockDev *__restrict__ blocks, int n, int bd, int trh, int trv,
                                                int skipW, int cut1, int cut2) {
  constexpr int NB = (W * H >= 256) ? 1 : 256 / (W * H);
  __shared__ int16_t mh[W * W], mv[H * H];
  __shared__ int32_t x[NB * W * H], t[NB * W * H];
  const int tid = threadIdx.x;
  for (int i = tid; i < W * W; i += 256) mh[i] = (int16_t)tr_coef(trh, W, i / W, i % W);
  for (int i = tid; i < H * H; i += 256) mv[i] = (int16_t)tr_coef(trv, H, i / H, i % H);
  constexpr int lw = W == 4 ? 2 : W == 8 ? 3 : W == 16 ? 4 : W == 32 ? 5 : 6;
  constexpr int lh = H == 4 ? 2 : H == 8 ? 3 : H == 16 ? 4 : H == 32 ? 5 : 6;
  const int s1 = lw + bd + 6 - 15, s2 = lh + 6;
  const int r1 = 1 << (s1 - 1), r2 = 1 << (s2 - 1);
  for (int b0 = blockIdx.x * NB; b0 < n; b0 += gridDim.x * NB) {
    __syncthreads();   // matrices staged / previous blocks' LDS consumed
    for (int i = tid; i < NB * W * H; i += 256) {
      const int b = i / (W * H), e = i % (W * H);
      x[i] = b0 + b < n ? (int)resi[blocks[b0 + b].src_off + (int64_t)(e / W) * blocks[b0 + b].src_stride + (e % W)] : 0;
    }
    __syncthreads();
    // pass 1 (rows, fastFwdTrans[trh][W]): t[b][k * H + j] = (sum_m mh[k][m] x[b][j][m] + r1) >> s1
    for (int i = tid; i < NB * W * H; i += 256) {
      const int b = i / (W * H), e = i % (W * H), k = e / H, j = e % H;
      int v = 0;
      if (k < cut1) {
        const int32_t *xr = x + b * W * H + j * W;
        const int16_t *m = mh + k * W;
        int s = 0;
#pragma unroll
        for (int q = 0; q < W; q++) s += m[q] * xr[q];
        v = (s + r1) >> s1;
      }
      t[i] = v;
    }
    __syncthreads();
    // pass 2 (columns, fastFwdTrans[trv][H], line = W, skipLine = skipW): out[b][kv * W + i2]
    for (int i = tid; i < NB * W * H; i += 256) {
      const int b = i / (W * H), e = i % (W * H), kv = e / W, i2 = e % W;
      if (b0 + b >= n) continue;
      int v = 0;
      if (kv < cut2 && i2 < W - skipW) {
        const int32_t *tr = t + b * W * H + i2 * H;
        const int16_t *m = mv + kv * H;
        int s = 0;
#pragma unroll
        for (int q = 0; q < H; q++) s += m[q] * tr[q];
        v = (s + r2) >> s2;
      }
      coef[blocks[b0 + b].dst_off + e] = v;
    }
  }
}


// MFMA form of a size class with W, H >= 16 (the forward transform is the one dense contraction of the
// path). Both passes are 16x16x32 f16 MFMAs with f32 accumulation, and stay exact:
//  * pass 1: residuals (|x| <= 1023) and matrix entries (|m| <= 90) are exact f16 integers; every
//    partial sum is an integer below 64 * 90 * 1023 < 2^24, so f32 accumulation is exact in any order;
//  * pass 2: first-pass outputs v (|v| < 2^16) are split v = 256 * hi + lo, lo in [0, 255], |hi| <= 256,
//    both exact f16; each of the two MFMA sums stays below 64 * 90 * 256 < 2^24 and the int32
//    recombination 256 * S_hi + S_lo is exact.
// The first pass writes its output transposed (T1T[k][j]) so that the second pass reads its B fragments
// as contiguous 16-byte rows, like the first. Fragment maps (mfma_f32_16x16x32_f16): lane l holds
// A[l & 15][8 (l >> 4) + e] and B[8 (l >> 4) + e][l & 15], e = 0..7; C/D col = l & 15,
// row = 4 (l >> 4) + r.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int W, int H>
__global__ __launch_bounds__(256) void k_fwd_mfma(const int16_t *__restrict__ resi, int32_t *__restrict__ coef,
                                                  const FwdBlockDev *__restrict__ blocks, int n, int bd, int trh, int trv,
                                                  int skipW, int cut1, int cut2) {
  constexpr int TPB = (W / 16) * (H / 16);             // 16x16 output tiles per block and pass
  constexpr int NB = TPB >= 4 ? 1 : 4 / TPB;           // blocks per iteration: >= 4 tiles for the 4 waves
  constexpr int PW = W + 8, PH = H + 8;                // f16 row pitches (16-byte aligned, spread banks)
  __shared__ __attribute__((aligned(16))) _Float16 mh[W * PW], mv[H * PH];
  __shared__ __attribute__((aligned(16))) _Float16 xs[NB * H * PW];
  __shared__ __attribute__((aligned(16))) _Float16 thi[NB * W * PH], tlo[NB * W * PH];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < W * W; i += 256) mh[(i / W) * PW + i % W] = (_Float16)tr_coef(trh, W, i / W, i % W);
  for (int i = tid; i < H * H; i += 256) mv[(i / H) * PH + i % H] = (_Float16)tr_coef(trv, H, i / H, i % H);
  constexpr int lw = W == 16 ? 4 : W == 32 ? 5 : 6;
  constexpr int lh = H == 16 ? 4 : H == 32 ? 5 : 6;
  const int s1 = lw + bd + 6 - 15, s2 = lh + 6;
  const int r1 = 1 << (s1 - 1), r2 = 1 << (s2 - 1);
  const int fr = lane & 15, fk = 8 * (lane >> 4);      // fragment row / first k of this lane
  for (int b0 = blockIdx.x * NB; b0 < n; b0 += gridDim.x * NB) {
    __syncthreads();
    for (int i = tid; i < NB * W * H; i += 256) {
      const int b = i / (W * H), e = i % (W * H), y = e / W, x = e % W;
      xs[(b * H + y) * PW + x] = (_Float16)(b0 + b < n ? (int)resi[blocks[b0 + b].src_off + (int64_t)y * blocks[b0 + b].src_stride + x] : 0);
    }
    __syncthreads();
    // ---- pass 1: T1[j][k] = sum_n X[j][n] Mh[k][n]  (A = X rows, B = Mh rows as columns)
    for (int t = wv; t < NB * TPB; t += 4) {
      const int b = t / TPB, tt = t % TPB, tr = tt / (W / 16), tc = tt % (W / 16);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < W; kk += 32) {
        f16x8 a, bb;
        if (kk + fk < W) {
          a = *(const f16x8 *)&xs[(b * H + 16 * tr + fr) * PW + kk + fk];
          bb = *(const f16x8 *)&mh[(16 * tc + fr) * PW + kk + fk];
        } else {
          a = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
          bb = a;
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bb, acc, 0, 0, 0);
      }
      const int k = 16 * tc + fr;                       // output column (frequency) of this lane
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int j = 16 * tr + 4 * (lane >> 4) + r;    // output row
        const int v = k < cut1 ? (((int)acc[r]) + r1) >> s1 : 0;
        thi[(b * W + k) * PH + j] = (_Float16)(v >> 8);
        tlo[(b * W + k) * PH + j] = (_Float16)(v & 255);
      }
    }
    __syncthreads();
    // ---- pass 2: out[kv][i2] = sum_q Mv[kv][q] T1[q][i2]  (A = Mv rows, B = T1T rows as columns)
    for (int t = wv; t < NB * TPB; t += 4) {
      const int b = t / TPB, tt = t % TPB, tr = tt / (W / 16), tc = tt % (W / 16);
      f32x4 ah = {0.f, 0.f, 0.f, 0.f}, al = ah;
#pragma unroll
      for (int kk = 0; kk < H; kk += 32) {
        f16x8 a, bh, bl;
        if (kk + fk < H) {
          a = *(const f16x8 *)&mv[(16 * tr + fr) * PH + kk + fk];
          bh = *(const f16x8 *)&thi[(b * W + 16 * tc + fr) * PH + kk + fk];
          bl = *(const f16x8 *)&tlo[(b * W + 16 * tc + fr) * PH + kk + fk];
        } else {
          a = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
          bh = a;
          bl = a;
        }
        ah = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bh, ah, 0, 0, 0);
        al = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bl, al, 0, 0, 0);
      }
      if (b0 + b < n) {
        const int i2 = 16 * tc + fr;
        int32_t *dst = coef + blocks[b0 + b].dst_off;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int kv = 16 * tr + 4 * (lane >> 4) + r;
          const int sum = (int)ah[r] * 256 + (int)al[r];
          dst[kv * W + i2] = (kv < cut2 && i2 < W - skipW) ? (sum + r2) >> s2 : 0;
        }
      }
    }
  }
}

}  // namespace

// VVCR_FWD_MFMA=0 selects the int32 VALU kernels for every class (A/B and fallback)
static const bool g_fwd_mfma = [] { const char *e = getenv("VVCR_FWD_MFMA"); return !(e && e[0] == '0'); }();

void launch_rd_tiles(int kind, const int16_t *org, const int16_t *cur, const RdTile *tiles, int n, const RdBlockDev *blocks,
                     uint32_t *sad, uint32_t *satd, hipStream_t s) {
  if (n <= 0) return;
  static const int lanes[RD_KINDS] = {8, 16, 4, 8, 8, 4, 2};   // tile rows per kind
  const int g = (n * lanes[kind] + 255) / 256;
  switch (kind) {
    case RD_16x8: hipLaunchKernelGGL((k_rd_tiles<16, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x16: hipLaunchKernelGGL((k_rd_tiles<8, 16>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x4: hipLaunchKernelGGL((k_rd_tiles<8, 4>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_4x8: hipLaunchKernelGGL((k_rd_tiles<4, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x8: hipLaunchKernelGGL((k_rd_tiles<8, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_4x4: hipLaunchKernelGGL((k_rd_tiles<4, 4>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    default: hipLaunchKernelGGL((k_rd_tiles<2, 2>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
  }
}

template <int W, int H>
static void launch_sz(const int16_t *resi, int32_t *coef, const FwdBlockDev *blocks, int n, int bd, int trh, int trv, int skipW,
                      int cut1, int cut2, hipStream_t s) {
  if constexpr (W >= 16 && H >= 16) {
    if (g_fwd_mfma) {
      constexpr int TPB = (W / 16) * (H / 16), NB = TPB >= 4 ? 1 : 4 / TPB;
      const int g = std::min((n + NB - 1) / NB, 4096);
      hipLaunchKernelGGL((k_fwd_mfma<W, H>), dim3(g), dim3(256), 0, s, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2);
      return;
    }
  }
  constexpr int NB = (W * H >= 256) ? 1 : 256 / (W * H);
  const int g = std::min((n + NB - 1) / NB, 4096);
  hipLaunchKernelGGL((k_fwd_sz<W, H>), dim3(g), dim3(256), 0, s, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2);
}
template <int W>
static void launch_w(int h, const int16_t *resi, int32_t *coef, const FwdBlockDev *blocks, int n, int bd, int trh, int trv,
                     int skipW, int cut1, int cut2, hipStream_t s) {
  switch (h) {
    case 4: launch_sz<W, 4>(resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 8: launch_sz<W, 8>(resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 16: launch_sz<W, 16>(resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 32: launch_sz<W, 32>(resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    default: launch_sz<W, 64>(resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
  }
}

// One launch per class of blocks sharing (w, h, trh, trv, lfnst), blocks[0, n) of the class; the
// zero-out of TrQuant::xT (:762-777) and the per-type output cut-off are uniform per class.
void launch_fwd_tr(const int16_t *resi, int32_t *coef, const FwdBlockDev *blocks, int n, int bd, int w, int h, int trh,
                   int trv, int lfnst, hipStream_t s) {
  if (n <= 0) return;
  int skipW = (trh != 0 && w == 32) ? 16 : (w > 32 ? w - 32 : 0);
  int skipH = (trv != 0 && h == 32) ? 16 : (h > 32 ? h - 32 : 0);
  if (lfnst) {
    if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
    else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
  }
  const int cut1 = (trh == 0 && w <= 32) ? w : w - skipW, cut2 = (trv == 0 && h <= 32) ? h : h - skipH;
  switch (w) {
    case 4: launch_w<4>(h, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 8: launch_w<8>(h, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 16: launch_w<16>(h, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    case 32: launch_w<32>(h, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
    default: launch_w<64>(h, resi, coef, blocks, n, bd, trh, trv, skipW, cut1, cut2, s); break;
  }
}
