// vvcr_mcdev.h — device helpers shared by the motion-compensation kernels (gfx950): packed integer FIR
// on int16 sample pairs with v_dot2c_i32_i16, and the constants of InterpolationFilter.h:48-52.
#pragma once
#include "vvcr_internal.h"

namespace mcdev {

constexpr int IF_INTERNAL_PREC = 14;
constexpr int IF_FILTER_PREC = 6;
constexpr int IF_INTERNAL_OFFS = 1 << (IF_INTERNAL_PREC - 1);

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

typedef short short2_t __attribute__((ext_vector_type(2)));
// a.lo * b.lo + a.hi * b.hi + c (signed 16-bit halves)
// a * b + c over int16 pairs, always in the three-operand form: the clamp bit (an i32 saturation no sum of
// ours reaches: filter sums stay below 2^24) keeps the compiler from the two-operand v_dot2c, whose
// accumulator is its destination and costs a v_mov per chain start (13 % of k_mc's filter VALU, r04).
__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, a), __builtin_bit_cast(short2_t, b), c, true);
}
__host__ __device__ constexpr uint32_t pk(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }

// Packed pair coefficients of an N-tap filter c[0..N): A[k] = (c[2k], c[2k+1]) for an output whose first
// tap sits on an even sample of the pair sequence, B[k] = (c[2k-1], c[2k]) with c[-1] = c[N] = 0 for one
// whose first tap sits on an odd sample. Either way every operand is an aligned dword of sample pairs.
template <int N>
struct Taps {
  uint32_t A[N / 2], B[N / 2 + 1];
};
template <int N, class T>
__host__ __device__ constexpr Taps<N> make_taps(const T *c) {
  Taps<N> t{};
  for (int k = 0; k < N / 2; k++) t.A[k] = pk(c[2 * k], c[2 * k + 1]);
  t.B[0] = pk(0, c[0]);
  for (int k = 1; k < N / 2; k++) t.B[k] = pk(c[2 * k - 1], c[2 * k]);
  t.B[N / 2] = pk(c[N - 1], 0);
  return t;
}

// Four consecutive outputs from aligned sample pairs w[]: output j's first tap is element PAR + j.
template <int N, int PAR>
__device__ __forceinline__ void fir4(const uint32_t *w, const Taps<N> &t, int (&o)[4]) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int e = PAR + j;
    int s = 0;
    if ((e & 1) == 0) {
#pragma unroll
      for (int k = 0; k < N / 2; k++) s = dot2(w[e / 2 + k], t.A[k], s);
    } else {
#pragma unroll
      for (int k = 0; k < N / 2 + 1; k++) s = dot2(w[(e - 1) / 2 + k], t.B[k], s);
    }
    o[j] = s;
  }
}
// The same with a lane-dependent parity par (0 / 1); reads w[0 .. N/2 + 1].
template <int N>
__device__ __forceinline__ void fir4_var(const uint32_t *w, const Taps<N> &t, int par, int (&o)[4]) {
  uint32_t u[N / 2 + 1];
#pragma unroll
  for (int k = 0; k < N / 2 + 1; k++) u[k] = par ? w[k + 1] : w[k];
  int ea[2], eb[2];      // A over u (outputs with an even first tap), B over w (odd first tap)
#pragma unroll
  for (int m = 0; m < 2; m++) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < N / 2; k++) s = dot2(u[m + k], t.A[k], s);
    ea[m] = s;
    s = 0;
#pragma unroll
    for (int k = 0; k < N / 2 + 1; k++) s = dot2(w[m + k], t.B[k], s);
    eb[m] = s;
  }
  o[0] = par ? eb[0] : ea[0];
  o[1] = par ? ea[0] : eb[0];
  o[2] = par ? eb[1] : ea[1];
  o[3] = par ? ea[1] : eb[1];
}

// N = 4 or 8 samples of a reference row starting at column c0 (a multiple of N), the row index clamped to
// the picture: one vector load when the chunk lies inside the row, else per-sample loads with clamped
// columns. Clamping reproduces the edge-replicated margin of the reference picture
// (Picture::extendPicBorder, Picture.cpp:737), so no window needs a slower path at picture edges; the
// loads of both branches are plain issues (their wait comes at the LDS write).
__device__ __forceinline__ uint2 chunk4(const int16_t *p, int stride, int w, int h, int y, int c0) {
  const int16_t *row = p + (size_t)clampi(y, 0, h - 1) * stride;
  if (c0 >= 0 && c0 + 4 <= w) return *(const uint2 *)(row + c0);
  const int a = row[clampi(c0, 0, w - 1)], b = row[clampi(c0 + 1, 0, w - 1)];
  const int c = row[clampi(c0 + 2, 0, w - 1)], d = row[clampi(c0 + 3, 0, w - 1)];
  return make_uint2(pk(a, b), pk(c, d));
}
__device__ __forceinline__ uint4 chunk8(const int16_t *p, int stride, int w, int h, int y, int c0) {
  const int16_t *row = p + (size_t)clampi(y, 0, h - 1) * stride;
  if (c0 >= 0 && c0 + 8 <= w) return *(const uint4 *)(row + c0);
  int v[8];
#pragma unroll
  for (int e = 0; e < 8; e++) v[e] = row[clampi(c0 + e, 0, w - 1)];
  return make_uint4(pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7]));
}

// Two H-pass intermediates (a, b: filter sums) as the packed int16 pair ((a + off1) >> sh, (b + off1) >> sh)
// with off1 = -(IF_INTERNAL_OFFS << sh): shift both, take their low halves with one byte permute, and
// subtract IF_INTERNAL_OFFS from both halves with one packed 16-bit op (exact: every value fits int16).
__device__ __forceinline__ uint32_t pack_h(int a, int b, int sh) {
  const uint32_t p = __builtin_amdgcn_perm((uint32_t)(b >> sh), (uint32_t)(a >> sh), 0x05040100u);
  const short2_t r = __builtin_bit_cast(short2_t, p) - (short2_t){(short)IF_INTERNAL_OFFS, (short)IF_INTERNAL_OFFS};
  return __builtin_bit_cast(uint32_t, r);
}

__device__ __forceinline__ int lo16(uint32_t v) { return (int16_t)(v & 0xffff); }
__device__ __forceinline__ int hi16(uint32_t v) { return (int16_t)(v >> 16); }

}  // namespace mcdev
