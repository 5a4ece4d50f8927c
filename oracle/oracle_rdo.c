/*
 * oracle_rdo.c — TEST INFRASTRUCTURE. Plain-C restatement of the encoder RDO distortion kernels of
 * VTM 7.3: RdCost::xGetSAD (RdCost.cpp:503) and RdCost::xGetHADs
 * (RdCost.cpp:2800) with the Hadamard block kernels xCalcHADs2x2 / 4x4 / 8x8 / 16x8 / 8x16 / 4x8 / 8x4
 * (:2150-2798). Pinned against the reference's own outputs (tests/golden/rdo, oracle/capture/rdo_kat.cpp).
 * Never linked into the product.
 *
 * The reference writes each Hadamard kernel as explicit butterflies; the sum of absolute transform
 * coefficients does not depend on the order (or signs) of the Walsh-Hadamard basis, so one in-place
 * fast WHT per dimension computes the same sums. Normalisations: 2x2 none, 4x4 (s+1)>>1, 8x8 (s+2)>>2,
 * rectangles (int)(s / sqrt(w*h) * 2) in double precision.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

uint32_t or_sad(const int16_t *org, int os, const int16_t *cur, int cs, int w, int h) {
  uint32_t s = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) s += (uint32_t)abs(org[y * os + x] - cur[y * cs + x]);
  return s;   /* DISTORTION_PRECISION_ADJUSTMENT = 0 (TypeDef.h:287) */
}

static void wht(int32_t *v, int n, int stride) {
  for (int len = 1; len < n; len <<= 1)
    for (int i = 0; i < n; i += 2 * len)
      for (int j = i; j < i + len; j++) {
        const int32_t a = v[j * stride], b = v[(j + len) * stride];
        v[j * stride] = a + b;
        v[(j + len) * stride] = a - b;
      }
}

/* one bw x bh Hadamard block: sum |H_bh D H_bw^T| with the kernel's normalisation */
static uint32_t had_block(const int16_t *org, int os, const int16_t *cur, int cs, int bw, int bh) {
  int32_t d[128];
  for (int y = 0; y < bh; y++)
    for (int x = 0; x < bw; x++) d[y * bw + x] = org[y * os + x] - cur[y * cs + x];
  for (int y = 0; y < bh; y++) wht(d + y * bw, bw, 1);
  for (int x = 0; x < bw; x++) wht(d + x, bh, bw);
  uint32_t s = 0;
  for (int i = 0; i < bw * bh; i++) s += (uint32_t)abs(d[i]);
  if (bw == 2 && bh == 2) return s;
  if (bw == 4 && bh == 4) return (s + 1) >> 1;
  if (bw == 8 && bh == 8) return (s + 2) >> 2;
  return (uint32_t)(int)(s / sqrt((double)(bw * bh)) * 2);
}

uint32_t or_satd(const int16_t *org, int os, const int16_t *cur, int cs, int w, int h) {
  int bw, bh;
  if (w > h && (h & 7) == 0 && (w & 15) == 0) { bw = 16; bh = 8; }
  else if (w < h && (w & 7) == 0 && (h & 15) == 0) { bw = 8; bh = 16; }
  else if (w > h && (h & 3) == 0 && (w & 7) == 0) { bw = 8; bh = 4; }
  else if (w < h && (w & 3) == 0 && (h & 7) == 0) { bw = 4; bh = 8; }
  else if (h % 8 == 0 && w % 8 == 0) { bw = 8; bh = 8; }
  else if (h % 4 == 0 && w % 4 == 0) { bw = 4; bh = 4; }
  else if (h % 2 == 0 && w % 2 == 0) { bw = 2; bh = 2; }
  else return 0xffffffffu;   /* THROW("Invalid size") */
  uint32_t s = 0;
  for (int y = 0; y < h; y += bh)
    for (int x = 0; x < w; x += bw) s += had_block(org + y * os + x, os, cur + y * cs + x, cs, bw, bh);
  return s;
}
