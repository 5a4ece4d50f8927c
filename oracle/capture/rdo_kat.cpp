// rdo_kat.cpp — TEST INFRASTRUCTURE: known-answer vectors for the encoder RDO inner loop (SURVEY.md
// §8(f) rank 3, BASELINE config 5), produced by the REFERENCE's own functions (VTM 7.3 CommonLib, built
// from /root/reference by oracle/ref.mk; nothing here is product code):
//   * distortion: the SAD (RdCost::xGetSAD, RdCost.cpp:503) and Hadamard SATD (RdCost::xGetHADs,
//     RdCost.cpp:2800, with its 2x2 / 4x4 / 8x8 / 16x8 / 8x16 / 8x4 / 4x8 kernels, :2150-2798) exactly as
//     the encoder calls them: RdCost::setDistParam (RdCost.h:181) picks the size's entry of the table
//     RdCost::init() fills (x86 SIMD variants where enabled) and DistParam::distFunc runs it;
//   * forward transform: the fastFwdTrans[trType][size] partial butterflies (TrQuant.cpp:69-74,
//     TrQuant_EMT.cpp) driven with the shifts and zero-out of TrQuant::xT (TrQuant.cpp:749-824).
// Usage: rdo_kat <seed> <dist.bin> <tr.bin>
//        rdo_kat --bench <width> <height> <seconds>   (CPU baseline of bench_rdo.py: the same block set —
//        every rectangle w x h, w, h in {8..128}, on its own size grid inside each 128x128 CTU, clipped to
//        the picture — SAD + SATD + DCT2 forward transform (w, h <= 64) per block, one thread)
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>
#include <string>
#include "RdCost.h"
#include "TrQuant_EMT.h"
#include "Rom.h"
#include "TrQuant.h"
extern FwdTrans *fastFwdTrans[NUM_TRANS_TYPE][g_numTransformMatrixSizes];   // TrQuant.cpp:69

static const int kSizes[6] = {4, 8, 16, 32, 64, 128};

#include <chrono>
static int bench(int W, int H, double seconds) {
  RdCost rc;
  std::mt19937 rng(5);
  std::vector<int16_t> org((size_t)W * H), cur((size_t)W * H);
  for (size_t i = 0; i < org.size(); i++) {
    org[i] = (int16_t)(rng() % 1024);
    cur[i] = (int16_t)std::min(1023, std::max(0, org[i] + (int)(rng() % 81) - 40));
  }
  struct B { int x, y, w, h; };
  std::vector<B> bl;
  for (int cy = 0; cy < H; cy += 128)
    for (int cx = 0; cx < W; cx += 128)
      for (int w = 8; w <= 128; w <<= 1)
        for (int h = 8; h <= 128; h <<= 1)
          for (int y = cy; y < cy + 128; y += h)
            for (int x = cx; x < cx + 128; x += w)
              if (x + w <= W && y + h <= H) bl.push_back({x, y, w, h});
  const int maxLog2 = 15, mshift = g_transformMatrixShift[TRANSFORM_FORWARD], bd = 10;
  std::vector<TCoeff> blk(128 * 128), tmp(128 * 128), coef(128 * 128);
  double samples = 0;
  uint64_t acc = 0;
  int passes = 0;
  const auto t0 = std::chrono::steady_clock::now();
  double el = 0;
  do {
    for (const B &b : bl) {
      const CPelBuf ob(&org[(size_t)b.y * W + b.x], W, b.w, b.h), cb(&cur[(size_t)b.y * W + b.x], W, b.w, b.h);
      DistParam dp;
      rc.setDistParam(dp, ob, cb, bd, COMPONENT_Y, false);
      acc += dp.distFunc(dp);
      rc.setDistParam(dp, ob, cb, bd, COMPONENT_Y, true);
      acc += dp.distFunc(dp);
      if (b.w <= 64 && b.h <= 64) {
        for (int y = 0; y < b.h; y++)
          for (int x = 0; x < b.w; x++) blk[y * b.w + x] = org[(size_t)(b.y + y) * W + b.x + x] - cur[(size_t)(b.y + y) * W + b.x + x];
        const int skipW = b.w > 32 ? b.w - 32 : 0, skipH = b.h > 32 ? b.h - 32 : 0;
        fastFwdTrans[DCT2][floorLog2(b.w) - 1](blk.data(), tmp.data(), (floorLog2(b.w) + bd + mshift) - maxLog2, b.h, 0, skipW);
        fastFwdTrans[DCT2][floorLog2(b.h) - 1](tmp.data(), coef.data(), floorLog2(b.h) + mshift, b.w, skipW, skipH);
        acc += coef[0];
      }
      samples += (double)b.w * b.h;
    }
    passes++;
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  } while (el < seconds);
  printf("{\"blocks\": %zu, \"passes\": %d, \"seconds\": %.3f, \"msamples_per_s\": %.3f, \"check\": %llu}\n", bl.size(), passes, el,
         samples / el / 1e6, (unsigned long long)acc);
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 5 && std::string(argv[1]) == "--bench") return bench(atoi(argv[2]), atoi(argv[3]), atof(argv[4]));
  if (argc < 4) { fprintf(stderr, "usage: rdo_kat seed dist.bin tr.bin\n"); return 2; }
  std::mt19937 rng((unsigned)atoi(argv[1]));
  RdCost rc;   // RdCost::init() fills m_afpDistortFunc (with the x86 SIMD variants when enabled)
  const int bd = 10;
  // ---------------- distortion
  FILE *fd = fopen(argv[2], "wb");
  std::vector<std::pair<int, int>> dims;
  for (int a = 0; a < 6; a++)
    for (int b = 0; b < 6; b++)
      if (kSizes[a] * kSizes[b] <= 64 * 64) dims.push_back({kSizes[a], kSizes[b]});
  dims.push_back({128, 128}); dims.push_back({128, 64}); dims.push_back({64, 128});
  const int reps = 3;
  int32_t n = (int32_t)dims.size() * reps;
  fwrite(&n, 4, 1, fd);
  for (int r = 0; r < reps; r++)
    for (auto wh : dims) {
      const int w = wh.first, h = wh.second;
      std::vector<int16_t> org(w * h), cur(w * h);
      const int amp = r == 0 ? 8 : (r == 1 ? 64 : 1023);
      for (int i = 0; i < w * h; i++) {
        org[i] = (int16_t)(rng() % 1024);
        int c = org[i] + (int)(rng() % (2 * amp + 1)) - amp;
        cur[i] = (int16_t)std::min(1023, std::max(0, c));
      }
      const CPelBuf ob(org.data(), w, w, h), cb(cur.data(), w, w, h);
      DistParam dp;
      rc.setDistParam(dp, ob, cb, bd, COMPONENT_Y, false);
      const uint32_t sadT = (uint32_t)dp.distFunc(dp);
      rc.setDistParam(dp, ob, cb, bd, COMPONENT_Y, true);
      const uint32_t hadT = (uint32_t)dp.distFunc(dp);
      int32_t hdr[2] = {w, h};
      fwrite(hdr, 4, 2, fd);
      fwrite(org.data(), 2, w * h, fd);
      fwrite(cur.data(), 2, w * h, fd);
      uint32_t out[2] = {sadT, hadT};
      fwrite(out, 4, 2, fd);
    }
  fclose(fd);
  // ---------------- forward transform (TrQuant::xT with maxLog2TrDynamicRange 15, bitDepth 10)
  FILE *ft = fopen(argv[3], "wb");
  struct T { int w, h, th, tv, lfnst; };
  std::vector<T> ts;
  const int tsz[5] = {4, 8, 16, 32, 64};
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 5; b++) {
      ts.push_back({tsz[a], tsz[b], DCT2, DCT2, 0});
      if (tsz[a] <= 32 && tsz[b] <= 32) {
        ts.push_back({tsz[a], tsz[b], DST7, DST7, 0});
        ts.push_back({tsz[a], tsz[b], DCT8, DST7, 0});
        ts.push_back({tsz[a], tsz[b], DST7, DCT8, 0});
        ts.push_back({tsz[a], tsz[b], DCT8, DCT8, 0});
      }
      if (tsz[a] <= 32 && tsz[b] <= 32) ts.push_back({tsz[a], tsz[b], DCT2, DCT2, 1});
    }
  n = (int32_t)ts.size();
  fwrite(&n, 4, 1, ft);
  const int maxLog2 = 15, mshift = g_transformMatrixShift[TRANSFORM_FORWARD];
  for (const T &t : ts) {
    const int w = t.w, h = t.h;
    std::vector<int16_t> resi(w * h);
    const int amp = (rng() & 1) ? 1023 : 64;
    for (int i = 0; i < w * h; i++) resi[i] = (int16_t)((int)(rng() % (2 * amp + 1)) - amp);
    // TrQuant::xT (TrQuant.cpp:749-824)
    int skipW = (t.th != DCT2 && w == 32) ? 16 : w > JVET_C0024_ZERO_OUT_TH ? w - JVET_C0024_ZERO_OUT_TH : 0;
    int skipH = (t.tv != DCT2 && h == 32) ? 16 : h > JVET_C0024_ZERO_OUT_TH ? h - JVET_C0024_ZERO_OUT_TH : 0;
    if (t.lfnst) {
      if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
      else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
    }
    std::vector<TCoeff> block(w * h), tmp(w * h), coef(w * h, 0);
    for (int i = 0; i < w * h; i++) block[i] = resi[i];
    const int s1 = (floorLog2(w) + bd + mshift) - maxLog2 + COM16_C806_TRANS_PREC;
    const int s2 = floorLog2(h) + mshift + COM16_C806_TRANS_PREC;
    fastFwdTrans[t.th][floorLog2(w) - 1](block.data(), tmp.data(), s1, h, 0, skipW);
    fastFwdTrans[t.tv][floorLog2(h) - 1](tmp.data(), coef.data(), s2, w, skipW, skipH);
    // our transform-type ids: 0 DCT2, 1 DST7, 2 DCT8
    auto id = [](int tr) { return tr == DCT2 ? 0 : (tr == DST7 ? 1 : 2); };
    int32_t hdr[5] = {w, h, id(t.th), id(t.tv), t.lfnst};
    fwrite(hdr, 4, 5, ft);
    fwrite(resi.data(), 2, w * h, ft);
    std::vector<int32_t> c32(coef.begin(), coef.end());
    fwrite(c32.data(), 4, w * h, ft);
  }
  fclose(ft);
  printf("rdo_kat: %zu distortion blocks, %zu transform blocks\n", dims.size() * reps, ts.size());
  return 0;
}
