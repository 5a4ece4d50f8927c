// mc_kat.cpp — TEST INFRASTRUCTURE: known-answer vectors for motion compensation (SURVEY.md §8(c),
// VERDICT r02 item 2e), produced by the REFERENCE's own interpolation (VTM 7.3 CommonLib, built from
// /root/reference by oracle/ref.mk; nothing here is product code).
//
// Two random 10-bit reference pictures and a picture tiled with prediction blocks of every size from
// 4x4 to 32x32, each with random motion: every luma (1/16) and chroma (1/32) fraction, whole-sample
// offsets reaching up to 56 samples past the picture's edges, uni-prediction from either list and
// bi-prediction, IMV_HPEL blocks (alternative half-sample filter). The prediction of each block is
// computed the way InterPrediction::xPredInterBlk (InterPrediction.cpp:698-804) drives the reference's
// filters: InterpolationFilter::filterHor / filterVer (InterpolationFilter.cpp:743,828; copy, 8-tap,
// the 6-tap 4x4 set, alt half-pel, 4-tap chroma; isFirst / isLast) on a reference picture whose borders
// are extended by edge replication (Picture::extendPicBorder, Picture.cpp:737), the H pass over
// height + N - 1 rows into the 14-bit intermediate, then V; bi-prediction averages the two 14-bit
// predictions with AreaBuf<Pel>::addAvg (Buffer.cpp). Vectors: tests/golden/mc_kat/*.bin (format below).
//
// Usage: mc_kat <seed> <out.bin>
// Format (little endian): int32 magic 'MCKT', W, H, bit depth, nblocks; int16 planes of reference 0
// (Y W*H, Cb, Cr W/2*H/2) and reference 1; nblocks * int32 {x, y, w, h, interdir, mv0x, mv0y, mv1x,
// mv1y, alt_hpel}; int16 expected prediction planes Y, Cb, Cr.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>
#include "InterpolationFilter.h"
#include "Buffer.h"

namespace {

constexpr int W = 128, H = 128, BD = 10, MARGIN = 96;

struct Plane {   // a component plane with its border extended by MARGIN samples (edge replication)
  int w, h, m, stride;
  std::vector<Pel> buf;
  Plane(int w_, int h_, int m_) : w(w_), h(h_), m(m_), stride(w_ + 2 * m_), buf((size_t)(w_ + 2 * m_) * (h_ + 2 * m_)) {}
  Pel *at(int x, int y) { return buf.data() + (size_t)(y + m) * stride + (x + m); }
  void extend() {
    for (int y = -m; y < h + m; y++)
      for (int x = -m; x < w + m; x++) {
        const int cx = std::min(std::max(x, 0), w - 1), cy = std::min(std::max(y, 0), h - 1);
        *at(x, y) = *at(cx, cy);
      }
  }
};

struct Block { int x, y, w, h, dir, mv[2][2], alt; };

void split(std::mt19937 &rng, int x, int y, int w, int h, std::vector<Block> &out) {
  // keep the block, or split it in halves (the partition of a CU tree, down to 4x4)
  const bool canH = h > 4, canV = w > 4;
  const int r = rng() % 8;
  if ((w > 32 || h > 32 || r < 5) && (canH || canV)) {
    const bool hor = canH && (!canV || (rng() & 1));
    if (hor) { split(rng, x, y, w, h / 2, out); split(rng, x, y + h / 2, w, h / 2, out); }
    else { split(rng, x, y, w / 2, h, out); split(rng, x + w / 2, y, w / 2, h, out); }
    return;
  }
  Block b{x, y, w, h, 0, {{0, 0}, {0, 0}}, 0};
  const bool biOk = w + h > 12;   // 4x4, 8x4, 4x8: uni-prediction only (PU::isBipredRestriction)
  b.dir = biOk ? 1 + (int)(rng() % 3) : 1 + (int)(rng() % 2);
  for (int l = 0; l < 2; l++)
    for (int c = 0; c < 2; c++) {
      int full;
      const int k = rng() % 10;
      if (k < 6) full = (int)(rng() % 17) - 8;                   // near the block
      else if (k < 9) full = (int)(rng() % 81) - 40;             // anywhere around
      else full = (c ? (rng() & 1 ? -(y + h + 56) : H - y + 56) : (rng() & 1 ? -(x + w + 56) : W - x + 56));   // far outside
      b.mv[l][c] = full * 16 + (int)(rng() % 16);
    }
  b.alt = (rng() % 6) == 0;
  out.push_back(b);
}

// one component of one list: InterPrediction::xPredInterBlk without DMVR / BDOF / RPR / wrap-around
void pred_comp(InterpolationFilter &F, Plane &ref, ComponentID comp, const Block &b, int l, bool bi, Pel *dst, int dstStride,
               const ClpRng &clp) {
  const int cs = comp == COMPONENT_Y ? 0 : 1;
  const int shift = 4 + cs, mask = (1 << shift) - 1;
  const int mvx = b.mv[l][0], mvy = b.mv[l][1];
  const int xFrac = mvx & mask, yFrac = mvy & mask;
  const int w = b.w >> cs, h = b.h >> cs;
  const int ox = (b.x >> cs) + (mvx >> shift), oy = (b.y >> cs) + (mvy >> shift);
  Pel *src = ref.at(ox, oy);
  const bool rnd = !bi;
  if (yFrac == 0) {
    F.filterHor(comp, src, ref.stride, dst, dstStride, w, h, xFrac, rnd, CHROMA_420, clp, 0, false, b.alt);
  } else if (xFrac == 0) {
    F.filterVer(comp, src, ref.stride, dst, dstStride, w, h, yFrac, true, rnd, CHROMA_420, clp, 0, false, b.alt);
  } else {
    const int N = comp == COMPONENT_Y ? NTAPS_LUMA : NTAPS_CHROMA;
    std::vector<Pel> tmp((size_t)w * (h + N - 1));
    F.filterHor(comp, src - ((N >> 1) - 1) * ref.stride, ref.stride, tmp.data(), w, w, h + N - 1, xFrac, false, CHROMA_420, clp, 0, false, b.alt);
    F.filterVer(comp, tmp.data() + ((N >> 1) - 1) * w, w, dst, dstStride, w, h, yFrac, false, rnd, CHROMA_420, clp, 0, false, b.alt);
  }
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 3) { fprintf(stderr, "usage: mc_kat <seed> <out.bin>\n"); return 2; }
  std::mt19937 rng((unsigned)atoi(argv[1]));
  InterpolationFilter F;
  F.initInterpolationFilter(true);   // as InterPrediction::init (InterPrediction.cpp:229)
  g_pelBufOP.initPelBufOpsX86();
  const ClpRng clp{0, (1 << BD) - 1, BD, 0};
  // reference pictures: smooth gradients plus noise, with saturated patches (clipping of the filters)
  std::vector<Plane> refs;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++) {
      const int cw = c ? W / 2 : W, ch = c ? H / 2 : H;
      refs.emplace_back(cw, ch, MARGIN);
      Plane &p = refs.back();
      const int fx = 1 + rng() % 7, fy = 1 + rng() % 7;
      for (int y = 0; y < ch; y++)
        for (int x = 0; x < cw; x++) {
          int v = 512 + (int)(300 * std::sin(0.05 * fx * x + 0.07 * fy * y + r)) + (int)(rng() % 161) - 80;
          if (((x >> 3) + (y >> 3) + r) % 11 == 0) v = (rng() & 1) ? 1023 : 0;
          *p.at(x, y) = (Pel)std::min(std::max(v, 0), (1 << BD) - 1);
        }
      p.extend();
    }
  std::vector<Block> blocks;
  for (int y = 0; y < H; y += 32)
    for (int x = 0; x < W; x += 32) split(rng, x, y, 32, 32, blocks);
  std::vector<Pel> out[3] = {std::vector<Pel>((size_t)W * H), std::vector<Pel>((size_t)W * H / 4), std::vector<Pel>((size_t)W * H / 4)};
  for (const Block &b : blocks)
    for (int c = 0; c < 3; c++) {
      const ComponentID comp = (ComponentID)c;
      const int cs = c ? 1 : 0, w = b.w >> cs, h = b.h >> cs, pw = W >> cs;
      Pel *dst = out[c].data() + (size_t)(b.y >> cs) * pw + (b.x >> cs);
      const bool bi = b.dir == 3;
      if (!bi) {
        const int l = b.dir == 1 ? 0 : 1;
        pred_comp(F, refs[3 * l + c], comp, b, l, false, dst, pw, clp);
      } else {
        std::vector<Pel> p0((size_t)w * h), p1((size_t)w * h);
        pred_comp(F, refs[c], comp, b, 0, true, p0.data(), w, clp);
        pred_comp(F, refs[3 + c], comp, b, 1, true, p1.data(), w, clp);
        PelBuf d(dst, pw, w, h);
        d.addAvg(CPelBuf(p0.data(), w, w, h), CPelBuf(p1.data(), w, w, h), clp);
      }
    }
  FILE *f = fopen(argv[2], "wb");
  if (!f) { perror(argv[2]); return 1; }
  const int32_t hdr[5] = {0x544b434d, W, H, BD, (int32_t)blocks.size()};
  fwrite(hdr, 4, 5, f);
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++) {
      Plane &p = refs[3 * r + c];
      for (int y = 0; y < p.h; y++) fwrite(p.at(0, y), sizeof(Pel), p.w, f);
    }
  for (const Block &b : blocks) {
    const int32_t row[10] = {b.x, b.y, b.w, b.h, b.dir, b.mv[0][0], b.mv[0][1], b.mv[1][0], b.mv[1][1], b.alt};
    fwrite(row, 4, 10, f);
  }
  for (int c = 0; c < 3; c++) fwrite(out[c].data(), sizeof(Pel), out[c].size(), f);
  fclose(f);
  int nbi = 0, nalt = 0;
  for (const Block &b : blocks) { nbi += b.dir == 3; nalt += b.alt; }
  printf("%zu blocks (%d bi, %d alt-hpel) -> %s\n", blocks.size(), nbi, nalt, argv[2]);
  return 0;
}
