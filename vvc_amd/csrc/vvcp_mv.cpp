// vvcp_mv.cpp — motion derivation (see vvcp_mv.h). Every function cites the reference function it
// restates; MVs are in 1/16 luma sample (MV_FRACTIONAL_BITS_INTERNAL = 4).
#include "vvcp_mv.h"

#include <algorithm>
#include <cstdint>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "vvcp_stream.h"

namespace vvcp {

// Mi's flag bitfields must be laid out as MotionRec::flags (vvcp_mv.h); a compiler that orders them otherwise
// would corrupt every consumer of the motion rows, so the library refuses to load (constexpr bit_cast of
// bitfields is not available to a static_assert).
namespace {
struct MiLayoutCheck {
  MiLayoutCheck() {
    Mi m;
    m.isInter = 1; m.altHpel = 0; m.bcw = 2;
    uint8_t b[sizeof(Mi)];
    std::memcpy(b, &m, sizeof m);
    Mi n;
    n.isInter = 0; n.altHpel = 1; n.bcw = 0;
    uint8_t c[sizeof(Mi)];
    std::memcpy(c, &n, sizeof n);
    if (b[offsetof(MotionRec, flags)] != 0x09 || c[offsetof(MotionRec, flags)] != 0x02) {
      std::fprintf(stderr, "libvvcr: Mi flag bitfields are not laid out as MotionRec::flags\n");
      std::abort();
    }
  }
} const g_mi_layout_check;
}  // namespace


bool Mi::same(const Mi &o) const {
  if (isInter != o.isInter) return false;
  if (isInter) {
    if (slice != o.slice || interDir != o.interDir) return false;
    if (interDir != 2 && (ref[0] != o.ref[0] || mv[0][0] != o.mv[0][0] || mv[0][1] != o.mv[0][1])) return false;
    if (interDir != 1 && (ref[1] != o.ref[1] || mv[1][0] != o.mv[1][0] || mv[1][1] != o.mv[1][1])) return false;
  }
  return true;
}

namespace {

enum { MODE_INTER = 0, MODE_INTRA = 1 };
enum { MRG_DEFAULT = 0, MRG_SUBPU_ATMVP = 1 };
constexpr int BCW_DEFAULT = 2, IMV_HPEL = 3, AFF_4P = 0, AFF_6P = 1, AFF_NUM = 2, MAX_CU_DEPTH = 7;

struct Mv {
  int32_t h = 0, v = 0;
  Mv() = default;
  Mv(int32_t a, int32_t b) : h(a), v(b) {}
  bool operator==(const Mv &o) const { return h == o.h && v == o.v; }
  bool operator!=(const Mv &o) const { return !(*this == o); }
  Mv operator+(const Mv &o) const { return Mv(h + o.h, v + o.v); }
  Mv operator-(const Mv &o) const { return Mv(h - o.h, v - o.v); }
};
inline int clipStore(int x) { return clip3(-(1 << 17), (1 << 17) - 1, x); }
inline Mv clipStore(Mv m) { return Mv(clipStore(m.h), clipStore(m.v)); }
inline int wrapStore(int x) {   // Mv::mvCliptoStorageBitDepth (periodic)
  const int P = 1 << 18, H = 1 << 17;
  x = (x + P) & (P - 1);
  return x >= H ? x - P : x;
}
inline Mv wrapStore(Mv m) { return Mv(wrapStore(m.h), wrapStore(m.v)); }
// Mv::changePrecision (Mv.h)
inline int changePrec(int x, int shift) {
  if (shift >= 0) return x * (1 << shift);
  const int r = -shift, off = 1 << (r - 1);
  return x >= 0 ? (x + off - 1) >> r : (x + off) >> r;
}
inline Mv changePrec(Mv m, int shift) { return Mv(changePrec(m.h, shift), changePrec(m.v, shift)); }
inline Mv roundPrec(Mv m, int shift) { return changePrec(changePrec(m, -shift), shift); }   // roundToPrecision(internal -> internal-shift)
// m_amvrPrecision {quarter, int, 4pel, half} / m_amvrPrecAffine {quarter, sixteenth, int}: shift from internal (1/16)
const int kAmvrShift[4] = {2, 4, 6, 3};
const int kAffShift[3] = {2, 0, 4};
inline void roundAffineMv(int &x, int &y, int s) {
  const int off = 1 << (s - 1);
  x = (x + off - (x >= 0)) >> s;
  y = (y + off - (y >= 0)) >> s;
}
// roundMvComp (UnitTools.cpp:1309-1342): 6-bit mantissa / 4-bit exponent compression of stored MVs
int roundMvComp(int val) {
  const int sign = val >> 31;
  const int scale = floorLog2((uint32_t)((val ^ sign) | 31)) - 5;
  int exponent, mantissa;
  if (scale >= 0) {
    const int round = (1 << scale) >> 1;
    const int n = (val + round) >> scale;
    exponent = scale + ((n ^ sign) >> 5);
    mantissa = (n & 31) | (sign * (1 << 5));
  } else {
    exponent = 0;
    mantissa = val;
  }
  const int f = exponent | (mantissa * (1 << 4));
  const int e = f & 15, m = f >> 4;
  return e == 0 ? m : (m ^ 32) * (1 << (e - 1));
}
int distScale(int curPoc, int curRefPoc, int colPoc, int colRefPoc) {   // xGetDistScaleFactor (:1290)
  const int d = colPoc - colRefPoc, b = curPoc - curRefPoc;
  if (d == b) return 4096;
  const int tb = clip3(-128, 127, b), td = clip3(-128, 127, d);
  const int x = (0x4000 + std::abs(td / 2)) / td;
  return clip3(-4096, 4095, (tb * x + 32) >> 6);
}
// an entry of the collocated view (MotionPicture::mf) with its MVs compressed as getColocatedMVP reads
// them (roundMvComp, UnitTools.cpp:1472-1473): once per stored 8x8 unit instead of per read
inline Mi colMi(Mi m) {
  for (int l = 0; l < 2; l++)
    for (int k = 0; k < 2; k++) m.mv[l][k] = roundMvComp(m.mv[l][k]);
  return m;
}
inline Mv scaleMv(Mv m, int s) {   // Mv::scaleMv
  auto f = [&](int c) { const long long p = (long long)s * c; return clip3(-(1 << 17), (1 << 17) - 1, (int)((p + 128 - (p >= 0)) >> 8)); };
  return Mv(f(m.h), f(m.v));
}

struct MvField { Mv mv; int ref = -1; };
struct MergeCtx {
  MvField mvf[2 * 6];
  int interDir[6] = {0}, bcw[6] = {0}, mrgType[6] = {0};
  bool altHpel[6] = {false};
  int numValid = 0;
  MvField mmvdBase[2][2];
  bool mmvdAltHpel[2] = {false, false};
};
struct AffMergeCtx {
  MvField mvf[2 * 5][3];
  int interDir[5] = {0}, affType[5] = {0}, mrgType[5] = {0}, bcw[5] = {0};
  int numValid = 0;
};

struct Deriver {
  PictureUnit &P;
  PictureSyntax &S;
  const SPS &sps;
  const PicHeader &ph;
  MotionField &mf;
  MotionField *col8f = nullptr;   // the collocated view being built (MotionPicture::mf: 8x8 subsample)
  int w8 = 0;
  std::vector<vvcr_geo> &geoRows;
  const std::vector<const MotionPicture *> &dpb;
  const SliceHeader *sh = nullptr;
  int sliceIdx = 0;
  const MotionPicture *col = nullptr;
  std::vector<Mi> lut;            // HMVP table (CodingStructure::motionLut.lut), oldest first
  std::vector<Mi> subPu;          // SbTMVP sub-block motion of the current PU (mrgCtx.subPuMvpMiBuf)
  int subW = 0;
  // per-CU derived state
  std::vector<int> cuImv, cuBcw, cuAffType;
  std::vector<Mv> puMv[2];
  std::vector<int> puRef[2], puInterDir, puMrgType;
  std::vector<Mv> puAff[2][3];

  Deriver(PictureUnit &p, MotionField &f, std::vector<vvcr_geo> &g, const std::vector<const MotionPicture *> &d)
      : P(p), S(p.syn), sps(p.sps), ph(p.ph), mf(f), geoRows(g), dpb(d) {}

  Mi &at(int x, int y) { return mf[(size_t)(y >> 2) * S.w4 + (x >> 2)]; }
  // the units of CU ci at 8-aligned positions into the collocated view, once its span is final (each
  // unit is written by its own CU only; DMVR refinements follow in refine_motion)
  void col8(const vvcr_cu &c) {
    for (int y = (c.y + 7) & ~7; y < c.y + c.h; y += 8)
      for (int x = (c.x + 7) & ~7; x < c.x + c.w; x += 8) (*col8f)[(size_t)(y >> 3) * w8 + (x >> 3)] = colMi(at(x, y));
  }
  bool isBipredRestriction(const vvcr_cu &c) const { return (c.w == 4 && c.h == 4) || c.w + c.h == 12; }
  bool isDiffMER(int x1, int y1, int x2, int y2) const {   // PU::isDiffMER (:1506) on the PU top-left corners
    const int l = sps.log2ParMrgLevel;
    return (x1 >> l) != (x2 >> l) || (y1 >> l) != (y2 >> l);
  }
  // CodingStructure::getPURestricted (CodingStructure.cpp:1550): CU index or -1
  int puRestricted(int ci, int x, int y) const {
    const int n = S.cuAt(0, x, y);
    if (n < 0 || n > ci) return -1;
    if (P.pps.entropySync && (x >> sps.ctuLog2) >= (S.cu[ci].x >> sps.ctuLog2) + 1) return -1;
    if (S.cux[n].slice != S.cux[ci].slice || S.cux[n].tile != S.cux[ci].tile) return -1;
    return n;
  }
  bool isInterCu(int n) const { return S.cu[n].predmode == MODE_INTER; }
  int refPoc(int l, int r) const { return sh->refPoc[l][r]; }

  // ----------------------------------------------------------------------------------------------
  // Temporal candidates: PU::getColocatedMVP (UnitTools.cpp:1387)
  // ----------------------------------------------------------------------------------------------
  bool colocatedMVP(int l, int px, int py, Mv &out, int refIdx, bool sbFlag) const {
    if (!col || col->intra) return false;
    const int x = px & ~7, y = py & ~7;
    const Mi &mi = col->at8(x, y);
    if (!mi.isInter) return false;
    int colList = sh->checkLDC ? l : (sh->colFromL0 ? 1 : 0);
    int colRef = mi.ref[colList];
    if (sbFlag && !sh->checkLDC) {
      colList = l;
      colRef = mi.ref[colList];
      if (colRef < 0) return false;
    } else if (colRef < 0) {
      colList = 1 - colList;
      colRef = mi.ref[colList];
      if (colRef < 0) return false;
    }
    VVCP_CHECK(mi.slice >= col->slices.size(), "collocated slice missing");
    const SliceRefs &cs = col->slices[mi.slice];
    const bool curLT = sh->refLT[l][refIdx], colLT = cs.refLT[colList][colRef];
    if (curLT != colLT) return false;
    const Mv m(mi.mv[colList][0], mi.mv[colList][1]);   // (stored compressed: colMi)
    if (curLT) { out = clipStore(m); return true; }
    const int s = distScaleCol(sh->poc - refPoc(l, refIdx), col->poc - cs.refPoc[colList][colRef]);
    out = s == 4096 ? clipStore(m) : scaleMv(m, s);
    return true;
  }
  // distScale of the temporal candidates, memoised on the two POC distances (an SbTMVP CU asks per
  // 8x8 sub-block and list, with a handful of distinct pairs per picture)
  mutable int dsB[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN}, dsD[4] = {}, dsV[4] = {}, dsNext = 0;
  int distScaleCol(int b, int d) const {
    for (int k = 0; k < 4; k++)
      if (dsB[k] == b && dsD[k] == d) return dsV[k];
    const int v = distScale(b, 0, d, 0);
    const int k = dsNext++ & 3;
    dsB[k] = b; dsD[k] = d; dsV[k] = v;
    return v;
  }
  // C0 (bottom-right) / C1 (centre) positions shared by the temporal candidates
  bool posC0(const vvcr_cu &c, int &x, int &y) const {
    const int rx = c.x + c.w - 1 - 3, ry = c.y + c.h - 1 - 3;
    if (rx + 4 < S.W && ry + 4 < S.H) {
      const int inCtu = ry & (S.ctuSize - 1);
      if (inCtu + 4 < S.ctuSize) { x = rx + 4; y = ry + 4; return true; }
    }
    return false;
  }

  // ----------------------------------------------------------------------------------------------
  // PU::getInterMergeCandidates (UnitTools.cpp:845) + addMergeHMVPCand (:680)
  // ----------------------------------------------------------------------------------------------
  void setCand(MergeCtx &m, int cnt, const Mi &mi, int bcw) {
    m.interDir[cnt] = mi.interDir;
    m.altHpel[cnt] = mi.altHpel;
    m.bcw[cnt] = mi.interDir == 3 ? bcw : BCW_DEFAULT;
    m.mvf[cnt << 1].mv = Mv(mi.mv[0][0], mi.mv[0][1]);
    m.mvf[cnt << 1].ref = mi.ref[0];
    if (sh->isInterB()) { m.mvf[(cnt << 1) + 1].mv = Mv(mi.mv[1][0], mi.mv[1][1]); m.mvf[(cnt << 1) + 1].ref = mi.ref[1]; }
  }
  void mergeCandidates(int ci, MergeCtx &m, int mrgCandIdx) {
    const vvcr_cu &c = S.cu[ci];
    const int maxN = ph.maxNumMergeCand;
    for (int i = 0; i < maxN; i++) {
      m.bcw[i] = BCW_DEFAULT; m.interDir[i] = 0; m.mrgType[i] = MRG_DEFAULT;
      m.mvf[i << 1].ref = -1; m.mvf[(i << 1) + 1].ref = -1;
      m.altHpel[i] = false;
    }
    m.numValid = maxN;
    int cnt = 0;
    const int xR = c.x + c.w - 1, yB = c.y + c.h - 1;
    Mi miAbove, miLeft;
    // B1
    const int pA = puRestricted(ci, xR, c.y - 1);
    const bool avB1 = pA >= 0 && isDiffMER(c.x, c.y, S.cu[pA].x, S.cu[pA].y) && pA != ci && isInterCu(pA);
    if (avB1) {
      miAbove = at(xR, c.y - 1);
      setCand(m, cnt, miAbove, cuBcw[pA]);
      if (mrgCandIdx == cnt) return;
      cnt++;
    }
    if (cnt == maxN) return;
    // A1
    const int pL = puRestricted(ci, c.x - 1, yB);
    const bool avA1 = pL >= 0 && isDiffMER(c.x, c.y, S.cu[pL].x, S.cu[pL].y) && pL != ci && isInterCu(pL);
    if (avA1) {
      miLeft = at(c.x - 1, yB);
      if (!avB1 || !miAbove.same(miLeft)) {
        setCand(m, cnt, miLeft, cuBcw[pL]);
        if (mrgCandIdx == cnt) return;
        cnt++;
      }
    }
    if (cnt == maxN) return;
    // B0
    const int pAR = puRestricted(ci, xR + 1, c.y - 1);
    if (pAR >= 0 && isDiffMER(c.x, c.y, S.cu[pAR].x, S.cu[pAR].y) && isInterCu(pAR)) {
      const Mi miAR = at(xR + 1, c.y - 1);
      if (!avB1 || !miAbove.same(miAR)) {
        setCand(m, cnt, miAR, cuBcw[pAR]);
        if (mrgCandIdx == cnt) return;
        cnt++;
      }
    }
    if (cnt == maxN) return;
    // A0
    const int pBL = puRestricted(ci, c.x - 1, yB + 1);
    if (pBL >= 0 && isDiffMER(c.x, c.y, S.cu[pBL].x, S.cu[pBL].y) && isInterCu(pBL)) {
      const Mi miBL = at(c.x - 1, yB + 1);
      if (!avA1 || !miBL.same(miLeft)) {
        setCand(m, cnt, miBL, cuBcw[pBL]);
        if (mrgCandIdx == cnt) return;
        cnt++;
      }
    }
    if (cnt == maxN) return;
    // B2
    if (cnt < 4) {
      const int pAL = puRestricted(ci, c.x - 1, c.y - 1);
      if (pAL >= 0 && isDiffMER(c.x, c.y, S.cu[pAL].x, S.cu[pAL].y) && isInterCu(pAL)) {
        const Mi miAL = at(c.x - 1, c.y - 1);
        if ((!avA1 || !miLeft.same(miAL)) && (!avB1 || !miAbove.same(miAL))) {
          setCand(m, cnt, miAL, cuBcw[pAL]);
          if (mrgCandIdx == cnt) return;
          cnt++;
        }
      }
    }
    if (cnt == maxN) return;
    // temporal
    if (ph.tmvp && c.w + c.h > 12) {
      int x0 = 0, y0 = 0;
      const bool c0 = posC0(c, x0, y0);
      const int x1 = c.x + (c.w >> 1), y1 = c.y + (c.h >> 1);
      Mv cm;
      int dir = 0;
      const int a = cnt;
      if ((c0 && colocatedMVP(0, x0, y0, cm, 0, false)) || colocatedMVP(0, x1, y1, cm, 0, false)) {
        dir |= 1;
        m.mvf[2 * a].mv = cm;
        m.mvf[2 * a].ref = 0;
      }
      if (sh->isInterB()) {
        if ((c0 && colocatedMVP(1, x0, y0, cm, 0, false)) || colocatedMVP(1, x1, y1, cm, 0, false)) {
          dir |= 2;
          m.mvf[2 * a + 1].mv = cm;
          m.mvf[2 * a + 1].ref = 0;
        }
      }
      if (dir) {
        m.interDir[a] = dir;
        m.bcw[a] = BCW_DEFAULT;
        m.altHpel[a] = false;
        if (mrgCandIdx == cnt) return;
        cnt++;
      }
    }
    if (cnt == maxN) return;
    // history
    const int maxMin1 = maxN - 1;
    if (cnt != maxMin1) {
      const int n = (int)lut.size();
      for (int k = 1; k <= n; k++) {
        const Mi &nb = lut[n - k];
        if (k > 2 || ((!avA1 || !miLeft.same(nb)) && (!avB1 || !miAbove.same(nb)))) {
          m.interDir[cnt] = nb.interDir;
          m.altHpel[cnt] = nb.altHpel;
          m.bcw[cnt] = nb.interDir == 3 ? nb.bcw : BCW_DEFAULT;
          m.mvf[cnt << 1].mv = Mv(nb.mv[0][0], nb.mv[0][1]);
          m.mvf[cnt << 1].ref = nb.ref[0];
          if (sh->isInterB()) { m.mvf[(cnt << 1) + 1].mv = Mv(nb.mv[1][0], nb.mv[1][1]); m.mvf[(cnt << 1) + 1].ref = nb.ref[1]; }
          if (mrgCandIdx == cnt) return;
          cnt++;
          if (cnt == maxMin1) break;
        }
      }
      if (cnt < maxMin1) m.altHpel[cnt] = false;
    }
    // pairwise average
    if (cnt > 1 && cnt < maxN) {
      m.mvf[cnt * 2] = MvField();
      m.mvf[cnt * 2 + 1] = MvField();
      int dir = 0;
      m.altHpel[cnt] = m.altHpel[0] == m.altHpel[1] ? m.altHpel[0] : false;
      for (int l = 0; l < (sh->isInterB() ? 2 : 1); l++) {
        const int ri = m.mvf[l].ref, rj = m.mvf[2 + l].ref;
        if (ri == -1 && rj == -1) continue;
        dir += 1 << l;
        if (ri != -1 && rj != -1) {
          int h = m.mvf[l].mv.h + m.mvf[2 + l].mv.h, v = m.mvf[l].mv.v + m.mvf[2 + l].mv.v;
          roundAffineMv(h, v, 1);
          m.mvf[cnt * 2 + l].mv = Mv(h, v);
          m.mvf[cnt * 2 + l].ref = ri;
        } else if (ri != -1) {
          m.mvf[cnt * 2 + l] = m.mvf[l];
        } else {
          m.mvf[cnt * 2 + l] = m.mvf[2 + l];
        }
      }
      m.interDir[cnt] = dir;
      if (dir > 0) cnt++;
    }
    if (cnt == maxN) return;
    // zero candidates
    int a = cnt;
    const int numRef = sh->isInterB() ? std::min(sh->numRef[0], sh->numRef[1]) : sh->numRef[0];
    int r = 0, refcnt = 0;
    while (a < maxN) {
      m.interDir[a] = 1;
      m.bcw[a] = BCW_DEFAULT;
      m.mvf[a << 1].mv = Mv();
      m.mvf[a << 1].ref = r;
      m.altHpel[a] = false;
      if (sh->isInterB()) {
        m.interDir[a] = 3;
        m.mvf[(a << 1) + 1].mv = Mv();
        m.mvf[(a << 1) + 1].ref = r;
      }
      a++;
      if (refcnt == numRef - 1) r = 0;
      else { ++r; ++refcnt; }
    }
    m.numValid = a;
  }

  // ----------------------------------------------------------------------------------------------
  // AMVP: PU::fillMvpCand (:1710), addMVPCandUnscaled (:2136), addAMVPHMVPCand (:2191)
  // ----------------------------------------------------------------------------------------------
  bool addMvpUnscaled(int ci, int l, int refIdx, int nx, int ny, Mv *cand, int &num) {
    const int n = puRestricted(ci, nx, ny);
    if (n < 0 || !isInterCu(n)) return false;
    const Mi &mi = at(nx, ny);
    const int cur = refPoc(l, refIdx);
    for (int src = 0; src < 2; src++) {
      const int ll = src == 0 ? l : 1 - l;
      const int r = mi.ref[ll];
      if (r >= 0 && cur == refPoc(ll, r)) {
        cand[num++] = Mv(mi.mv[ll][0], mi.mv[ll][1]);
        return true;
      }
    }
    return false;
  }
  void fillMvpCand(int ci, int l, int refIdx, int imv, Mv out[2]) {
    const vvcr_cu &c = S.cu[ci];
    Mv cand[8];
    int num = 0;
    if (refIdx < 0) return;
    const int xR = c.x + c.w - 1, yB = c.y + c.h - 1;
    if (!addMvpUnscaled(ci, l, refIdx, c.x - 1, yB + 1, cand, num)) addMvpUnscaled(ci, l, refIdx, c.x - 1, yB, cand, num);
    if (!addMvpUnscaled(ci, l, refIdx, xR + 1, c.y - 1, cand, num))
      if (!addMvpUnscaled(ci, l, refIdx, xR, c.y - 1, cand, num)) addMvpUnscaled(ci, l, refIdx, c.x - 1, c.y - 1, cand, num);
    const int sh_ = kAmvrShift[imv];
    for (int i = 0; i < num; i++) cand[i] = roundPrec(cand[i], sh_);
    if (num == 2 && cand[0] == cand[1]) num = 1;
    if (ph.tmvp && num < 2 && c.w + c.h > 12) {
      int x0, y0;
      const bool c0 = posC0(c, x0, y0);
      Mv cm;
      if ((c0 && colocatedMVP(l, x0, y0, cm, refIdx, false)) || colocatedMVP(l, c.x + (c.w >> 1), c.y + (c.h >> 1), cm, refIdx, false))
        cand[num++] = roundPrec(cm, sh_);
    }
    if (num < 2) {   // history, oldest entry first
      const int cur = refPoc(l, refIdx);
      const int allowed = std::min(4, (int)lut.size());
      for (int k = 1; k <= allowed && num < 2; k++) {
        const Mi &nb = lut[k - 1];
        for (int src = 0; src < 2; src++) {
          const int ll = src == 0 ? l : 1 - l;
          const int r = nb.ref[ll];
          if (r >= 0 && cur == refPoc(ll, r)) {
            cand[num++] = roundPrec(Mv(nb.mv[ll][0], nb.mv[ll][1]), sh_);
            if (num >= 2) break;
          }
        }
      }
    }
    if (num > 2) num = 2;
    while (num < 2) cand[num++] = Mv();
    out[0] = roundPrec(cand[0], sh_);
    out[1] = roundPrec(cand[1], sh_);
  }

  // ----------------------------------------------------------------------------------------------
  // Affine: xInheritedAffineMv (:1889), fillAffineMvpCand (:1967), getAffineMergeCand (:2461),
  // getAffineControlPointCand (:2243), setAllAffineMv (:2784)
  // ----------------------------------------------------------------------------------------------
  void inheritedAffineMv(int ci, int n, int l, int curType, Mv out[3]) {
    const vvcr_cu &c = S.cu[ci], &nb = S.cu[n];
    int pnx = nb.x, pny = nb.y;
    const int nw = nb.w, nh = nb.h;
    Mv lt = puAff[l][0][n], rt = puAff[l][1][n], lb = puAff[l][2][n];
    bool topCtu = false;
    if ((pny + nh) % S.ctuSize == 0 && (pny + nh) == c.y) {
      const Mi &a = at(nb.x, nb.y + nh - 1), &b = at(nb.x + nw - 1, nb.y + nh - 1);
      lt = Mv(a.mv[l][0], a.mv[l][1]);
      rt = Mv(b.mv[l][0], b.mv[l][1]);
      pny += nh;
      topCtu = true;
    }
    const int s = MAX_CU_DEPTH;
    const int dHx = (rt - lt).h * (1 << (s - floorLog2(nw))), dHy = (rt - lt).v * (1 << (s - floorLog2(nw)));
    int dVx, dVy;
    if (cuAffType[n] == AFF_6P && !topCtu) {
      dVx = (lb - lt).h * (1 << (s - floorLog2(nh)));
      dVy = (lb - lt).v * (1 << (s - floorLog2(nh)));
    } else {
      dVx = -dHy;
      dVy = dHx;
    }
    const int bx = lt.h * (1 << s), by = lt.v * (1 << s);
    auto pt = [&](int px, int py) {
      int h = bx + dHx * (px - pnx) + dVx * (py - pny);
      int v = by + dHy * (px - pnx) + dVy * (py - pny);
      roundAffineMv(h, v, s);
      return clipStore(Mv(h, v));
    };
    out[0] = pt(c.x, c.y);
    out[1] = pt(c.x + c.w, c.y);
    if (curType == AFF_6P) out[2] = pt(c.x, c.y + c.h);
  }
  bool addAffineMvpUnscaled(int ci, int l, int refIdx, int nx, int ny, int curType, int imv, Mv lt[], Mv rt[], Mv lb[], int &num) {
    const int n = puRestricted(ci, nx, ny);
    if (n < 0 || !isInterCu(n) || !S.cu[n].affine || puMrgType[n] != MRG_DEFAULT) return false;
    const Mi &mi = at(nx, ny);
    const int cur = refPoc(l, refIdx);
    for (int src = 0; src < 2; src++) {
      const int ll = src == 0 ? l : 1 - l;
      if ((puInterDir[n] & (ll + 1)) == 0 || refPoc(ll, mi.ref[ll]) != cur) continue;
      Mv o[3];
      inheritedAffineMv(ci, n, ll, curType, o);
      lt[num] = roundPrec(o[0], kAffShift[imv]);
      rt[num] = roundPrec(o[1], kAffShift[imv]);
      if (curType == AFF_6P) lb[num] = roundPrec(o[2], kAffShift[imv]);
      num++;
      return true;
    }
    return false;
  }
  void fillAffineMvpCand(int ci, int l, int refIdx, int imv, int type, Mv lt[2], Mv rt[2], Mv lb[2]) {
    const vvcr_cu &c = S.cu[ci];
    int num = 0;
    Mv LT[4], RT[4], LB[4];
    const int xR = c.x + c.w - 1, yB = c.y + c.h - 1;
    if (!addAffineMvpUnscaled(ci, l, refIdx, c.x - 1, yB + 1, type, imv, LT, RT, LB, num))
      addAffineMvpUnscaled(ci, l, refIdx, c.x - 1, yB, type, imv, LT, RT, LB, num);
    if (!addAffineMvpUnscaled(ci, l, refIdx, xR + 1, c.y - 1, type, imv, LT, RT, LB, num))
      if (!addAffineMvpUnscaled(ci, l, refIdx, xR, c.y - 1, type, imv, LT, RT, LB, num))
        addAffineMvpUnscaled(ci, l, refIdx, c.x - 1, c.y - 1, type, imv, LT, RT, LB, num);
    const int sft = kAffShift[imv];
    if (num < 2) {
      Mv a0[1], a1[1], a2[1];
      int n0 = 0, n1 = 0, n2 = 0;
      addMvpUnscaled(ci, l, refIdx, c.x - 1, c.y - 1, a0, n0);
      if (n0 < 1) addMvpUnscaled(ci, l, refIdx, c.x, c.y - 1, a0, n0);
      if (n0 < 1) addMvpUnscaled(ci, l, refIdx, c.x - 1, c.y, a0, n0);
      addMvpUnscaled(ci, l, refIdx, xR, c.y - 1, a1, n1);
      if (n1 < 1) addMvpUnscaled(ci, l, refIdx, xR + 1, c.y - 1, a1, n1);
      addMvpUnscaled(ci, l, refIdx, c.x - 1, yB, a2, n2);
      if (n2 < 1) addMvpUnscaled(ci, l, refIdx, c.x - 1, yB + 1, a2, n2);
      const int pattern = n0 | (n1 << 1) | (n2 << 2);
      Mv o[3] = {n0 ? roundPrec(a0[0], sft) : Mv(), n1 ? roundPrec(a1[0], sft) : Mv(), n2 ? roundPrec(a2[0], sft) : Mv()};
      if (pattern == 7 || (pattern == 3 && type == AFF_4P)) { LT[num] = o[0]; RT[num] = o[1]; LB[num] = o[2]; num++; }
      if (num < 2) {
        for (int i = 2; i >= 0 && num < 2; i--)
          if (pattern & (1 << i)) { LT[num] = RT[num] = LB[num] = o[i]; num++; }
        if (num < 2 && ph.tmvp) {
          int x0, y0;
          const bool c0 = posC0(c, x0, y0);
          Mv cm;
          if ((c0 && colocatedMVP(l, x0, y0, cm, refIdx, false)) || colocatedMVP(l, c.x + (c.w >> 1), c.y + (c.h >> 1), cm, refIdx, false)) {
            cm = roundPrec(cm, sft);
            LT[num] = RT[num] = LB[num] = cm;
            num++;
          }
        }
        while (num < 2) { LT[num] = RT[num] = LB[num] = Mv(); num++; }
      }
    }
    for (int i = 0; i < 2; i++) { lt[i] = roundPrec(LT[i], sft); rt[i] = roundPrec(RT[i], sft); lb[i] = roundPrec(LB[i], sft); }
  }
  static bool spreadOverLimit(int a, int b, int c, int d, int predType) {   // InterPrediction.cpp:850
    const int s4 = 4 << 11, tap = 6;
    if (predType == 3) {
      int W = std::max(std::max(0, 4 * a + s4), std::max(4 * c, 4 * a + 4 * c + s4)) - std::min(std::min(0, 4 * a + s4), std::min(4 * c, 4 * a + 4 * c + s4));
      int H = std::max(std::max(0, 4 * b), std::max(4 * d + s4, 4 * b + 4 * d + s4)) - std::min(std::min(0, 4 * b), std::min(4 * d + s4, 4 * b + 4 * d + s4));
      W = (W >> 11) + tap + 3;
      H = (H >> 11) + tap + 3;
      return W * H > (tap + 9) * (tap + 9);
    }
    int W = std::max(0, 4 * a + s4) - std::min(0, 4 * a + s4), H = std::max(0, 4 * b) - std::min(0, 4 * b);
    W = (W >> 11) + tap + 3;
    H = (H >> 11) + tap + 3;
    if (W * H > (tap + 9) * (tap + 5)) return true;
    W = std::max(0, 4 * c) - std::min(0, 4 * c);
    H = std::max(0, 4 * d + s4) - std::min(0, 4 * d + s4);
    W = (W >> 11) + tap + 3;
    H = (H >> 11) + tap + 3;
    return W * H > (tap + 5) * (tap + 9);
  }
  void setAllAffineMv(int ci, Mv lt, Mv rt, Mv lb, int l, bool clip) {
    const vvcr_cu &c = S.cu[ci];
    const int type = cuAffType[ci];
    if (clip) {
      lt = wrapStore(lt);
      rt = wrapStore(rt);
      if (type == AFF_6P) lb = wrapStore(lb);
    }
    const int s = MAX_CU_DEPTH;
    const int dHx = (rt - lt).h * (1 << (s - floorLog2(c.w))), dHy = (rt - lt).v * (1 << (s - floorLog2(c.w)));
    int dVx, dVy;
    if (type == AFF_6P) {
      dVx = (lb - lt).h * (1 << (s - floorLog2(c.h)));
      dVy = (lb - lt).v * (1 << (s - floorLog2(c.h)));
    } else {
      dVx = -dHy;
      dVy = dHx;
    }
    const int bx = lt.h * (1 << s), by = lt.v * (1 << s);
    const bool over = spreadOverLimit(dHx, dHy, dVx, dVy, puInterDir[c.firstpu]);
    for (int h = 0; h < c.h; h += 4)
      for (int w = 0; w < c.w; w += 4) {
        int mx, my;
        if (!over) { mx = bx + dHx * (2 + w) + dVx * (2 + h); my = by + dHy * (2 + w) + dVy * (2 + h); }
        else { mx = bx + dHx * (c.w >> 1) + dVx * (c.h >> 1); my = by + dHy * (c.w >> 1) + dVy * (c.h >> 1); }
        roundAffineMv(mx, my, s);
        const Mv m = clipStore(Mv(mx, my));
        Mi &d = at(c.x + w, c.y + h);
        d.mv[l][0] = m.h;
        d.mv[l][1] = m.v;
      }
    const int pi = c.firstpu;
    puAff[l][0][pi] = lt;
    puAff[l][1][pi] = rt;
    puAff[l][2][pi] = lb;
  }
  void controlPointCand(int ci, const Mi mi[4], const bool avail[4], const int *verIdx, int bcw, int model, int verNum, AffMergeCtx &am) {
    const vvcr_cu &c = S.cu[ci];
    const int s = MAX_CU_DEPTH;
    const int shiftHtoW = s + floorLog2(c.w) - floorLog2(c.h);
    Mv cm[2][4];
    int ref[2] = {-1, -1}, dir = 0;
    const int type = verNum == 2 ? AFF_4P : AFF_6P;
    for (int i = 0; i < verNum; i++)
      if (!avail[verIdx[i]]) return;
    for (int l = 0; l < 2; l++) {
      bool ok = true;
      for (int i = 0; i < verNum; i++) ok &= mi[verIdx[i]].ref[l] >= 0;
      if (!ok) continue;
      bool same = true;
      for (int i = 1; i < verNum; i++) same &= mi[verIdx[i]].ref[l] == mi[verIdx[0]].ref[l];
      if (same) { dir |= l + 1; ref[l] = mi[verIdx[0]].ref[l]; }
    }
    if (dir == 0) return;
    for (int l = 0; l < 2; l++) {
      if (dir & (l + 1)) {
        for (int i = 0; i < verNum; i++) cm[l][verIdx[i]] = Mv(mi[verIdx[i]].mv[l][0], mi[verIdx[i]].mv[l][1]);
        switch (model) {
          case 1: cm[l][2] = clipStore(Mv(cm[l][3].h + cm[l][0].h - cm[l][1].h, cm[l][3].v + cm[l][0].v - cm[l][1].v)); break;
          case 2: cm[l][1] = clipStore(Mv(cm[l][3].h + cm[l][0].h - cm[l][2].h, cm[l][3].v + cm[l][0].v - cm[l][2].v)); break;
          case 3: cm[l][0] = clipStore(Mv(cm[l][1].h + cm[l][2].h - cm[l][3].h, cm[l][1].v + cm[l][2].v - cm[l][3].v)); break;
          case 5: {
            int vx = cm[l][0].h * (1 << s) + (cm[l][2].v - cm[l][0].v) * (1 << shiftHtoW);
            int vy = cm[l][0].v * (1 << s) - (cm[l][2].h - cm[l][0].h) * (1 << shiftHtoW);
            roundAffineMv(vx, vy, s);
            cm[l][1] = clipStore(Mv(vx, vy));
            break;
          }
          default: break;
        }
      } else {
        for (int i = 0; i < 4; i++) cm[l][i] = Mv();
      }
    }
    const int k = am.numValid;
    for (int i = 0; i < 3; i++) {
      am.mvf[(k << 1)][i].mv = cm[0][i]; am.mvf[(k << 1)][i].ref = ref[0];
      am.mvf[(k << 1) + 1][i].mv = cm[1][i]; am.mvf[(k << 1) + 1][i].ref = ref[1];
    }
    am.interDir[k] = dir;
    am.affType[k] = type;
    am.bcw[k] = dir == 3 ? bcw : BCW_DEFAULT;
    am.numValid++;
  }
  void clipColPos(const vvcr_cu &c, int &x, int &y) const {   // clipColPos (:2857)
    const int l2 = sps.ctuLog2;
    const int cx = (c.x >> l2) << l2, cy = (c.y >> l2) << l2;
    const int horMax = std::min(S.W - 1, cx + S.ctuSize + 3), horMin = std::max(0, cx);
    const int verMax = std::min(S.H - 1, cy + S.ctuSize - 1), verMin = std::max(0, cy);
    x = std::min(horMax, std::max(horMin, x));
    y = std::min(verMax, std::max(verMin, y));
  }
  // PU::getInterMergeSubPuMvpCand (:2872) with the left candidate as the only spatial input
  // fill: also build the sub-block motion (only needed when this candidate is the one selected)
  bool subPuMvpCand(int ci, const MergeCtx &sp, int count, MvField out[2], int &outDir, bool fill) {
    const vvcr_cu &c = S.cu[ci];
    const int colPoc = sh->isInterB() ? refPoc(sh->colFromL0 ? 1 : 0, sh->colRefIdx) : refPoc(0, sh->colRefIdx);
    const int colList = sh->isInterB() ? 1 - (sh->colFromL0 ? 1 : 0) : 0;
    (void)colPoc;
    Mv tmv;
    if (count) {
      if ((sp.interDir[0] & 1) && sh->refPoc[0][sp.mvf[0].ref] == refPoc(colList, sh->colRefIdx)) tmv = sp.mvf[0].mv;
      else if (sh->isInterB() && (sp.interDir[0] & 2) && sh->refPoc[1][sp.mvf[1].ref] == refPoc(colList, sh->colRefIdx)) tmv = sp.mvf[1].mv;
    }
    const int nLine = std::max(c.w >> 3, 1), nCol = std::max(c.h >> 3, 1);
    const int pH = nCol == 1 ? c.h : 8, pW = nLine == 1 ? c.w : 8;
    const Mv t = changePrec(tmv, -4);   // sixteenth -> integer
    int cx = c.x + (c.w >> 1) + t.h, cy = c.y + (c.h >> 1) + t.v;
    clipColPos(c, cx, cy);
    cx &= ~7; cy &= ~7;
    if (!col || col->intra) return false;
    const Mi &mi = col->at8(cx, cy);
    bool found = false;
    outDir = 0;
    if (mi.isInter) {
      for (int l = 0; l < (sh->isInterB() ? 2 : 1); l++) {
        Mv cm;
        if (colocatedMVP(l, cx, cy, cm, 0, true)) {
          out[l].mv = cm; out[l].ref = 0;
          outDir |= 1 << l;
          found = true;
        } else {
          out[l].mv = Mv(); out[l].ref = -1;
          outDir &= ~(1 << l);
        }
      }
    }
    if (!found || !fill) return found;
    subW = c.w >> 2;
    subPu.assign((size_t)(c.w >> 2) * (c.h >> 2), Mi());
    const int xOff = (pW >> 1) + t.h, yOff = (pH >> 1) + t.v;
    const bool restrictBi = isBipredRestriction(c);
    // a sub-block's motion depends only on the collocated record it reads (getColocatedMVP with refIdx 0):
    // neighbouring sub-blocks mostly read records of one collocated PU, so the last derivation is reused
    // when the record is byte-identical (no scaling / compression redone)
    const Mi *prevCm = nullptr;
    Mi m;
    for (int y = c.y; y < c.y + c.h; y += pH)
      for (int x = c.x; x < c.x + c.w; x += pW) {
        int px = x + xOff, py = y + yOff;
        clipColPos(c, px, py);
        px &= ~7; py &= ~7;
        const Mi &cm = col->at8(px, py);
        if (!prevCm || std::memcmp(prevCm, &cm, sizeof(Mi)) != 0) {
          prevCm = &cm;
          m = Mi();
          m.isInter = true;
          m.slice = (uint16_t)sliceIdx;
          bool f = false;
          if (cm.isInter) {
            for (int l = 0; l < (sh->isInterB() ? 2 : 1); l++) {
              Mv v;
              if (colocatedMVP(l, px, py, v, 0, true)) { m.ref[l] = 0; m.mv[l][0] = v.h; m.mv[l][1] = v.v; f = true; }
            }
          }
          if (!f) {
            for (int l = 0; l < 2; l++) { m.mv[l][0] = out[l].mv.h; m.mv[l][1] = out[l].mv.v; m.ref[l] = out[l].ref; }
            if (!sh->isInterB()) { m.mv[1][0] = m.mv[1][1] = 0; m.ref[1] = -1; }
          }
          m.interDir = (m.ref[0] != -1 ? 1 : 0) + (m.ref[1] != -1 ? 2 : 0);
          if (restrictBi && m.interDir == 3) { m.interDir = 1; m.mv[1][0] = m.mv[1][1] = 0; m.ref[1] = -1; }
        }
        for (int yy = (y - c.y) >> 2; yy < (y - c.y + pH) >> 2; yy++)
          for (int xx = (x - c.x) >> 2; xx < (x - c.x + pW) >> 2; xx++) subPu[(size_t)yy * subW + xx] = m;
      }
    return true;
  }
  void affineMergeCand(int ci, AffMergeCtx &am, int mrgCandIdx) {
    const vvcr_cu &c = S.cu[ci];
    const int maxN = ph.maxNumAffineMergeCand;
    for (int i = 0; i < maxN; i++) {
      for (int k = 0; k < 3; k++) { am.mvf[i << 1][k] = MvField(); am.mvf[(i << 1) + 1][k] = MvField(); }
      am.interDir[i] = 0; am.affType[i] = AFF_4P; am.mrgType[i] = MRG_DEFAULT; am.bcw[i] = BCW_DEFAULT;
    }
    am.numValid = 0;
    const bool enableSubPu = sps.sbtmvp && !(sh->poc == refPoc(0, 0) && (sh->nalType >= 7 && sh->nalType <= 10));
    if (enableSubPu && ph.tmvp) {
      MergeCtx sp;
      int pos = 0;
      const int yB = c.y + c.h - 1;
      const int pL = puRestricted(ci, c.x - 1, yB);
      if (pL >= 0 && isDiffMER(c.x, c.y, S.cu[pL].x, S.cu[pL].y) && pL != ci && isInterCu(pL)) {
        const Mi &ml = at(c.x - 1, yB);
        sp.interDir[pos] = ml.interDir;
        sp.mvf[pos << 1].mv = Mv(ml.mv[0][0], ml.mv[0][1]);
        sp.mvf[pos << 1].ref = ml.ref[0];
        if (sh->isInterB()) { sp.mvf[(pos << 1) + 1].mv = Mv(ml.mv[1][0], ml.mv[1][1]); sp.mvf[(pos << 1) + 1].ref = ml.ref[1]; }
        pos++;
      }
      MvField out[2];
      int dir = 0;
      if (subPuMvpCand(ci, sp, pos, out, dir, mrgCandIdx == am.numValid)) {
        for (int k = 0; k < 3; k++) { am.mvf[am.numValid << 1][k] = out[0]; am.mvf[(am.numValid << 1) + 1][k] = out[1]; }
        am.interDir[am.numValid] = dir;
        am.affType[am.numValid] = AFF_NUM;
        am.mrgType[am.numValid] = MRG_SUBPU_ATMVP;
        if (am.numValid == mrgCandIdx) return;
        am.numValid++;
        if (am.numValid == maxN) return;
      }
    }
    if (sps.affine) {
      int npu[5], num = 0;
      const int xR = c.x + c.w - 1, yB = c.y + c.h - 1;
      auto affNeigh = [&](int x, int y) {
        const int n = puRestricted(ci, x, y);
        return (n >= 0 && S.cu[n].affine && puMrgType[n] == MRG_DEFAULT && isDiffMER(c.x, c.y, S.cu[n].x, S.cu[n].y)) ? n : -1;
      };
      int n = affNeigh(c.x - 1, yB + 1);
      if (n >= 0) npu[num++] = n;
      else if ((n = affNeigh(c.x - 1, yB)) >= 0) npu[num++] = n;
      n = affNeigh(xR + 1, c.y - 1);
      if (n >= 0) npu[num++] = n;
      else if ((n = affNeigh(xR, c.y - 1)) >= 0) npu[num++] = n;
      else if ((n = affNeigh(c.x - 1, c.y - 1)) >= 0) npu[num++] = n;
      for (int k = 0; k < num; k++) {
        const int nb = npu[k];
        Mv cm[2][3];
        const int type = cuAffType[nb];
        cuAffType[ci] = type;   // the reference sets the current CU's model to the neighbour's here (:2559)
        if (puInterDir[nb] != 2) inheritedAffineMv(ci, nb, 0, type, cm[0]);
        if (sh->isInterB() && puInterDir[nb] != 1) inheritedAffineMv(ci, nb, 1, type, cm[1]);
        for (int i = 0; i < 3; i++) {
          am.mvf[am.numValid << 1][i].mv = cm[0][i]; am.mvf[am.numValid << 1][i].ref = puRef[0][nb];
          am.mvf[(am.numValid << 1) + 1][i].mv = cm[1][i]; am.mvf[(am.numValid << 1) + 1][i].ref = puRef[1][nb];
        }
        am.interDir[am.numValid] = puInterDir[nb];
        am.affType[am.numValid] = type;
        am.bcw[am.numValid] = cuBcw[nb];
        if (am.numValid == mrgCandIdx) return;
        am.numValid++;
        if (am.numValid == maxN) return;
      }
      // constructed candidates
      Mi mi[4];
      bool avail[4] = {false, false, false, false};
      int neighBcw[2] = {BCW_DEFAULT, BCW_DEFAULT};
      const int ltp[3][2] = {{c.x - 1, c.y - 1}, {c.x, c.y - 1}, {c.x - 1, c.y}};
      for (int i = 0; i < 3; i++) {
        const int q = puRestricted(ci, ltp[i][0], ltp[i][1]);
        if (q >= 0 && isInterCu(q) && isDiffMER(c.x, c.y, S.cu[q].x, S.cu[q].y)) {
          avail[0] = true; mi[0] = at(ltp[i][0], ltp[i][1]); neighBcw[0] = cuBcw[q]; break;
        }
      }
      const int rtp[2][2] = {{xR, c.y - 1}, {xR + 1, c.y - 1}};
      for (int i = 0; i < 2; i++) {
        const int q = puRestricted(ci, rtp[i][0], rtp[i][1]);
        if (q >= 0 && isInterCu(q) && isDiffMER(c.x, c.y, S.cu[q].x, S.cu[q].y)) {
          avail[1] = true; mi[1] = at(rtp[i][0], rtp[i][1]); neighBcw[1] = cuBcw[q]; break;
        }
      }
      const int lbp[2][2] = {{c.x - 1, yB}, {c.x - 1, yB + 1}};
      for (int i = 0; i < 2; i++) {
        const int q = puRestricted(ci, lbp[i][0], lbp[i][1]);
        if (q >= 0 && isInterCu(q) && isDiffMER(c.x, c.y, S.cu[q].x, S.cu[q].y)) {
          avail[2] = true; mi[2] = at(lbp[i][0], lbp[i][1]); break;
        }
      }
      if (ph.tmvp) {
        int x0, y0;
        const bool c0 = posC0(c, x0, y0);
        Mv cm;
        if (c0 && colocatedMVP(0, x0, y0, cm, 0, false)) {
          mi[3].mv[0][0] = cm.h; mi[3].mv[0][1] = cm.v; mi[3].ref[0] = 0; mi[3].interDir = 1; avail[3] = true;
        }
        if (sh->isInterB() && c0 && colocatedMVP(1, x0, y0, cm, 0, false)) {
          mi[3].mv[1][0] = cm.h; mi[3].mv[1][1] = cm.v; mi[3].ref[1] = 0; mi[3].interDir |= 2; avail[3] = true;
        }
      }
      static const int model[6][4] = {{0, 1, 2}, {0, 1, 3}, {0, 2, 3}, {1, 2, 3}, {0, 1}, {0, 2}};
      static const int verNum[6] = {3, 3, 3, 3, 2, 2};
      for (int idx = sps.affineType ? 0 : 4; idx < 6; idx++) {
        controlPointCand(ci, mi, avail, model[idx], idx == 3 ? neighBcw[1] : neighBcw[0], idx, verNum[idx], am);
        if (am.numValid != 0 && am.numValid - 1 == mrgCandIdx) return;
        if (am.numValid == maxN) return;
      }
    }
    int cnt = am.numValid;
    while (cnt < maxN) {
      for (int k = 0; k < 3; k++) { am.mvf[cnt << 1][k].mv = Mv(); am.mvf[cnt << 1][k].ref = 0; }
      am.interDir[cnt] = 1;
      if (sh->isInterB()) {
        for (int k = 0; k < 3; k++) { am.mvf[(cnt << 1) + 1][k].mv = Mv(); am.mvf[(cnt << 1) + 1][k].ref = 0; }
        am.interDir[cnt] = 3;
      }
      am.affType[cnt] = AFF_4P;
      if (cnt == mrgCandIdx) return;
      cnt++;
      am.numValid++;
    }
  }

  // ----------------------------------------------------------------------------------------------
  // PU::spanMotionInfo (:3027)
  // ----------------------------------------------------------------------------------------------
  void span(int ci) {
    const vvcr_cu &c = S.cu[ci];
    const int pi = c.firstpu;
    if (puMrgType[pi] == MRG_SUBPU_ATMVP) {
      for (int y = 0; y < c.h >> 2; y++) std::memcpy((void *)&at(c.x, c.y + 4 * y), &subPu[(size_t)y * subW], (size_t)(c.w >> 2) * sizeof(Mi));
      col8(c);
      return;
    }
    Mi mi;
    mi.isInter = true;
    mi.slice = (uint16_t)sliceIdx;
    mi.interDir = (int8_t)puInterDir[pi];
    mi.altHpel = cuImv[ci] == IMV_HPEL;
    for (int l = 0; l < 2; l++) { mi.mv[l][0] = puMv[l][pi].h; mi.mv[l][1] = puMv[l][pi].v; mi.ref[l] = (int16_t)puRef[l][pi]; }
    mi.bcw = 0;
    if (c.affine) {   // the AMVR / BCW bits stay as the memset left them (zero); the MVs are setAllAffineMv's
      for (int y = c.y; y < c.y + c.h; y += 4) {
        Mi *d = &at(c.x, y);
        for (int x = 0; x < c.w >> 2; x++) {
          Mi t = mi;
          for (int l = 0; l < 2; l++)
            if (mi.ref[l] != -1) { t.mv[l][0] = d[x].mv[l][0]; t.mv[l][1] = d[x].mv[l][1]; }
            else t.mv[l][0] = t.mv[l][1] = 0;
          t.altHpel = 0;
          d[x] = t;
        }
      }
      col8(c);
      return;
    }
    {   // the first unit row, then whole-row copies (wide stores instead of two per 24-byte record)
      const int n = c.w >> 2;
      Mi *d0 = &at(c.x, c.y);
      for (int x = 0; x < n; x++) d0[x] = mi;
      for (int y = c.y + 4; y < c.y + c.h; y += 4) std::memcpy((void *)&at(c.x, y), d0, (size_t)n * sizeof(Mi));
    }
    // the collocated view of a CU of one motion: mi at its 8-aligned units
    const Mi cmi = colMi(mi);
    for (int y = (c.y + 7) & ~7; y < c.y + c.h; y += 8)
      for (int x = (c.x + 7) & ~7; x < c.x + c.w; x += 8) (*col8f)[(size_t)(y >> 3) * w8 + (x >> 3)] = cmi;
  }
  // the parse-time spanMotionInfo (CABACReader::prediction_unit :2072): merge PUs carry their parsed
  // (not yet derived) fields; only what later derivation does not overwrite survives (GEO / affine areas)
  void spanParse(int ci) {
    const vvcr_cu &c = S.cu[ci];
    const vvcr_pu &u = S.pu[c.firstpu];
    Mi mi;
    mi.isInter = true;
    mi.slice = (uint16_t)sliceIdx;
    mi.interDir = (int8_t)u.interdir;
    mi.altHpel = c.imv == IMV_HPEL;
    mi.ref[0] = (int16_t)u.ref0; mi.ref[1] = (int16_t)u.ref1;
    for (int y = c.y; y < c.y + c.h; y += 4)
      for (int x = c.x; x < c.x + c.w; x += 4) {
        Mi &d = at(x, y);
        if (c.affine) {
          d.isInter = true; d.altHpel = 0; d.bcw = 0; d.pad_ = 0; d.interDir = mi.interDir; d.slice = mi.slice;
          for (int l = 0; l < 2; l++) { if (mi.ref[l] == -1) d.mv[l][0] = d.mv[l][1] = 0; d.ref[l] = mi.ref[l]; }
        } else {
          d = mi;
        }
      }
  }

  // ----------------------------------------------------------------------------------------------
  // GEO: PU::getGeoMergeCandidates (:3357), spanGeoMotionInfo (:3416)
  // ----------------------------------------------------------------------------------------------
  void geo(int ci) {
    const vvcr_cu &c = S.cu[ci];
    const vvcr_pu &u = S.pu[c.firstpu];
    MergeCtx tmp, g;
    mergeCandidates(ci, tmp, -1);
    g.numValid = 0;
    for (int i = 0; i < 6; i++) { g.interDir[i] = 0; g.mvf[2 * i] = MvField(); g.mvf[2 * i + 1] = MvField(); }
    for (int i = 0; i < ph.maxNumMergeCand && g.numValid < 6; i++) {
      const int par = i & 1;
      if (tmp.interDir[i] & (1 + par)) {
        g.interDir[g.numValid] = 1 + par;
        g.mvf[(g.numValid << 1) + !par] = MvField();
        g.mvf[(g.numValid << 1) + par] = tmp.mvf[(i << 1) + par];
        g.numValid++;
        continue;
      }
      if (tmp.interDir[i] & (2 - par)) {
        g.interDir[g.numValid] = 2 - par;
        g.mvf[(g.numValid << 1) + !par] = tmp.mvf[(i << 1) + !par];
        g.mvf[(g.numValid << 1) + par] = MvField();
        g.numValid++;
      }
    }
    const int i0 = u.geoi0, i1 = u.geoi1;
    vvcr_geo row;
    std::memset(&row, 0, sizeof(row));
    row.cu = ci;
    for (int k = 0; k < 2; k++) {
      const int i = k ? i1 : i0;
      const int dir = g.interDir[i];
      const MvField &f = dir == 2 ? g.mvf[2 * i + 1] : g.mvf[2 * i];
      row.cand[k][0] = dir; row.cand[k][1] = dir == 2 ? 1 : 0; row.cand[k][2] = f.ref;
      row.cand[k][3] = f.mv.h; row.cand[k][4] = f.mv.v; row.cand[k][5] = 0;
    }
    geoRows.push_back(row);
    // motion field
    Mi bi;
    bi.isInter = true;
    bi.slice = (uint16_t)sliceIdx;
    const int d0 = g.interDir[i0], d1 = g.interDir[i1];
    auto mvOf = [&](int i, int l) { return g.mvf[2 * i + l]; };
    if (d0 == 1 && d1 == 2) {
      bi.interDir = 3; bi.ref[0] = (int16_t)mvOf(i0, 0).ref; bi.ref[1] = (int16_t)mvOf(i1, 1).ref;
      bi.mv[0][0] = mvOf(i0, 0).mv.h; bi.mv[0][1] = mvOf(i0, 0).mv.v; bi.mv[1][0] = mvOf(i1, 1).mv.h; bi.mv[1][1] = mvOf(i1, 1).mv.v;
    } else if (d0 == 2 && d1 == 1) {
      bi.interDir = 3; bi.ref[0] = (int16_t)mvOf(i1, 0).ref; bi.ref[1] = (int16_t)mvOf(i0, 1).ref;
      bi.mv[0][0] = mvOf(i1, 0).mv.h; bi.mv[0][1] = mvOf(i1, 0).mv.v; bi.mv[1][0] = mvOf(i0, 1).mv.h; bi.mv[1][1] = mvOf(i0, 1).mv.v;
    } else if (d0 == 1 && d1 == 1) {
      bi.interDir = 1; bi.ref[0] = (int16_t)mvOf(i1, 0).ref; bi.ref[1] = -1;
      bi.mv[0][0] = mvOf(i1, 0).mv.h; bi.mv[0][1] = mvOf(i1, 0).mv.v;
    } else if (d0 == 2 && d1 == 2) {
      bi.interDir = 2; bi.ref[0] = -1; bi.ref[1] = (int16_t)mvOf(i1, 1).ref;
      bi.mv[1][0] = mvOf(i1, 1).mv.h; bi.mv[1][1] = mvOf(i1, 1).mv.v;
    }
    static int16_t angleOf[64], distOf[64];
    static std::once_flag once;
    std::call_once(once, [] {
      static const int8_t a2m[32] = {0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1, 0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1};
      int m = 0;
      for (int a = 0; a < 32; a++)
        for (int d = 0; d < 4; d++) {
          if ((d == 0 && a >= 16) || ((d == 2 || d == 0) && (a2m[a] == 0 || a2m[a] == 5)) || a2m[a] == -1) continue;
          if (m < 64) { angleOf[m] = (int16_t)a; distOf[m] = (int16_t)d; }
          m++;
        }
    });
    static const int8_t dis[32] = {8, 8, 8, 8, 4, 4, 2, 1, 0, -1, -2, -4, -4, -8, -8, -8, -8, -8, -8, -8, -4, -4, -2, -1, 0, 1, 2, 4, 4, 8, 8, 8};
    const int angle = angleOf[u.geodir], distIdx = distOf[u.geodir];
    const bool isFlip = angle >= 13 && angle <= 27;
    const int dX = angle, dY = (dX + 8) % 32;
    int offX = (-c.w) >> 1, offY = (-c.h) >> 1;
    if (distIdx > 0) {
      if (angle % 16 == 8 || (angle % 16 != 0 && c.h >= c.w)) offY += angle < 16 ? ((distIdx * c.h) >> 3) : -((distIdx * c.h) >> 3);
      else offX += angle < 16 ? ((distIdx * c.w) >> 3) : -((distIdx * c.w) >> 3);
    }
    for (int y = 0; y < c.h >> 2; y++) {
      const int lookY = (((4 * y + offY) << 1) + 5) * dis[dY];
      for (int x = 0; x < c.w >> 2; x++) {
        const int midx = (((4 * x + offX) << 1) + 5) * dis[dX] + lookY;
        const int mask = std::abs(midx) < 32 ? 2 : (midx <= 0 ? (1 - isFlip) : isFlip);
        Mi &d = at(c.x + 4 * x, c.y + 4 * y);
        d.isInter = true;
        d.slice = (uint16_t)sliceIdx;
        if (mask == 2) {
          d.interDir = bi.interDir; d.ref[0] = bi.ref[0]; d.ref[1] = bi.ref[1];
          std::memcpy(d.mv, bi.mv, sizeof(d.mv));
        } else {
          const int i = mask == 0 ? i0 : i1;
          d.interDir = (int8_t)g.interDir[i];
          for (int l = 0; l < 2; l++) {
            d.ref[l] = (int16_t)mvOf(i, l).ref;
            d.mv[l][0] = mvOf(i, l).mv.h;
            d.mv[l][1] = mvOf(i, l).mv.v;
          }
        }
      }
    }
    col8(c);
    // InterPrediction::motionCompensationGeo (InterPrediction.cpp:1761-1769) leaves the PU with
    // setMergeInfo of the second candidate
    const int pi = c.firstpu;
    puInterDir[pi] = g.interDir[i1];
    for (int l = 0; l < 2; l++) { puMv[l][pi] = mvOf(i1, l).mv; puRef[l][pi] = mvOf(i1, l).ref; }
    puMrgType[pi] = MRG_DEFAULT;
    S.pu[pi].mergeidx = i1;
    cuImv[ci] = 0;
    cuBcw[ci] = BCW_DEFAULT;
  }

  // ----------------------------------------------------------------------------------------------
  // DecCu::xDeriveCUMV (DecCu.cpp:878) for one CU, then CU::saveMotionInHMVP (UnitTools.cpp:243)
  // ----------------------------------------------------------------------------------------------
  bool isBiPredDiffDirEqDist(int pi) const {   // PU::isBiPredFromDifferentDirEqDistPoc (:3162)
    if (puRef[0][pi] < 0 || puRef[1][pi] < 0) return false;
    if (sh->refLT[0][puRef[0][pi]] || sh->refLT[1][puRef[1][pi]]) return false;
    const int p0 = refPoc(0, puRef[0][pi]), p1 = refPoc(1, puRef[1][pi]), p = sh->poc;
    return (p - p0) * (p - p1) < 0 && std::abs(p - p0) == std::abs(p - p1);
  }
  void deriveCu(int ci) {
    vvcr_cu &c = S.cu[ci];
    const int pi = c.firstpu;
    vvcr_pu &u = S.pu[pi];
    const PuSyntax &s = S.pux[pi];
    // the parse-time span survives in part only for GEO (its AMVR bit); an affine CU's span writes every
    // byte after the derivation, which reads no unit of the CU itself (its neighbours are outside it)
    if (c.geo) spanParse(ci);
    if (u.merge) {
      if (u.mmvd) {   // getInterMergeCandidates + getInterMMVDMergeCandidates + setMmvdMergeCandiInfo
        const int base = s.mmvdMergeIdx / 32;
        MergeCtx m;
        mergeCandidates(ci, m, base + 1);
        int nb = 0;
        for (int k = 0; k < m.numValid && nb < 2; k++) {
          if (m.mrgType[k] != MRG_DEFAULT) continue;
          const int r0 = m.mvf[k << 1].ref, r1 = m.mvf[(k << 1) + 1].ref;
          if (r0 >= 0 && r1 >= 0) { m.mmvdBase[nb][0] = m.mvf[k << 1]; m.mmvdBase[nb][1] = m.mvf[(k << 1) + 1]; }
          else if (r0 >= 0) { m.mmvdBase[nb][0] = m.mvf[k << 1]; m.mmvdBase[nb][1] = MvField(); }
          else if (r1 >= 0) { m.mmvdBase[nb][0] = MvField(); m.mmvdBase[nb][1] = m.mvf[(k << 1) + 1]; }
          m.mmvdAltHpel[nb] = m.altHpel[k];
          nb++;
        }
        mmvdInfo(ci, m, s.mmvdMergeIdx);
      } else if (c.geo) {
        geo(ci);
        return;   // spanGeoMotionInfo done; GEO CUs are not added to the history table
      } else if (c.affine) {
        AffMergeCtx am;
        affineMergeCand(ci, am, u.mergeidx);
        const int k = u.mergeidx;
        puInterDir[pi] = am.interDir[k];
        cuAffType[ci] = am.affType[k];
        cuBcw[ci] = am.bcw[k];
        puMrgType[pi] = am.mrgType[k];
        if (am.mrgType[k] == MRG_SUBPU_ATMVP) {
          puRef[0][pi] = am.mvf[k << 1][0].ref;
          puRef[1][pi] = am.mvf[(k << 1) + 1][0].ref;
        } else {
          for (int l = 0; l < 2; l++)
            if (sh->numRef[l] > 0) {
              setAllAffineMv(ci, am.mvf[(k << 1) + l][0].mv, am.mvf[(k << 1) + l][1].mv, am.mvf[(k << 1) + l][2].mv, l, false);
              puRef[l][pi] = am.mvf[(k << 1) + l][0].ref;
            }
        }
        span(ci);
        return;   // affine CUs are not added to the history table
      } else {
        MergeCtx m;
        mergeCandidates(ci, m, u.mergeidx);
        setMergeInfo(ci, m, u.mergeidx);
      }
      span(ci);
    } else {
      const int imv = c.imv;
      if (c.affine) {
        for (int l = 0; l < 2; l++) {
          if (sh->numRef[l] <= 0 || !(puInterDir[pi] & (1 << l))) continue;
          Mv lt[2], rt[2], lb[2];
          const int ref = l ? u.ref1 : u.ref0;
          fillAffineMvpCand(ci, l, ref, imv, cuAffType[ci], lt, rt, lb);
          const int mp = s.mvpIdx[l];
          const int sft = kAffShift[imv];
          const Mv d0 = changePrec(Mv(s.mvdAffi[l][0][0], s.mvdAffi[l][0][1]), sft);
          const Mv d1 = changePrec(Mv(s.mvdAffi[l][1][0], s.mvdAffi[l][1][1]), sft);
          const Mv d2 = changePrec(Mv(s.mvdAffi[l][2][0], s.mvdAffi[l][2][1]), sft);
          const Mv mLT = lt[mp] + d0;
          const Mv mRT = rt[mp] + d1 + d0;
          Mv mLB;
          if (cuAffType[ci] == AFF_6P) mLB = lb[mp] + d2 + d0;
          setAllAffineMv(ci, mLT, mRT, mLB, l, true);
        }
        span(ci);
        return;
      }
      for (int l = 0; l < 2; l++) {
        if (sh->numRef[l] <= 0 || !(puInterDir[pi] & (1 << l))) continue;
        Mv cand[2];
        const int ref = l ? u.ref1 : u.ref0;
        fillMvpCand(ci, l, ref, imv, cand);
        const Mv d = changePrec(Mv(s.mvd[l][0], s.mvd[l][1]), kAmvrShift[imv]);
        puMv[l][pi] = wrapStore(cand[s.mvpIdx[l]] + d);
      }
      span(ci);
    }
    // CU::saveMotionInHMVP
    if (!c.geo && !c.affine) {
      Mi mi = at(c.x, c.y);
      mi.bcw = mi.interDir == 3 ? (uint8_t)cuBcw[ci] : BCW_DEFAULT;
      const int L = sps.log2ParMrgLevel;
      const int xBr = c.x + c.w, yBr = c.y + c.h;
      if ((xBr >> L) > (c.x >> L) && (yBr >> L) > (c.y >> L)) {
        int same = -1;
        for (int k = 0; k < (int)lut.size(); k++)
          if (lut[k].same(mi)) { same = k; break; }
        if (same >= 0) lut.erase(lut.begin() + same);
        else if (lut.size() == 5) lut.erase(lut.begin());
        lut.push_back(mi);
      }
    }
  }
  void setMergeInfo(int ci, const MergeCtx &m, int k) {   // MergeCtx::setMergeInfo (ContextModelling.cpp:320)
    vvcr_cu &c = S.cu[ci];
    const int pi = c.firstpu;
    puInterDir[pi] = m.interDir[k];
    cuImv[ci] = (!c.geo && m.altHpel[k]) ? IMV_HPEL : 0;
    puMrgType[pi] = m.mrgType[k];
    for (int l = 0; l < 2; l++) { puMv[l][pi] = m.mvf[(k << 1) + l].mv; puRef[l][pi] = m.mvf[(k << 1) + l].ref; }
    cuBcw[ci] = m.interDir[k] == 3 ? m.bcw[k] : BCW_DEFAULT;
    restrictBiOne(ci);
  }
  void restrictBiOne(int ci) {   // PU::restrictBiPredMergeCandsOne (:3185)
    const int pi = S.cu[ci].firstpu;
    if (isBipredRestriction(S.cu[ci]) && puInterDir[pi] == 3) {
      puInterDir[pi] = 1;
      puRef[1][pi] = -1;
      puMv[1][pi] = Mv();
      cuBcw[ci] = BCW_DEFAULT;
    }
  }
  void mmvdInfo(int ci, const MergeCtx &m, int candIdx) {   // MergeCtx::setMmvdMergeCandiInfo (ContextModelling.cpp:359)
    const int pi = S.cu[ci].firstpu;
    const int refMvd[8] = {1 << 2, 2 << 2, 4 << 2, 8 << 2, 16 << 2, 32 << 2, 64 << 2, 128 << 2};
    int t = candIdx;
    const int group = t / 64;
    t -= group * 64;
    const int base = t / 32;
    t -= base * 32;
    const int step = t / 4, posn = t - step * 4;
    int off = refMvd[step];
    if (ph.disFracMmvd) off <<= 2;
    const int r0 = m.mmvdBase[base][0].ref, r1 = m.mmvdBase[base][1].ref;
    auto dirMv = [&](int p) { return p == 0 ? Mv(off, 0) : p == 1 ? Mv(-off, 0) : p == 2 ? Mv(0, off) : Mv(0, -off); };
    Mv t0, t1;
    if (r0 != -1 && r1 != -1) {
      const int poc0 = refPoc(0, r0), poc1 = refPoc(1, r1), cur = sh->poc;
      t0 = dirMv(posn);
      if (poc0 - cur == poc1 - cur) t1 = t0;
      else if (std::abs(poc1 - cur) > std::abs(poc0 - cur)) {
        const int sc = distScale(cur, poc0, cur, poc1);
        t1 = t0;
        if (sh->refLT[0][r0] || sh->refLT[1][r1]) {
          if ((poc1 - cur) * (poc0 - cur) > 0) t0 = t1;
          else t0 = Mv(-t1.h, -t1.v);
        } else t0 = scaleMv(t1, sc);
      } else {
        const int sc = distScale(cur, poc1, cur, poc0);
        if (sh->refLT[0][r0] || sh->refLT[1][r1]) {
          if ((poc1 - cur) * (poc0 - cur) > 0) t1 = t0;
          else t1 = Mv(-t0.h, -t0.v);
        } else t1 = scaleMv(t0, sc);
      }
      puInterDir[pi] = 3;
      puMv[0][pi] = m.mmvdBase[base][0].mv + t0; puRef[0][pi] = r0;
      puMv[1][pi] = m.mmvdBase[base][1].mv + t1; puRef[1][pi] = r1;
    } else if (r0 != -1) {
      t0 = dirMv(posn);
      puInterDir[pi] = 1;
      puMv[0][pi] = m.mmvdBase[base][0].mv + t0; puRef[0][pi] = r0;
      puMv[1][pi] = Mv(); puRef[1][pi] = -1;
    } else if (r1 != -1) {
      t1 = dirMv(posn);
      puInterDir[pi] = 2;
      puMv[0][pi] = Mv(); puRef[0][pi] = -1;
      puMv[1][pi] = m.mmvdBase[base][1].mv + t1; puRef[1][pi] = r1;
    }
    S.pu[pi].mergeidx = candIdx;
    puMrgType[pi] = MRG_DEFAULT;
    cuImv[ci] = m.mmvdAltHpel[base] ? IMV_HPEL : 0;
    cuBcw[ci] = m.interDir[base] == 3 ? m.bcw[base] : BCW_DEFAULT;
    for (int l = 0; l < 2; l++)
      if (puRef[l][pi] >= 0) puMv[l][pi] = clipStore(puMv[l][pi]);
    restrictBiOne(ci);
  }

  void run() {
    static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;   // diagnostics: phase times to stderr
    auto tp = std::chrono::steady_clock::now();
    auto mark = [&](const char *n) {
      if (!prof) return;
      const auto t = std::chrono::steady_clock::now();
      fprintf(stderr, "  derive %-8s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t - tp).count());
      tp = t;
    };
    const size_t ncu = S.cu.size(), npu = S.pu.size();
    cuImv.assign(ncu, 0); cuBcw.assign(ncu, BCW_DEFAULT); cuAffType.assign(ncu, 0);
    for (int l = 0; l < 2; l++) {
      puMv[l].assign(npu, Mv()); puRef[l].assign(npu, -1);
      for (int k = 0; k < 3; k++) puAff[l][k].assign(npu, Mv());
    }
    puInterDir.assign(npu, 255); puMrgType.assign(npu, MRG_DEFAULT);
    for (size_t i = 0; i < ncu; i++) {
      cuImv[i] = S.cu[i].imv; cuBcw[i] = S.cu[i].bcw; cuAffType[i] = S.cu[i].affinetype;
      const int pi = S.cu[i].firstpu;
      if (pi >= 0) {
        puInterDir[pi] = S.pu[pi].interdir;
        puRef[0][pi] = S.pu[pi].ref0; puRef[1][pi] = S.pu[pi].ref1;
      }
    }
    mark("arrays");
    // CodingStructure::initStructData memsets the field; here only the units that no span writes are
    // zeroed, those of intra CUs (span and spanParse write every byte of an inter CU's units, the affine
    // ones included: setAllAffineMv the MVs of the lists in use, the span the rest). The luma CUs tile
    // the picture.
    mf.alloc((size_t)S.w4 * S.h4, false);
    for (size_t i = 0; i < ncu; i++) {
      const vvcr_cu &c = S.cu[i];
      if (!c.yvalid || c.predmode != MODE_INTRA) continue;
      for (int y = c.y >> 2; y < (c.y + c.h) >> 2; y++) std::memset((void *)&mf[(size_t)y * S.w4 + (c.x >> 2)], 0, (size_t)(c.w >> 2) * sizeof(Mi));
      col8(c);
    }
    mark("field");
    int curSlice = -1;
    for (size_t i = 0; i < ncu; i++) {
      const vvcr_cu &c = S.cu[i];
      if (S.cux[i].slice != curSlice) {
        curSlice = S.cux[i].slice;
        sh = &P.slices[curSlice];
        sliceIdx = curSlice;
        col = nullptr;
        if (!sh->isIntra() && ph.tmvp) {
          const int cl = sh->isInterB() ? (sh->colFromL0 ? 0 : 1) : 0;
          const int poc = sh->refPoc[cl][sh->colRefIdx];
          for (const MotionPicture *mp : dpb)
            if (mp && mp->poc == poc) col = mp;
          VVCP_CHECK(!col, "collocated picture not decoded");
        }
      }
      if (S.cux[i].hmvpReset) lut.clear();
      if (c.predmode == MODE_INTRA || !c.yvalid) continue;
      deriveCu((int)i);
    }
    mark("cus");
    // write the derived fields back into the rows
    for (size_t i = 0; i < ncu; i++) {
      vvcr_cu &c = S.cu[i];
      if (c.predmode == MODE_INTRA || !c.yvalid) continue;
      c.imv = cuImv[i]; c.bcw = cuBcw[i]; c.affinetype = cuAffType[i];
      const int pi = c.firstpu;
      vvcr_pu &u = S.pu[pi];
      u.interdir = puInterDir[pi];
      u.mv0x = puMv[0][pi].h; u.mv0y = puMv[0][pi].v; u.mv1x = puMv[1][pi].h; u.mv1y = puMv[1][pi].v;
      u.ref0 = puRef[0][pi]; u.ref1 = puRef[1][pi];
      u.mrgtype = puMrgType[pi];
      for (int l = 0; l < 2; l++)
        for (int k = 0; k < 3; k++) { u.aff[(l * 3 + k) * 2] = puAff[l][k][pi].h; u.aff[(l * 3 + k) * 2 + 1] = puAff[l][k][pi].v; }
      // decoder-side refinement decisions (InterPrediction.cpp:1584-1635, PU::checkDMVRCondition :1249)
      u.dmvr = 0; u.bdof = 0;
      if (u.interdir == 3 && !c.geo) {
        const SliceHeader &s = P.slices[S.cux[i].slice];
        const SliceHeader *keep = sh;
        sh = &s;
        bool wp = false;
        for (int k = 0; k < 3; k++) wp |= s.wp[0][u.ref0][k][0] || s.wp[1][u.ref1][k][0];
        const bool eq = isBiPredDiffDirEqDist(pi);
        if (sps.dmvr && !ph.disDmvr)
          u.dmvr = u.merge && u.mrgtype == MRG_DEFAULT && !u.ciip && !c.affine && !u.mmvd && !c.mmvdskip && eq && c.h >= 8 && c.w >= 8 &&
                   c.h * c.w >= 128 && c.bcw == BCW_DEFAULT && !wp;
        if (sps.bdof && !ph.disBdof && !c.affine && u.mrgtype == MRG_DEFAULT) {
          const bool c0 = !(wp && s.isInterB());
          const bool c1 = !(P.pps.useWP && s.isInterP());
          bool b = c0 && c1 && eq && c.h >= 8 && c.w >= 8 && c.h * c.w >= 128;
          if (u.ciip || c.smvd || (sps.bcw && c.bcw != BCW_DEFAULT)) b = false;
          u.bdof = b;
        }
        sh = keep;
      }
    }
    int off = 0;
    for (vvcr_pu &u : S.pu) {
      if (u.dmvr) {
        u.dmvr_off = off;
        const int dy = std::min(u.h, 16), dx = std::min(u.w, 16);
        off += (u.h / dy) * (u.w / dx);
      } else u.dmvr_off = -1;
    }
    mark("back");
  }
};

}  // namespace

void derive_motion(PictureUnit &p, const std::vector<const MotionPicture *> &dpb, MotionField &field,
                   MotionRows &motionRows, std::vector<vvcr_geo> &geoRows) {
  geoRows.clear();
  bool intra = true;
  for (const SliceHeader &s : p.slices) intra &= s.isIntra();
  if (intra) {   // no inter CU: no field and no rows (all-zero, CodingStructure::initStructData; nothing reads them)
    field.reset();
    motionRows.clear();
    return;
  }
  static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;   // diagnostics: phase times to stderr
  auto tp = std::chrono::steady_clock::now();
  auto mark = [&](const char *n) {
    if (!prof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "  derive %-8s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t - tp).count());
    tp = t;
  };
  // the field itself becomes the motion rows (Mi has the layout of a MotionRec); `field` gets the
  // collocated view, the top-left 4x4 unit of every 8x8 block (MotionPicture), as each CU's span is final
  MotionField full;
  Deriver d(p, full, geoRows, dpb);
  d.w8 = (p.syn.w4 + 1) >> 1;
  field.alloc((size_t)d.w8 * ((p.syn.h4 + 1) >> 1), false);
  d.col8f = &field;
  mark("init");
  d.run();
  mark("run");
  // a picture parsed in part (vvcp_set_parse_rows): the rows outside it hold no CU; zero them as
  // CodingStructure::initStructData would (never read for this shard, but defined)
  const int lg = p.sps.ctuLog2;
  const int u0 = std::min(p.syn.h4, (p.parseR0 << lg) >> 2), u1 = std::min(p.syn.h4, (int)std::min<int64_t>((int64_t)p.parseR1 << lg, 1 << 30) >> 2);
  if (u0 > 0 || u1 < p.syn.h4) {
    const size_t w4 = (size_t)p.syn.w4, w8 = (size_t)d.w8, h8 = (size_t)(p.syn.h4 + 1) >> 1;
    std::memset((void *)&full[0], 0, (size_t)u0 * w4 * sizeof(Mi));
    if (u1 < p.syn.h4) std::memset((void *)&full[(size_t)u1 * w4], 0, (size_t)(p.syn.h4 - u1) * w4 * sizeof(Mi));
    const size_t e0 = std::min<size_t>(h8, (size_t)u0 >> 1), e1 = std::min<size_t>(h8, ((size_t)u1 + 1) >> 1);
    std::memset((void *)&field[0], 0, e0 * w8 * sizeof(Mi));
    if (e1 < h8) std::memset((void *)&field[e1 * w8], 0, (h8 - e1) * w8 * sizeof(Mi));
  }
  motionRows.adopt(std::move(full));
}

void refine_motion(const PictureUnit &p, MotionField &&field, const int32_t *deltas, int64_t ndeltas,
                   MotionPicture &out) {
  const PictureSyntax &S = p.syn;
  out.poc = p.poc;
  out.w4 = S.w4;
  out.h4 = S.h4;
  out.w8 = (S.w4 + 1) >> 1;
  out.h8 = (S.h4 + 1) >> 1;
  out.intra = field.empty();
  out.mf = std::move(field);
  out.slices.resize(p.slices.size());
  for (size_t s = 0; s < p.slices.size(); s++)
    for (int l = 0; l < 2; l++)
      for (int r = 0; r < VVCR_MAX_REF; r++) { out.slices[s].refPoc[l][r] = p.slices[s].refPoc[l][r]; out.slices[s].refLT[l][r] = p.slices[s].refLT[l][r]; }
  for (const vvcr_pu &u : S.pu) {
    if (!u.dmvr) continue;
    const vvcr_cu &c = S.cu[u.cu];
    const int dy = std::min(u.h, 16), dx = std::min(u.w, 16);
    int num = 0;
    for (int y = u.y; y < u.y + u.h; y += dy)
      for (int x = u.x; x < u.x + u.w; x += dx, num++) {
        const int64_t k = (int64_t)u.dmvr_off + num;
        VVCP_CHECK(!deltas || k >= ndeltas, "DMVR deltas missing");
        const int ddx = deltas[2 * k], ddy = deltas[2 * k + 1];
        Mi mi;
        mi.isInter = true;
        mi.slice = (uint16_t)S.cux[u.cu].slice;
        mi.interDir = (int8_t)u.interdir;
        mi.altHpel = c.imv == IMV_HPEL;
        mi.ref[0] = (int16_t)u.ref0; mi.ref[1] = (int16_t)u.ref1;
        mi.mv[0][0] = clipStore(u.mv0x + ddx); mi.mv[0][1] = clipStore(u.mv0y + ddy);
        mi.mv[1][0] = clipStore(u.mv1x - ddx); mi.mv[1][1] = clipStore(u.mv1y - ddy);
        // the kept units inside the sub-block: 8-aligned positions (a CU may start at x or y = 4 mod 8)
        for (int yy = (y + 7) & ~7; yy < y + dy; yy += 8)
          for (int xx = (x + 7) & ~7; xx < x + dx; xx += 8) out.mf[(size_t)(yy >> 3) * out.w8 + (xx >> 3)] = colMi(mi);
      }
  }
}

}  // namespace vvcp
