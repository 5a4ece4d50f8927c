// vvcp_ctu.cpp — CABAC slice-data parser of the host parser (see vvcp_ctu.h). Each function cites the
// reference function whose decisions it restates; the data model is flat (rows + 4x4 maps) instead of
// the reference's CodingStructure objects.
#include "vvcp_ctu.h"
#include "vvcr_tables.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

namespace vvcp {
namespace {

using namespace vvcp_ctx;

enum { MODE_INTER = 0, MODE_INTRA = 1, MODE_IBC = 2, MODE_PLT = 3 };
enum { TREE_D = 0, TREE_L = 1, TREE_C = 2 };
enum { MT_ALL = 0, MT_INTER = 1, MT_INTRA = 2 };
// PartSplit (UnitPartitioner.h:56)
enum {
  CTU_LEVEL = 0, S_QT = 1, S_BH = 2, S_BV = 3, S_TH = 4, S_TV = 5, TU_MAX = 6, TU_NO_ISP = 7, ISP_H = 8, ISP_V = 9,
  SBT_VH0 = 10, SBT_VH1, SBT_HH0, SBT_HH1, SBT_VQ0, SBT_VQ1, SBT_HQ0, SBT_HQ1, S_DONT = 2000
};
enum { SBT_OFF = 0, SBT_VER_HALF = 1, SBT_HOR_HALF = 2, SBT_VER_QUAD = 3, SBT_HOR_QUAD = 4 };
constexpr int PLANAR = 0, DC = 1, HOR = 18, VER = 50, VDIA = 66, LM = 67, MDLM_L = 68, MDLM_T = 69, DM = 70;
constexpr int MTS_DCT2 = 0, MTS_SKIP = 1, MTS_DST7 = 2;
constexpr int BCW_DEFAULT = 2;

// ------------------------------------------------------------------------------------------------
// Scan orders (Rom.cpp:252-380 initROM, ScanGenerator :91)
// ------------------------------------------------------------------------------------------------
struct ScanPos { uint16_t idx; uint8_t x, y; };

struct DiagGen {   // ScanGenerator, SCAN_DIAG
  int w, h, line = 0, col = 0;
  DiagGen(int w_, int h_) : w(w_), h(h_) {}
  void next() {
    if (col == w - 1 || line == 0) {
      line += col + 1;
      col = 0;
      if (line >= h) { col += line - (h - 1); line = h - 1; }
    } else { col++; line--; }
  }
};

// The regular residual path decodes levels into a padded block: row stride kPS, and the two columns
// right of a 64-wide block and the two rows below any block stay zero, so the context templates
// (CoeffCodingContext::sigCtxIdAbs / templateAbsSum, ContextModelling.h:105-190) read their five
// neighbours without bounds tests (the zeros are exactly the reference's "outside the block").
constexpr int kPS = 66;
struct Scans {
  std::vector<ScanPos> grouped[7][7], plain[7][7];
  std::vector<uint16_t> groupedInv[7][7];   // raster index -> first grouped scan position holding it
  std::vector<uint16_t> groupedP[7][7];     // grouped scan position -> index in the padded block
  Scans() {
    for (int lw = 0; lw < 7; lw++)
      for (int lh = 0; lh < 7; lh++) {
        const int w = 1 << lw, h = 1 << lh;
        std::vector<ScanPos> &p = plain[lw][lh];
        p.resize(w * h);
        DiagGen g(w, h);
        for (int i = 0; i < w * h; i++) { p[i] = {(uint16_t)(g.line * w + g.col), (uint8_t)g.col, (uint8_t)g.line}; g.next(); }
        const int sw = kLog2SbbSize[lw][lh][0], sh = kLog2SbbSize[lw][lh][1];
        const int gw = 1 << sw, gh = 1 << sh;
        const int wg = std::min(32, w) >> sw, hg = std::min(32, h) >> sh;
        std::vector<ScanPos> &s = grouped[lw][lh];
        s.assign(w * h, ScanPos{(uint16_t)(w * h - 1), (uint8_t)(w - 1), (uint8_t)(h - 1)});
        DiagGen gg(wg, hg);
        for (int gi = 0; gi < wg * hg; gi++) {
          const int ox = gg.col * gw, oy = gg.line * gh;
          DiagGen in(gw, gh);
          for (int k = 0; k < gw * gh; k++) {
            const int x = in.col + ox, y = in.line + oy;
            s[gi * gw * gh + k] = {(uint16_t)(y * w + x), (uint8_t)x, (uint8_t)y};
            in.next();
          }
          gg.next();
        }
        std::vector<uint16_t> &inv = groupedInv[lw][lh];
        inv.assign(w * h, (uint16_t)(w * h - 1));
        for (int sp = w * h - 2; sp >= 0; sp--) inv[s[sp].idx] = (uint16_t)sp;
        std::vector<uint16_t> &pp = groupedP[lw][lh];
        pp.resize(w * h);
        for (int sp = 0; sp < w * h; sp++) pp[sp] = (uint16_t)(s[sp].y * kPS + s[sp].x);
      }
  }
};
const Scans &scans() { static Scans s; return s; }

const uint32_t kGroupIdx[64] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9,
                                10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10,
                                11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11, 11};
const uint32_t kMinInGroup[14] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96};
const uint32_t kGoRiceParsCoeff[32] = {0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3};
const int kBcwParsingOrder[5] = {2, 3, 1, 4, 0};   // resetBcwCodingOrder (Rom.cpp:202)

inline int tbMax(uint32_t v) { return floorLog2(v); }   // g_tbMax (Rom.h:195) for v <= 256

// ------------------------------------------------------------------------------------------------
// Coefficient coding context (ContextModelling.h:51 CoeffCodingContext)
// ------------------------------------------------------------------------------------------------
struct CoefCtx {
  int ch, comp, w, h, log2w, log2CGw, log2CGh, log2CG, wg, hg, maxNumCoeff;
  bool signHiding, bdpcm;
  const ScanPos *scan, *scanCG;
  const uint16_t *scanInv, *pscan;
  int lastX, lastY, lastOffX = 0, lastOffY = 0, lastShX = 0, lastShY = 0;
  unsigned maxLastPosX, maxLastPosY;
  int scanPosLast = -1, subSetId = -1, subSetPos = -1, subSetPosX = -1, subSetPosY = -1, minSubPos = -1, maxSubPos = -1;
  unsigned sigGroupCtx = 0, sigGroupCtxTS = 0;
  int tmplCpSum1 = -1, tmplCpDiag = -1;
  uint64_t sigCG = 0;
  int regBinLimit = 0, numCtxBins = 0;
  unsigned sigSet[3], parSet, gtxSet[2];

  CoefCtx(int comp_, int w_, int h_, bool sh, bool bd) : comp(comp_), w(w_), h(h_), signHiding(sh), bdpcm(bd) {
    ch = comp ? 1 : 0;
    const int lw = floorLog2(w), lh = floorLog2(h);
    log2w = lw;
    log2CGw = kLog2SbbSize[lw][lh][0];
    log2CGh = kLog2SbbSize[lw][lh][1];
    log2CG = log2CGw + log2CGh;
    wg = std::min(32, w) >> log2CGw;
    hg = std::min(32, h) >> log2CGh;
    maxNumCoeff = w * h;
    scan = scans().grouped[lw][lh].data();
    scanInv = scans().groupedInv[lw][lh].data();
    pscan = scans().groupedP[lw][lh].data();
    scanCG = scans().plain[floorLog2(wg)][floorLog2(hg)].data();
    lastX = ch ? LastX1 : LastX0;
    lastY = ch ? LastY1 : LastY0;
    maxLastPosX = kGroupIdx[std::min(32, w) - 1];
    maxLastPosY = kGroupIdx[std::min(32, h) - 1];
    if (ch) {
      lastShX = clip3(0, 2, w >> 3);
      lastShY = clip3(0, 2, h >> 3);
    } else {
      static const int prefix[8] = {0, 0, 0, 3, 6, 10, 15, 21};
      lastOffX = prefix[lw]; lastOffY = prefix[lh];
      lastShX = (lw + 1) >> 2; lastShY = (lh + 1) >> 2;
    }
    static const unsigned sig[6] = {SigFlag0, SigFlag1, SigFlag2, SigFlag3, SigFlag4, SigFlag5};
    sigSet[0] = sig[ch]; sigSet[1] = sig[ch + 2]; sigSet[2] = sig[ch + 4];
    parSet = ch ? ParFlag1 : ParFlag0;
    static const unsigned gtx[4] = {GtxFlag0, GtxFlag1, GtxFlag2, GtxFlag3};
    gtxSet[0] = gtx[ch]; gtxSet[1] = gtx[ch + 2];
  }
  void initSubblock(int id) {
    subSetId = id;
    subSetPos = scanCG[id].idx;
    subSetPosY = subSetPos / wg;
    subSetPosX = subSetPos - subSetPosY * wg;
    minSubPos = id << log2CG;
    maxSubPos = minSubPos + (1 << log2CG) - 1;
    const unsigned sigRight = (subSetPosX + 1) < wg ? (sigCG >> (subSetPos + 1)) & 1 : 0;
    const unsigned sigLower = (subSetPosY + 1) < hg ? (sigCG >> (subSetPos + wg)) & 1 : 0;
    sigGroupCtx = (ch ? SigCoeffGroup1 : SigCoeffGroup0) + (sigRight | sigLower);
    const unsigned sigLeft = subSetPosX > 0 ? (sigCG >> (subSetPos - 1)) & 1 : 0;
    const unsigned sigAbove = subSetPosY > 0 ? (sigCG >> (subSetPos - wg)) & 1 : 0;
    sigGroupCtxTS = TsSigCoeffGroup + sigLeft + sigAbove;
  }
  void setSigGroup() { sigCG |= 1ull << subSetPos; }
  bool isLast() const { return (scanPosLast >> log2CG) == subSetId; }
  bool isSigGroup() const { return (sigCG >> subSetPos) & 1; }
  unsigned lastXCtx(unsigned p) const { return lastX + lastOffX + (p >> lastShX); }
  unsigned lastYCtx(unsigned p) const { return lastY + lastOffY + (p >> lastShY); }
  // (padded block, kPS: the neighbours outside the block read zeros)
  unsigned sigCtxIdAbs(int sp, const int32_t *coeff, int state) {
    const int diag = scan[sp].x + scan[sp].y;
    const int32_t *d = coeff + pscan[sp];
    int numPos = 0, sumAbs = 0;
    auto upd = [&](int32_t v) { const int a = std::abs(v); sumAbs += std::min(4 + (a & 1), a); numPos += !!a; };
    upd(d[1]);
    upd(d[2]);
    upd(d[kPS + 1]);
    upd(d[kPS]);
    upd(d[2 * kPS]);
    int ofs = std::min((sumAbs + 1) >> 1, 3) + (diag < 2 ? 4 : 0);
    if (ch == 0) ofs += diag < 5 ? 4 : 0;
    tmplCpDiag = diag;
    tmplCpSum1 = sumAbs - numPos;
    return sigSet[std::max(0, state - 1)] + ofs;
  }
  uint8_t ctxOffsetAbs() const {
    int off = 0;
    if (tmplCpDiag != -1) {
      off = std::min(tmplCpSum1, 4) + 1;
      off += !tmplCpDiag ? (ch == 0 ? 15 : 5) : (ch == 0 ? (tmplCpDiag < 3 ? 10 : (tmplCpDiag < 10 ? 5 : 0)) : 0);
    }
    return (uint8_t)off;
  }
  unsigned templateAbsSum(int sp, const int32_t *coeff, int base) const {   // (padded block)
    const int32_t *d = coeff + pscan[sp];
    const int sum = std::abs(d[1]) + std::abs(d[2]) + std::abs(d[kPS + 1]) + std::abs(d[kPS]) + std::abs(d[2 * kPS]);
    return (unsigned)std::max(std::min(sum - 5 * base, 31), 0);
  }
  unsigned sigCtxIdAbsTS(int sp, const int32_t *coeff) const {
    const int py = scan[sp].y, px = scan[sp].x;
    const int32_t *c = coeff + px + py * w;
    int n = 0;
    if (px > 0) n += !!c[-1];
    if (py > 0) n += !!c[-w];
    return TsSigFlag + n;
  }
  unsigned lrg1CtxIdAbsTS(int sp, const int32_t *coeff) const {
    const int py = scan[sp].y, px = scan[sp].x;
    const int32_t *c = coeff + px + py * w;
    int n = 0;
    if (bdpcm) n = 3;
    else {
      if (px > 0) n += !!c[-1];
      if (py > 0) n += !!c[-w];
    }
    return TsLrg1Flag + n;
  }
  unsigned signCtxIdAbsTS(int sp, const int32_t *coeff) const {
    const int py = scan[sp].y, px = scan[sp].x;
    const int32_t *d = coeff + px + py * w;
    int r = 0, b = 0;
    if (px > 0) r = d[-1];
    if (py > 0) b = d[-w];
    unsigned c;
    if ((r == 0 && b == 0) || (r * b) < 0) c = 0;
    else if (r >= 0 && b >= 0) c = 1;
    else c = 2;
    if (bdpcm) c += 3;
    return TsResidualSign + c;
  }
  void neighTS(int &r, int &b, int sp, const int32_t *coeff) const {
    const int py = scan[sp].y, px = scan[sp].x;
    const int32_t *d = coeff + px + py * w;
    r = b = 0;
    if (px > 0) r = d[-1];
    if (py > 0) b = d[-w];
  }
  static int decDeriveModCoeff(int r, int b, int a) {
    if (a == 0) return 0;
    const int pred1 = std::max(std::abs(b), std::abs(r));
    if (a == 1 && pred1 > 0) return pred1;
    return a - (a <= pred1);
  }
};

// ------------------------------------------------------------------------------------------------
// Partitioner (UnitPartitioner.cpp QTBTPartitioner / TUIntraSubPartitioner): luma-coordinate areas;
// in 4:2:0 without noChroma2x2 the chroma block of every partition is the luma block halved.
// ------------------------------------------------------------------------------------------------
struct Area { int x = 0, y = 0, w = 0, h = 0; bool cvalid = true; };

// the sub-partitions of one split (at most four): inline, no heap allocation per split
struct Parts {
  Area a[4];
  int n = 0;
  void push_back(const Area &x) { a[n++] = x; }
  size_t size() const { return (size_t)n; }
  const Area &operator[](int i) const { return a[i]; }
};

struct Level {
  int split = CTU_LEVEL;
  Parts parts;
  int idx = 0;
  bool checked = false, isImplicit = false;
  int implicitSplit = S_DONT;
  bool canQtSplit = true, qgEnable = true, qgChromaEnable = true;
  int modeType = MT_ALL;
};

struct Parser;

struct Partitioner {
  std::vector<Level> st;
  int depth = 0, trDepth = 0, btDepth = 0, mtDepth = 0, qtDepth = 0, subdiv = 0, implicitBtDepth = 0;
  int chType = 0, treeType = TREE_D, modeType = MT_ALL;
  const Area &area() const { return st.back().parts[st.back().idx]; }
  int partIdx() const { return st.back().idx; }
  bool qgEnable() const { return st.back().qgEnable; }
  bool qgChromaEnable() const { return st.back().qgChromaEnable; }
  void initCtu(const Area &a, int ch) {
    depth = trDepth = btDepth = mtDepth = qtDepth = subdiv = implicitBtDepth = 0;
    chType = ch;
    st.clear();
    Level l;
    l.parts.push_back(a);
    st.push_back(l);
    treeType = TREE_D;
    modeType = MT_ALL;
  }
  uint64_t splitSeries() const {
    uint64_t s = 0;
    int d = 0;
    for (const Level &l : st) {
      if (l.split == CTU_LEVEL) continue;
      s += (uint64_t)l.split << (d * 5);
      d++;
    }
    return s;
  }
};

inline int splitAtDepth(uint64_t series, int cuDepth, int d) {   // CU::getSplitAtDepth (UnitTools.cpp:269)
  if (d >= cuDepth) return S_DONT;
  return (int)((series >> (d * 5)) & 31);
}

struct CuCtx {   // CUCtx (ContextModelling.h:409)
  bool isDQPCoded = false, isChromaQpAdjCoded = false, qgStart = false, lfnstLastScanPos = false;
  int qp = 0;
  bool violatesLfnst[2] = {false, false};
  bool violatesMtsCoeffConstraint = false, mtsLastScanPos = false;
};

// ------------------------------------------------------------------------------------------------
// The per-slice parser
// ------------------------------------------------------------------------------------------------
struct Parser {
  PictureSyntax &pic;           // rows (CU / PU / TU, levels): the picture's, or a tile unit's own (parse_picture_data)
  PictureSyntax &shp;           // the picture: maps, per-CTB loop-filter syntax, geometry
  const SliceCtx &sc;
  const SPS &sps;
  const PPS &pps;
  const PicHeader &ph;
  const SliceHeader &sh;
  Cabac cab;
  bool dualTree = false;        // CS::isDualITree: I slice with the SPS dual tree
  int chromaQpAdj = 0;          // cs.chromaQpAdj
  int curTile = 0;
  int curCtu = 0;
  bool firstCuOfCtu = false, ctuHmvpReset = false;
  int minQT[3], maxBTD[3], maxBT[3], maxTT[3];
  int log2MaxTb, maxTb;
  int cuQpDeltaSubdiv, cuChromaQpOffsetSubdiv;

  Parser(PictureSyntax &rows, PictureSyntax &shared, const SliceCtx &s)
      : pic(rows), shp(shared), sc(s), sps(*s.sps), pps(*s.pps), ph(*s.ph), sh(*s.sh) {
    dualTree = sh.isIntra() && sps.dualTree;
    for (int k = 0; k < 3; k++) { minQT[k] = ph.minQT[k]; maxBTD[k] = ph.maxBTD[k]; maxBT[k] = ph.maxBT[k]; maxTT[k] = ph.maxTT[k]; }
    log2MaxTb = sps.log2MaxTb;
    maxTb = 1 << log2MaxTb;
    cuQpDeltaSubdiv = sh.isIntra() ? ph.cuQpDeltaSubdivIntra : ph.cuQpDeltaSubdivInter;
    cuChromaQpOffsetSubdiv = sh.isIntra() ? ph.cuChromaQpOffsetSubdivIntra : ph.cuChromaQpOffsetSubdivInter;
  }

  // PreCalcValues::getValIdx (Slice.cpp:3224): [I luma, inter, I chroma]
  int valIdx(int ch) const { return sh.isIntra() ? (!sps.dualTree ? 0 : (ch << 1)) : 1; }
  int minBtSize() const { return 1 << sps.log2MinCb; }

  // ---- maps ----
  int cuAt(int ch, int x, int y) const { return shp.cuAt(ch, x, y); }
  // CodingStructure::getCURestricted (CodingStructure.cpp:1519/1539): same slice and tile. The tile is
  // checked by position before the map is read: another tile's entries may belong to another unit's rows.
  int cuRestricted(int ch, int x, int y, int slice, int tile) const {
    const int lx = ch ? x << 1 : x, ly = ch ? y << 1 : y;
    if (lx < 0 || ly < 0 || lx >= shp.W || ly >= shp.H || tileOf(lx, ly) != tile) return -1;
    const int c = cuAt(ch, x, y);
    if (c < 0) return -1;
    return pic.cux[c].slice == slice ? c : -1;
  }
  int tileOf(int lx, int ly) const {
    return pps.tileIdx(lx >> pic.ctuLog2, ly >> pic.ctuLog2);
  }
  void fill_map(int ch, int cuIdx, int lx, int ly, int lw, int lh) {
    const int x0 = lx >> 2, y0 = ly >> 2;
    const int x1 = std::min(pic.w4, (lx + lw + 3) >> 2), y1 = std::min(pic.h4, (ly + lh + 3) >> 2);
    for (int y = y0; y < y1; y++)
      for (int x = x0; x < x1; x++) shp.map[ch][(size_t)y * pic.w4 + x] = cuIdx;
  }

  // ------------------------------------------------------------------------------------------------
  // QTBTPartitioner::canSplit (UnitPartitioner.cpp:361), getImplicitSplit (:508)
  // ------------------------------------------------------------------------------------------------
  int implicitSplit(Partitioner &p) {
    Level &lv = p.st.back();
    if (lv.checked) return lv.implicitSplit;
    const Area &a = p.area();
    int split = S_DONT;
    const bool isBlInPic = a.x < pic.W && a.y + a.h - 1 < pic.H;
    const bool isTrInPic = a.x + a.w - 1 < pic.W && a.y < pic.H;
    const int vi = valIdx(p.chType);
    const bool isBtAllowed = a.w <= maxBT[vi] && a.h <= maxBT[vi];
    const bool isQtAllowed = a.w > minQT[vi] && a.h > minQT[vi] && p.btDepth == 0;
    if (!isBlInPic && !isTrInPic && isQtAllowed) split = S_QT;
    else if (!isBlInPic && isBtAllowed) split = S_BH;
    else if (!isTrInPic && isBtAllowed) split = S_BV;
    else if (!isBlInPic || !isTrInPic) split = S_QT;
    if (dualTree && (a.w > 64 || a.h > 64)) split = S_QT;
    if ((!isBlInPic || !isTrInPic) && (a.w > 64 || a.h > 64)) split = S_QT;
    lv.checked = true;
    lv.isImplicit = split != S_DONT;
    lv.implicitSplit = split;
    return split;
  }
  void canSplit(Partitioner &p, bool &canNo, bool &canQt, bool &canBh, bool &canBv, bool &canTh, bool &canTv) {
    const int impl = implicitSplit(p);
    const int vi = valIdx(p.chType);
    const int maxBtd = maxBTD[vi] + p.implicitBtDepth;
    const int maxBtSize = maxBT[vi], minBt = minBtSize(), maxTtSize = maxTT[vi], minTt = minBtSize(), minQtSize = minQT[vi];
    canNo = canQt = canBh = canTh = canBv = canTv = true;
    bool canBtt = p.mtDepth < maxBtd;
    const Area &a = p.area();
    const int cw = a.w >> 1, ch = a.h >> 1;
    const Level &lv = p.st.back();
    const int lastSplit = lv.split;
    const int parlSplit = lastSplit == S_TH ? S_BH : S_BV;
    if (lastSplit != CTU_LEVEL && lastSplit != S_QT) canQt = false;
    if (a.w <= minQtSize) canQt = false;
    if (p.chType == 1 && cw <= 4) canQt = false;
    if (p.treeType == TREE_C) { canQt = canBh = canTh = canBv = canTv = false; return; }
    if (impl != S_DONT) {
      canNo = canTh = canTv = false;
      canBh = impl == S_BH;
      canBv = impl == S_BV;
      if (p.chType == 1 && cw == 4) canBv = false;
      return;
    }
    if ((lastSplit == S_TH || lastSplit == S_TV) && p.partIdx() == 1) {
      canBh = parlSplit != S_BH;
      canBv = parlSplit != S_BV;
    }
    if (canBtt && (a.w <= minBt && a.h <= minBt) && (a.w <= minTt && a.h <= minTt)) canBtt = false;
    if (canBtt && (a.w > maxBtSize || a.h > maxBtSize) && (a.w > maxTtSize || a.h > maxTtSize)) canBtt = false;
    if (!canBtt) { canBh = canTh = canBv = canTv = false; return; }
    if (a.w > maxBtSize || a.h > maxBtSize) canBh = canBv = false;
    if (a.h <= minBt) canBh = false;
    if (a.w > 64 && a.h <= 64) canBh = false;
    if (p.chType == 1 && cw * ch <= 16) canBh = false;
    if (a.w <= minBt) canBv = false;
    if (a.w <= 64 && a.h > 64) canBv = false;
    if (p.chType == 1 && (cw * ch <= 16 || cw == 4)) canBv = false;
    if (p.modeType == MT_INTER && a.w * a.h == 32) canBv = canBh = false;
    if (a.h <= 2 * minTt || a.h > maxTtSize || a.w > maxTtSize) canTh = false;
    if (a.w > 64 || a.h > 64) canTh = false;
    if (p.chType == 1 && cw * ch <= 32) canTh = false;
    if (a.w <= 2 * minTt || a.w > maxTtSize || a.h > maxTtSize) canTv = false;
    if (a.w > 64 || a.h > 64) canTv = false;
    if (p.chType == 1 && (cw * ch <= 32 || cw == 8)) canTv = false;
    if (p.modeType == MT_INTER && a.w * a.h == 64) canTv = canTh = false;
  }
  bool canSplitMode(Partitioner &p, int split) {
    bool n, q, bh, bv, th, tv;
    canSplit(p, n, q, bh, bv, th, tv);
    switch (split) {
      case S_QT: return q;
      case S_DONT: return n;
      case S_BH: return bh;
      case S_BV: return bv;
      case S_TH: return th;
      case S_TV: return tv;
    }
    return false;
  }
  // PartitionerImpl::getCUSubPartitions (UnitPartitioner.cpp:763)
  static Parts subParts(const Area &a, int split) {
    Parts r;
    switch (split) {
      case S_QT:
        for (int i = 0; i < 4; i++) r.push_back({a.x + (i & 1) * (a.w >> 1), a.y + (i >> 1) * (a.h >> 1), a.w >> 1, a.h >> 1, true});
        break;
      case S_BH: r.push_back({a.x, a.y, a.w, a.h >> 1, true}); r.push_back({a.x, a.y + (a.h >> 1), a.w, a.h >> 1, true}); break;
      case S_BV: r.push_back({a.x, a.y, a.w >> 1, a.h, true}); r.push_back({a.x + (a.w >> 1), a.y, a.w >> 1, a.h, true}); break;
      case S_TH:
        r.push_back({a.x, a.y, a.w, a.h >> 2, true});
        r.push_back({a.x, a.y + (a.h >> 2), a.w, a.h >> 1, true});
        r.push_back({a.x, a.y + 3 * (a.h >> 2), a.w, a.h >> 2, true});
        break;
      case S_TV:
        r.push_back({a.x, a.y, a.w >> 2, a.h, true});
        r.push_back({a.x + (a.w >> 2), a.y, a.w >> 1, a.h, true});
        r.push_back({a.x + 3 * (a.w >> 2), a.y, a.w >> 2, a.h, true});
        break;
    }
    return r;
  }
  // QTBTPartitioner::splitCurrArea (UnitPartitioner.cpp:266) for CU splits
  void splitCU(Partitioner &p, int split) {
    const bool isImpl = implicitSplit(p) == split;
    const bool canQt = canSplitMode(p, S_QT);
    bool qgEn = p.qgEnable(), qgcEn = p.qgChromaEnable();
    Level l;
    l.split = split;
    l.parts = subParts(p.area(), split);
    l.modeType = p.modeType;
    p.st.push_back(l);
    p.depth++;
    p.subdiv++;
    p.trDepth = 0;
    if (split != S_QT) {
      p.btDepth++;
      if (isImpl) p.implicitBtDepth++;
      p.mtDepth++;
      if (split == S_TH || split == S_TV) { p.btDepth++; p.subdiv++; }
      p.st.back().canQtSplit = canQt;
    } else {
      p.mtDepth = 0;
      p.btDepth = 0;
      p.qtDepth++;
      p.subdiv++;
    }
    qgEn &= p.subdiv <= cuQpDeltaSubdiv;
    qgcEn &= p.subdiv <= cuChromaQpOffsetSubdiv;
    p.st.back().qgEnable = qgEn;
    p.st.back().qgChromaEnable = qgcEn;
  }
  // QTBTPartitioner::nextPart (:614)
  bool nextPart(Partitioner &p) {
    Level &lv = p.st.back();
    const int idx = ++lv.idx;
    lv.checked = false;
    lv.isImplicit = false;
    if (idx < (int)lv.parts.size()) {
      if (lv.split == S_TH || lv.split == S_TV) {
        if (idx == 1) { p.btDepth--; p.subdiv--; }
        else { p.btDepth++; p.subdiv++; }
      }
      return true;
    }
    return false;
  }
  // QTBTPartitioner::exitCurrSplit (:561)
  void exitSplit(Partitioner &p) {
    const int split = p.st.back().split;
    const int idx = p.st.back().idx;
    p.st.pop_back();
    p.depth--;
    p.subdiv--;
    if (split == S_BH || split == S_BV || split == S_TH || split == S_TV) {
      p.mtDepth--;
      if (p.st.back().isImplicit) p.implicitBtDepth--;
      p.btDepth--;
      if ((split == S_TH || split == S_TV) && idx != 1) { p.btDepth--; p.subdiv--; }
    } else if (split == S_QT) {
      p.qtDepth--;
      p.subdiv--;
    }
  }

  // ------------------------------------------------------------------------------------------------
  // DeriveCtx::CtxSplit (ContextModelling.cpp:150) + CABACReader::split_cu_mode (CABACReader.cpp:726)
  // ------------------------------------------------------------------------------------------------
  int split_cu_mode(Partitioner &p) {
    bool canNo, canQt, canBh, canBv, canTh, canTv;
    canSplit(p, canNo, canQt, canBh, canBv, canTh, canTv);
    const Area &a = p.area();
    const int sx = p.chType ? a.x >> 1 : a.x, sy = p.chType ? a.y >> 1 : a.y;
    const int cw = p.chType ? a.w >> 1 : a.w, chh = p.chType ? a.h >> 1 : a.h;
    const int tile = tileOf(a.x, a.y);
    const int cl = cuRestricted(p.chType, sx - 1, sy, sc.sliceIdx, tile);
    const int ca = cuRestricted(p.chType, sx, sy - 1, sc.sliceIdx, tile);
    auto blkW = [&](int c) { return p.chType ? pic.cu[c].cw : pic.cu[c].w; };
    auto blkH = [&](int c) { return p.chType ? pic.cu[c].ch : pic.cu[c].h; };
    unsigned ctxSpl = 0;
    if (cl >= 0) ctxSpl += blkH(cl) < chh ? 1 : 0;
    if (ca >= 0) ctxSpl += blkW(ca) < cw ? 1 : 0;
    unsigned numSplit = (canQt ? 2 : 0) + canBh + canBv + canTh + canTv;
    if (numSplit > 0) numSplit--;
    ctxSpl += 3 * (numSplit >> 1);
    unsigned ctxQt = (cl >= 0 && pic.cu[cl].qtdepth > p.qtDepth) ? 1 : 0;
    ctxQt += (ca >= 0 && pic.cu[ca].qtdepth > p.qtDepth) ? 1 : 0;
    ctxQt += p.qtDepth < 2 ? 0 : 3;
    unsigned ctxHv = 0;
    const unsigned numHor = canBh + canTh, numVer = canBv + canTv;
    if (numVer == numHor) {
      const int wA = ca >= 0 ? blkW(ca) : 1, hL = cl >= 0 ? blkH(cl) : 1;
      const int depA = cw / wA, depL = chh / hL;
      if (depA == depL || cl < 0 || ca < 0) ctxHv = 0;
      else if (depA < depL) ctxHv = 1;
      else ctxHv = 2;
    } else if (numVer < numHor) ctxHv = 3;
    else ctxHv = 4;
    const unsigned ctxHorBt = p.mtDepth <= 1 ? 1 : 0, ctxVerBt = p.mtDepth <= 1 ? 3 : 2;

    bool isSplit = canBh || canBv || canTh || canTv || canQt;
    if (canNo && isSplit) isSplit = cab.bin(SplitFlag + ctxSpl);
    if (!isSplit) return S_DONT;
    const bool canBtt = canBh || canBv || canTh || canTv;
    bool isQt = canQt;
    if (isQt && canBtt) isQt = cab.bin(SplitQtFlag + ctxQt);
    if (isQt) return S_QT;
    const bool canHor = canBh || canTh;
    bool isVer = canBv || canTv;
    if (isVer && canHor) isVer = cab.bin(SplitHvFlag + ctxHv);
    const bool can14 = isVer ? canTv : canTh;
    bool is12 = isVer ? canBv : canBh;
    if (is12 && can14) is12 = cab.bin(Split12Flag + (isVer ? ctxVerBt : ctxHorBt));
    if (isVer && is12) return S_BV;
    if (isVer) return S_TV;
    if (is12) return S_BH;
    return S_TH;
  }

  // CodingStructure::signalModeCons (CodingStructure.cpp:198) + CABACReader::mode_constraint (:705)
  int mode_constraint(Partitioner &p, int split) {
    if (dualTree || p.modeType != MT_ALL) return p.modeType;
    const Area &a = p.area();
    int minLumaArea = a.w * a.h;
    if (split == S_QT || split == S_TH || split == S_TV) minLumaArea >>= 2;
    else if (split == S_BV || split == S_BH) minLumaArea >>= 1;
    const int minChromaBlock = minLumaArea >> 2;
    const bool is2xN = ((a.w >> 1) == 4 && split == S_BV) || ((a.w >> 1) == 8 && split == S_TV);
    if (minChromaBlock >= 16 && !is2xN) return p.modeType;   // inherit
    if (minLumaArea < 32 || sh.isIntra()) return MT_INTRA;   // infer
    // signal: DeriveCtx::CtxModeConsFlag (ContextModelling.cpp:135)
    const int tile = tileOf(a.x, a.y);
    const int cl = cuRestricted(0, a.x - 1, a.y, sc.sliceIdx, tile);
    const int ca = cuRestricted(0, a.x, a.y - 1, sc.sliceIdx, tile);
    const unsigned ctx = ((ca >= 0 && pic.cu[ca].predmode == MODE_INTRA) || (cl >= 0 && pic.cu[cl].predmode == MODE_INTRA)) ? 1 : 0;
    return cab.bin(ModeConsFlag + ctx) ? MT_INTRA : MT_INTER;
  }

  // ------------------------------------------------------------------------------------------------
  // CABACReader::coding_tree (CABACReader.cpp:469)
  // ------------------------------------------------------------------------------------------------
  bool inPic(int ch, const Area &a) const { (void)ch; return a.x < pic.W && a.y < pic.H; }

  void coding_tree(Partitioner &p, CuCtx &cuCtx, Partitioner *pc = nullptr, CuCtx *cuCtxC = nullptr) {
    if (pps.useDQP && p.qgEnable() && p.chType == 0) { cuCtx.qgStart = true; cuCtx.isDQPCoded = false; }
    if (sh.chromaQpAdj && p.qgChromaEnable()) { cuCtx.isChromaQpAdjCoded = false; chromaQpAdj = 0; }
    if (dualTree && pc) {
      if (pps.useDQP && pc->qgEnable()) { cuCtxC->qgStart = true; cuCtxC->isDQPCoded = false; }
      if (sh.chromaQpAdj && pc->qgChromaEnable()) { cuCtxC->isChromaQpAdjCoded = false; chromaQpAdj = 0; }
    }
    const int split = split_cu_mode(p);
    VVCP_CHECK(!canSplitMode(p, split), "invalid split");
    if (split != S_DONT) {
      if (dualTree && pc && (p.area().w >= 64 || p.area().h >= 64)) {
        splitCU(p, S_QT);
        splitCU(*pc, S_QT);
        bool more = true;
        while (more) {
          if (p.area().w > 64 || p.area().h > 64) {
            if (inPic(0, p.area())) coding_tree(p, cuCtx, pc, cuCtxC);
            const bool l = nextPart(p), c = nextPart(*pc);
            VVCP_CHECK(l != c, "luma / chroma partitions diverge");
            more = l;
          } else {
            if (inPic(0, p.area())) coding_tree(p, cuCtx);
            const bool l = nextPart(p);
            if (inPic(1, pc->area())) coding_tree(*pc, *cuCtxC);
            const bool c = nextPart(*pc);
            VVCP_CHECK(l != c, "luma / chroma partitions diverge");
            more = l;
          }
        }
        exitSplit(p);
        exitSplit(*pc);
      } else {
        const int modeTypeParent = p.modeType;
        p.modeType = mode_constraint(p, split);
        const bool chromaNotSplit = modeTypeParent == MT_ALL && p.modeType == MT_INTRA;
        VVCP_CHECK(chromaNotSplit && p.chType != 0, "mode constraint on a chroma tree");
        if (p.treeType == TREE_D) p.treeType = chromaNotSplit ? TREE_L : TREE_D;
        splitCU(p, split);
        do {
          if (inPic(p.chType, p.area())) coding_tree(p, cuCtx);
        } while (nextPart(p));
        exitSplit(p);
        if (chromaNotSplit) {
          p.chType = 1;
          p.treeType = TREE_C;
          if (inPic(1, p.area())) coding_tree(p, cuCtx);
          p.chType = 0;
          p.treeType = TREE_D;
        }
        p.modeType = modeTypeParent;
      }
      return;
    }
    make_cu(p, cuCtx);
  }

  // ------------------------------------------------------------------------------------------------
  // CU creation (CodingStructure::addCU, coding_tree :629-667) and coding_unit (:811)
  // ------------------------------------------------------------------------------------------------
  bool isSepTree(int treeType) const { return treeType != TREE_D || dualTree; }

  void make_cu(Partitioner &p, CuCtx &cuCtx) {
    const Area &a = p.area();
    const bool sep = isSepTree(p.treeType);
    vvcr_cu c;
    std::memset(&c, 0, sizeof(c));
    const bool yv = !sep || p.chType == 0, cv = !sep || p.chType == 1;
    if (yv) { c.x = a.x; c.y = a.y; c.w = a.w; c.h = a.h; }
    if (cv) { c.cx = a.x >> 1; c.cy = a.y >> 1; c.cw = a.w >> 1; c.ch = a.h >> 1; }
    c.chtype = p.chType;
    c.predmode = 4;   // NUMBER_OF_PREDICTION_MODES until pred_mode()
    c.treetype = p.treeType;
    c.modetype = p.modeType;
    c.rootcbf = 1;
    c.bcw = BCW_DEFAULT;
    c.depth = p.depth;
    c.qtdepth = p.qtDepth;
    c.firstpu = -1; c.firsttu = -1;
    c.slice = sh.sliceAddr;   // Slice::getSliceID (VLCReader.cpp:2737: the slice address); CuAux::slice is the index
    c.yvalid = yv; c.cvalid = cv;
    CuAux x;
    x.splitSeries = p.splitSeries();
    x.mtDepth = p.mtDepth;
    x.btDepth = p.btDepth;
    x.tile = tileOf(a.x, a.y);
    x.slice = sc.sliceIdx;
    x.ctu = curCtu;
    x.hmvpReset = firstCuOfCtu && ctuHmvpReset;
    firstCuOfCtu = false;
    const int idx = (int)pic.cu.size();
    pic.cu.push_back(c);
    pic.cux.push_back(x);
    if (yv != cv) shp.unshareMap();
    if (yv) fill_map(0, idx, a.x, a.y, a.w, a.h);
    if (cv && !shp.mapShared) fill_map(1, idx, a.x, a.y, a.w, a.h);

    int lumaQPinLocalDualTree = -1;
    if (cuCtx.qgStart) { cuCtx.qgStart = false; cuCtx.qp = predictQP(idx, cuCtx.qp); }
    if (pps.useDQP && sep && p.chType == 1) {   // chroma CU of a separate tree takes the co-located luma QP
      const int lx = ((a.x >> 1) + (a.w >> 2)) << 1, ly = ((a.y >> 1) + (a.h >> 2)) << 1;
      const int colL = cuAt(0, lx, ly);
      VVCP_CHECK(colL < 0, "co-located luma CU missing");
      lumaQPinLocalDualTree = cuCtx.qp;
      cuCtx.qp = pic.cu[colL].qp;
    }
    pic.cu[idx].qp = cuCtx.qp;
    pic.cu[idx].cqpadj = chromaQpAdj;
    coding_unit(p, idx, cuCtx);
    if (pps.useDQP && sep && p.chType == 1) cuCtx.qp = lumaQPinLocalDualTree;
    fill_tu_qp(idx);
  }

  // QpParam (Quant.cpp:65-138) of the blocks DecCu inverse-transforms (DecCu.cpp:243-266): the luma /
  // chroma blocks with a cbf, and for joint Cb-Cr the one coded block (Cb for modes 2/3, Cr for mode 1).
  // Blocks of such a TU that are not transformed report 0, TUs without any transform -1000 (the
  // capture's per-TU record, oracle/capture/vtm_capture.cpp:757).
  void fill_tu_qp(int ci) {
    const vvcr_cu &c = pic.cu[ci];
    const int off = sps.qpBdOffset;
    for (int k = 0; k < c.ntu; k++) {
      vvcr_tu &t = pic.tu[c.firsttu + k];
      bool tr[3] = {false, false, false};
      if (tuValid(t, 0) && cbfAt(t, 0, t.depth)) tr[0] = true;
      if (tuValid(t, 1)) {
        if (t.jccr) { if (t.jccr >> 1) tr[1] = true; else tr[2] = true; }
        else { tr[1] = cbfAt(t, 1, t.depth); tr[2] = cbfAt(t, 2, t.depth); }
      }
      if (!tr[0] && !tr[1] && !tr[2]) continue;
      for (int comp = 0; comp < 3; comp++) {
        if (!tuValid(t, comp)) continue;
        if (!tr[comp]) { t.b[comp][7] = 0; t.b[comp][8] = 0; continue; }
        int base;
        if (comp == 0) base = c.qp + off;
        else {
          const bool jqp = t.jccr == 3;   // |g_ictModes[.][jccr]| == 2
          const int cc = jqp ? 3 : comp;
          int cqo = (cc == 3 ? pps.jcQpOffset : (cc == 1 ? pps.cbQpOffset : pps.crQpOffset));
          cqo += cc == 3 ? sh.jcQpDelta : (cc == 1 ? sh.cbQpDelta : sh.crQpDelta);
          cqo += pps.cqpList[c.cqpadj][cc - 1];
          const int qpi = clip3(-off, 63, c.qp);
          base = sps.mappedChromaQp(cc, qpi);
          base = clip3(-off, 63, base + cqo) + off;
        }
        base = clip3(0, 63 + off, base);
        t.b[comp][7] = base;
        t.b[comp][8] = std::max(base, 4 + sps.minQpTsMinus4);
      }
    }
  }

  // CU::predictQP (UnitTools.cpp:199)
  int predictQP(int idx, int prevQP) {
    const vvcr_cu &c = pic.cu[idx];
    const int ch = c.chtype;
    const int bx = ch ? c.cx : c.x, by = ch ? c.cy : c.y;
    const int mask = (pic.ctuSize - 1) >> ch;
    const CuAux &x = pic.cux[idx];
    const int ctuX = x.ctu % pic.wCtu;
    const int tileX = pps.colBd[pps.ctuToTileCol[ctuX]];
    if (ctuX == tileX && !(bx & mask) && !(by & mask)) {
      const int above = cuRestricted(ch, bx, by - 1, x.slice, x.tile);
      if (above >= 0) return pic.cu[above].qp;
    }
    const int a = (by & mask) ? pic.cu[cuAt(ch, bx, by - 1)].qp : prevQP;
    const int b = (bx & mask) ? pic.cu[cuAt(ch, bx - 1, by)].qp : prevQP;
    return (a + b + 1) >> 1;
  }

  int new_pu(int cuIdx) {
    const vvcr_cu &c = pic.cu[cuIdx];
    vvcr_pu u;
    std::memset(&u, 0, sizeof(u));
    u.cu = cuIdx;
    u.x = c.x; u.y = c.y; u.w = c.w; u.h = c.h;
    u.cx = c.cx; u.cy = c.cy; u.cw = c.cw; u.ch = c.ch;
    u.chtype = c.chtype;
    u.idir_l = DC; u.idir_c = PLANAR;
    u.fidir_l = -1; u.fidir_c = -1;
    u.mergeidx = 255; u.geodir = 255; u.geoi0 = 255; u.geoi1 = 255;
    u.interdir = 255;
    u.ref0 = -1; u.ref1 = -1;
    u.dmvr_off = -1;
    const int idx = (int)pic.pu.size();
    pic.pu.push_back(u);
    pic.pux.push_back(PuSyntax());
    pic.cu[cuIdx].firstpu = idx;
    pic.cu[cuIdx].npu = 1;
    return idx;
  }

  int new_tu(int cuIdx, const Area &a, int chType, bool sep) {
    vvcr_tu t;
    std::memset(&t, 0, sizeof(t));
    t.cu = cuIdx;
    t.chtype = chType;
    const bool yv = !sep || chType == 0, cv = (!sep || chType == 1) && a.cvalid;
    for (int c = 0; c < 3; c++) {
      int32_t *b = t.b[c];
      b[6] = -1; b[7] = -1000; b[8] = -1000;
      if (c == 0 && yv) { b[0] = a.x; b[1] = a.y; b[2] = a.w; b[3] = a.h; }
      if (c > 0 && cv) { b[0] = a.x >> 1; b[1] = a.y >> 1; b[2] = a.w >> 1; b[3] = a.h >> 1; }
    }
    const int idx = (int)pic.tu.size();
    pic.tu.push_back(t);
    if (pic.cu[cuIdx].firsttu < 0) pic.cu[cuIdx].firsttu = idx;
    pic.cu[cuIdx].ntu++;
    return idx;
  }
  static bool tuValid(const vvcr_tu &t, int c) { return t.b[c][2] > 0 && t.b[c][3] > 0; }

  void coding_unit(Partitioner &p, int ci, CuCtx &cuCtx) {
    const int pi = new_pu(ci);
    vvcr_cu *c = &pic.cu[ci];
    if (!sh.isIntra() && c->yvalid) cu_skip_flag(ci);
    c = &pic.cu[ci];
    if (c->skip) {
      new_tu(ci, p.area(), p.chType, isSepTree(p.treeType));
      prediction_unit(ci, pi);
      return;
    }
    pred_mode(ci);
    VVCP_CHECK(pic.cu[ci].predmode == MODE_PLT || pic.cu[ci].predmode == MODE_IBC, "palette / IBC CUs are not supported");
    bdpcm_mode(ci, p.chType);
    if (!dualTree && p.chType == 0) bdpcm_mode(ci, 1);
    cu_pred_data(ci, pi);
    cu_residual(p, ci, pi, cuCtx);
  }

  // CABACReader::cu_skip_flag (:878) with IBC disabled; DeriveCtx::CtxSkipFlag (ContextModelling.cpp:279)
  void cu_skip_flag(int ci) {
    vvcr_cu &c = pic.cu[ci];
    if (c.w == 4 && c.h == 4) return;
    if (c.modetype == MT_INTRA) return;
    const int tile = pic.cux[ci].tile;
    const int cl = cuRestricted(0, c.x - 1, c.y, sc.sliceIdx, tile);
    const int ca = cuRestricted(0, c.x, c.y - 1, sc.sliceIdx, tile);
    const unsigned ctx = (cl >= 0 && pic.cu[cl].skip ? 1 : 0) + (ca >= 0 && pic.cu[ca].skip ? 1 : 0);
    if (cab.bin(SkipFlag + ctx)) {
      c.skip = 1;
      c.rootcbf = 0;
      c.predmode = MODE_INTER;
    }
  }

  // CABACReader::pred_mode (:1038), IBC / palette disabled
  void pred_mode(int ci) {
    vvcr_cu &c = pic.cu[ci];
    if (c.modetype == MT_INTER) { c.predmode = MODE_INTER; return; }
    if (sh.isIntra() || (c.w == 4 && c.h == 4) || c.modetype == MT_INTRA) { c.predmode = MODE_INTRA; return; }
    const int tile = pic.cux[ci].tile;
    const int cl = cuRestricted(0, c.x - 1, c.y, sc.sliceIdx, tile);
    const int ca = cuRestricted(0, c.x, c.y - 1, sc.sliceIdx, tile);
    const unsigned ctx = ((ca >= 0 && pic.cu[ca].predmode == MODE_INTRA) || (cl >= 0 && pic.cu[cl].predmode == MODE_INTRA)) ? 1 : 0;
    c.predmode = cab.bin(PredMode + ctx) ? MODE_INTRA : MODE_INTER;
  }

  // CU::bdpcmAllowed (UnitTools.cpp:3836) + CABACReader::bdpcm_mode (:1127)
  void bdpcm_mode(int ci, int ch) {
    vvcr_cu &c = pic.cu[ci];
    const int tsMax = 1 << pps.log2MaxTs;
    bool allowed = sps.bdpcm != 0;
    allowed &= ch == 0 || sps.bdpcm == 2;
    allowed &= c.predmode == MODE_INTRA;
    if (ch == 0) allowed &= c.w <= tsMax && c.h <= tsMax;
    else allowed &= c.cw <= tsMax && c.ch <= tsMax;
    if (!allowed) {
      if (ch == 0) { c.bdpcm = 0; if (!dualTree) c.bdpcmc = 0; }
      else c.bdpcmc = 0;
      return;
    }
    int m = cab.bin(BDPCMMode);
    if (m) m += cab.bin(BDPCMMode + 1);
    if (ch == 0) c.bdpcm = m; else c.bdpcmc = m;
  }

  // CABACReader::cu_pred_data (:1171)
  void cu_pred_data(int ci, int pi) {
    if (pic.cu[ci].predmode == MODE_INTRA) {
      intra_luma_pred_modes(ci, pi);
      intra_chroma_pred_modes(ci, pi);
      return;
    }
    VVCP_CHECK(!pic.cu[ci].yvalid, "inter CU without luma");
    prediction_unit(ci, pi);
    imv_mode(ci, pi);
    affine_amvr_mode(ci, pi);
    cu_bcw_flag(ci, pi);
  }

  // xReadTruncBinCode (:1237)
  uint32_t truncBin(uint32_t maxSymbol) {
    int thresh;
    if (maxSymbol > 256) {
      int tv = 1 << 8;
      thresh = 8;
      while (tv <= (int)maxSymbol) { thresh++; tv <<= 1; }
      thresh--;
    } else thresh = tbMax(maxSymbol);
    const int val = 1 << thresh, b = (int)maxSymbol - val;
    uint32_t s = cab.eps(thresh);
    if ((int)s >= val - b) {
      s = (s << 1) + cab.ep();
      s -= (val - b);
    }
    return s;
  }

  // intra_luma_pred_modes (:1311), mip_flag (:3682), extend_ref_line (:1269), isp_mode (:3061),
  // PU::getIntraMPMs (UnitTools.cpp:445)
  void intra_luma_pred_modes(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    if (!c.yvalid) return;
    if (c.bdpcm) { pic.pu[pi].idir_l = c.bdpcm == 2 ? VER : HOR; return; }
    // mip_flag: DeriveCtx::CtxMipFlag (ContextModelling.cpp:534)
    if (sps.mip) {
      const int tile = pic.cux[ci].tile;
      const int cl = cuRestricted(0, c.x - 1, c.y, sc.sliceIdx, tile);
      const int ca = cuRestricted(0, c.x, c.y - 1, sc.sliceIdx, tile);
      unsigned ctx = (cl >= 0 && pic.cu[cl].mip ? 1 : 0) + (ca >= 0 && pic.cu[ca].mip ? 1 : 0);
      if (c.w > 2 * c.h || c.h > 2 * c.w) ctx = 3;
      c.mip = cab.bin(MipFlag + ctx);
    } else c.mip = 0;
    if (c.mip) {
      pic.pu[pi].mipt = cab.ep();
      const int sizeId = (c.w == 4 && c.h == 4) ? 0 : ((c.w == 4 || c.h == 4 || (c.w == 8 && c.h == 8)) ? 1 : 2);
      static const int nModes[3] = {16, 8, 6};
      pic.pu[pi].idir_l = (int)truncBin(nModes[sizeId]);
      return;
    }
    // extend_ref_line
    vvcr_pu &u = pic.pu[pi];
    u.mrl = 0;
    if (c.predmode == MODE_INTRA && c.chtype == 0 && !c.bdpcm && sps.mrl) {
      const bool firstLineOfCtu = (c.y & (pic.ctuSize - 1)) == 0;
      if (!firstLineOfCtu) {
        int m = cab.bin(MultiRefLineIdx) ? 1 : 0;
        if (m) m = cab.bin(MultiRefLineIdx + 1) ? 2 : 1;
        u.mrl = m;
      }
    }
    // isp_mode (CU::canUseISP UnitTools.cpp:343)
    c.isp = 0;
    if (c.chtype == 0 && !u.mrl && sps.isp && !c.bdpcm) {
      const bool notEnough = floorLog2(c.w) + floorLog2(c.h) <= 4;
      if (!notEnough && c.w <= maxTb && c.h <= maxTb) {
        if (cab.bin(ISPMode)) c.isp = 1 + cab.bin(ISPMode + 1);
      }
    }
    const bool mpmFlag = u.mrl ? true : cab.bin(IntraLumaMpmFlag) != 0;
    unsigned mpm[6];
    getIntraMPMs(ci, mpm);
    if (mpmFlag) {
      uint32_t idx = 0;
      const unsigned ctx = c.isp == 0 ? 1 : 0;
      if (u.mrl == 0) idx = cab.bin(IntraLumaPlanarFlag + ctx);
      else idx = 1;
      if (idx) idx += cab.ep();
      if (idx > 1) idx += cab.ep();
      if (idx > 2) idx += cab.ep();
      if (idx > 3) idx += cab.ep();
      u.idir_l = (int)mpm[idx];
    } else {
      unsigned m = truncBin(67 - 6);
      std::sort(mpm, mpm + 6);
      for (int i = 0; i < 6; i++) m += (m >= mpm[i]);
      u.idir_l = (int)m;
    }
  }
  int intraDirLuma(int cuIdx) const {   // PU::getIntraDirLuma (UnitTools.cpp:561)
    if (pic.cu[cuIdx].mip) return PLANAR;
    return pic.pu[pic.cu[cuIdx].firstpu].idir_l;
  }
  void getIntraMPMs(int ci, unsigned *mpm) {
    const vvcr_cu &c = pic.cu[ci];
    int left = PLANAR, above = PLANAR;
    const int tile = pic.cux[ci].tile;
    const int pl = cuRestricted(0, c.x - 1, c.y + c.h - 1, sc.sliceIdx, tile);
    if (pl >= 0 && pic.cu[pl].predmode == MODE_INTRA) left = intraDirLuma(pl);
    const int pa = cuRestricted(0, c.x + c.w - 1, c.y - 1, sc.sliceIdx, tile);
    if (pa >= 0 && pic.cu[pa].predmode == MODE_INTRA && pic.cux[pa].ctu == pic.cux[ci].ctu) above = intraDirLuma(pa);
    const int offset = 67 - 6, mod = offset + 3;
    mpm[0] = PLANAR; mpm[1] = DC; mpm[2] = VER; mpm[3] = HOR; mpm[4] = VER - 4; mpm[5] = VER + 4;
    if (left == above) {
      if (left > DC) {
        mpm[0] = PLANAR; mpm[1] = left;
        mpm[2] = ((left + offset) % mod) + 2;
        mpm[3] = ((left - 1) % mod) + 2;
        mpm[4] = ((left + offset - 1) % mod) + 2;
        mpm[5] = (left % mod) + 2;
      }
    } else {
      if (left > DC && above > DC) {
        mpm[0] = PLANAR; mpm[1] = left; mpm[2] = above;
        const int maxI = mpm[1] > mpm[2] ? 1 : 2, minI = mpm[1] > mpm[2] ? 2 : 1;
        const int mx = (int)mpm[maxI], mn = (int)mpm[minI];
        if (mx - mn == 1) {
          mpm[3] = ((mn + offset) % mod) + 2; mpm[4] = ((mx - 1) % mod) + 2; mpm[5] = ((mn + offset - 1) % mod) + 2;
        } else if (mx - mn >= 62) {
          mpm[3] = ((mn - 1) % mod) + 2; mpm[4] = ((mx + offset) % mod) + 2; mpm[5] = (mn % mod) + 2;
        } else if (mx - mn == 2) {
          mpm[3] = ((mn - 1) % mod) + 2; mpm[4] = ((mn + offset) % mod) + 2; mpm[5] = ((mx - 1) % mod) + 2;
        } else {
          mpm[3] = ((mn + offset) % mod) + 2; mpm[4] = ((mn - 1) % mod) + 2; mpm[5] = ((mx + offset) % mod) + 2;
        }
      } else if (left + above >= 2) {
        mpm[0] = PLANAR;
        const int mx = left < above ? above : left;
        mpm[1] = mx;
        mpm[2] = ((mx + offset) % mod) + 2;
        mpm[3] = ((mx - 1) % mod) + 2;
        mpm[4] = ((mx + offset - 1) % mod) + 2;
        mpm[5] = (mx % mod) + 2;
      }
    }
  }

  // PU::getCoLocatedIntraLumaMode (UnitTools.cpp:642)
  int coLocatedLumaMode(int ci) const {
    const vvcr_cu &c = pic.cu[ci];
    int lc;
    if (isSepTree(c.treetype)) lc = cuAt(0, (c.cx << 1) + c.cw, (c.cy << 1) + c.ch);
    else lc = ci;
    VVCP_CHECK(lc < 0, "co-located luma PU missing");
    return intraDirLuma(lc);
  }
  // CodingUnit::checkCCLMAllowed (Unit.cpp:381)
  bool cclmAllowed(int ci) const {
    if (!dualTree) return true;
    if (sps.ctuSize <= 32) return true;
    const vvcr_cu &c = pic.cu[ci];
    const int d64 = sps.ctuSize == 128 ? 1 : 0;
    const uint64_t ss = pic.cux[ci].splitSeries;
    const int s1 = splitAtDepth(ss, c.depth, d64), s2 = splitAtDepth(ss, c.depth, d64 + 1);
    bool allow = false;
    if (s1 == S_QT || (s1 == S_BH && s2 == S_BV)) allow = true;
    else if (s1 == S_DONT) allow = true;
    else if (s1 == S_BH && s2 == S_DONT) allow = true;
    if (allow) {
      const int lc = cuAt(0, c.cx << 1, c.cy << 1);
      VVCP_CHECK(lc < 0, "co-located luma CU missing");
      const vvcr_cu &l = pic.cu[lc];
      if (l.w < 64 || l.h < 64) {
        if (splitAtDepth(pic.cux[lc].splitSeries, l.depth, d64) != S_QT) allow = false;
      } else if (l.w == 64 && l.h == 64 && l.isp) allow = false;
    }
    return allow;
  }
  // intra_chroma_pred_modes (:1409), intra_chroma_pred_mode (:1443), PU::getIntraChromaCandModes (:574)
  void intra_chroma_pred_modes(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    if (isSepTree(c.treetype) && c.chtype == 0) return;
    vvcr_pu &u = pic.pu[pi];
    if (c.bdpcmc) {
      unsigned modes[4] = {PLANAR, VER, HOR, DC};
      const int lm = coLocatedLumaMode(ci);
      for (int i = 0; i < 4; i++) if ((int)modes[i] == lm) { modes[i] = VDIA; break; }
      u.idir_c = (int)modes[0];
      return;
    }
    if (sps.cclm && cclmAllowed(ci)) {
      if (cab.bin(CclmModeFlag)) {
        int s = cab.bin(CclmModeIdx);
        if (s) s += cab.ep();
        static const int lmList[3] = {LM, MDLM_L, MDLM_T};
        u.idir_c = lmList[s];
        return;
      }
    }
    if (cab.bin(IntraChromaPredMode) == 0) { u.idir_c = DM; return; }
    const unsigned cand = cab.eps(2);
    unsigned modes[4] = {PLANAR, VER, HOR, DC};
    const int lm = coLocatedLumaMode(ci);
    for (int i = 0; i < 4; i++) if ((int)modes[i] == lm) { modes[i] = VDIA; break; }
    u.idir_c = (int)modes[cand];
  }

  // ------------------------------------------------------------------------------------------------
  // Inter prediction syntax (prediction_unit :1975 and helpers)
  // ------------------------------------------------------------------------------------------------
  bool bipredRestriction(const vvcr_cu &c) const { return (c.w == 4 && c.h == 4) || c.w + c.h == 12; }
  unsigned ctxAffine(int ci) const {
    const vvcr_cu &c = pic.cu[ci];
    const int tile = pic.cux[ci].tile;
    const int cl = cuRestricted(0, c.x - 1, c.y, sc.sliceIdx, tile);
    const int ca = cuRestricted(0, c.x, c.y - 1, sc.sliceIdx, tile);
    return (cl >= 0 && pic.cu[cl].affine ? 1 : 0) + (ca >= 0 && pic.cu[ca].affine ? 1 : 0);
  }
  void prediction_unit(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    vvcr_pu &u = pic.pu[pi];
    PuSyntax &s = pic.pux[pi];
    if (c.skip) u.merge = 1;
    else u.merge = cab.bin(MergeFlag);
    if (u.merge) {
      merge_data(ci, pi);
    } else {
      // inter_pred_idc (:2438)
      if (sh.isInterP()) u.interdir = 1;
      else {
        u.interdir = 0;
        if (!bipredRestriction(c)) {
          const unsigned ctx = 7 - ((floorLog2(c.w) + floorLog2(c.h) + 1) >> 1);
          if (cab.bin(InterDir + ctx)) u.interdir = 3;
        }
        if (!u.interdir) u.interdir = cab.bin(InterDir + 5) ? 2 : 1;
      }
      // affine_flag (:2109)
      if (sps.affine && c.w > 8 && c.h > 8) {
        c.affine = cab.bin(AffineFlag + ctxAffine(ci));
        if (c.affine && sps.affineType) c.affinetype = cab.bin(AffineType);
        else c.affinetype = 0;
      }
      // smvd_mode (:2075)
      c.smvd = 0;
      if (u.interdir == 3 && !c.affine && sh.biDirPred) c.smvd = cab.bin(SmvdFlag) ? 1 : 0;
      if (u.interdir != 2) {
        u.ref0 = ref_idx(c, 0);
        if (c.affine) {
          mvd_coding(s.mvdAffi[0][0]);
          mvd_coding(s.mvdAffi[0][1]);
          if (c.affinetype) mvd_coding(s.mvdAffi[0][2]);
        } else mvd_coding(s.mvd[0]);
        s.mvpIdx[0] = cab.bin(MVPIdx);
      }
      if (u.interdir != 1) {
        if (c.smvd != 1) {
          u.ref1 = ref_idx(c, 1);
          if (ph.mvdL1Zero && u.interdir == 3) {
            std::memset(s.mvd[1], 0, sizeof(s.mvd[1]));
            std::memset(s.mvdAffi[1], 0, sizeof(s.mvdAffi[1]));
          } else if (c.affine) {
            mvd_coding(s.mvdAffi[1][0]);
            mvd_coding(s.mvdAffi[1][1]);
            if (c.affinetype) mvd_coding(s.mvdAffi[1][2]);
          } else mvd_coding(s.mvd[1]);
        }
        s.mvpIdx[1] = cab.bin(MVPIdx);
      }
    }
    if (u.interdir == 3 && bipredRestriction(c)) {
      u.mv1x = u.mv1y = 0;
      u.ref1 = -1;
      u.interdir = 1;
      c.bcw = BCW_DEFAULT;
    }
    if (c.smvd) {
      const int cur = c.smvd - 1;
      s.mvd[1 - cur][0] = -s.mvd[cur][0];
      s.mvd[1 - cur][1] = -s.mvd[cur][1];
      if (1 - cur == 0) u.ref0 = sh.symRefIdx[0]; else u.ref1 = sh.symRefIdx[1];
    }
  }
  int ref_idx(const vvcr_cu &c, int l) {   // CABACReader::ref_idx (:2469)
    if (c.smvd) return sh.symRefIdx[l];
    const int n = sh.numRef[l];
    if (n <= 1 || !cab.bin(RefPic)) return 0;
    if (n <= 2 || !cab.bin(RefPic + 1)) return 1;
    for (int idx = 3;; idx++)
      if (n <= idx || !cab.ep()) return idx - 1;
  }
  void mvd_coding(int32_t *mvd) {   // CABACReader::mvd_coding (:2659)
    int hor = (int)cab.bin(Mvd), ver = (int)cab.bin(Mvd);
    if (hor) hor += (int)cab.bin(Mvd + 1);
    if (ver) ver += (int)cab.bin(Mvd + 1);
    if (hor) {
      if (hor > 1) hor += (int)cab.rem_abs(1, 0, 17);
      if (cab.ep()) hor = -hor;
    }
    if (ver) {
      if (ver > 1) ver += (int)cab.rem_abs(1, 0, 17);
      if (cab.ep()) ver = -ver;
    }
    mvd[0] = hor;
    mvd[1] = ver;
  }
  void merge_data(int ci, int pi) {   // CABACReader::merge_data (:2149) + merge_idx (:2266)
    vvcr_cu &c = pic.cu[ci];
    vvcr_pu &u = pic.pu[pi];
    PuSyntax &s = pic.pux[pi];
    // subblock_merge_flag (:2095)
    c.affine = 0;
    if (!sh.isIntra() && ph.maxNumAffineMergeCand > 0 && c.w >= 8 && c.h >= 8)
      c.affine = cab.bin(SubblockMergeFlag + ctxAffine(ci));
    if (c.affine) {
      const int n1 = ph.maxNumAffineMergeCand - 1;
      u.mergeidx = 0;
      if (n1 > 0 && cab.bin(AffMergeIdx)) {
        u.mergeidx++;
        for (; u.mergeidx < n1; u.mergeidx++)
          if (!cab.ep()) break;
      }
      u.regmerge = 0;
      return;
    }
    const bool ciipAvail = sps.ciip && !c.skip && c.w < 128 && c.h < 128 && c.w * c.h >= 64;
    const bool geoAvail = sps.geo && sh.isInterB() && ph.maxNumGeoCand > 1 && c.w >= 8 && c.h >= 8 && c.w <= 64 && c.h <= 64 &&
                          c.w < 8 * c.h && c.h < 8 * c.w;
    if (geoAvail || ciipAvail) u.regmerge = cab.bin(RegularMergeFlag + (c.skip ? 0 : 1));
    else u.regmerge = 1;
    if (u.regmerge) {
      u.mmvd = sps.mmvd ? cab.bin(MmvdFlag) : 0;
      // the reference assigns mmvdSkip on a copy of the CU here (CABACReader.cpp:2158/2201): the CU keeps 0
    } else {
      u.mmvd = 0;
      c.mmvdskip = 0;
      if (geoAvail && ciipAvail) u.ciip = cab.bin(CiipFlag);
      else u.ciip = ciipAvail ? 1 : 0;
      if (u.ciip) { u.idir_l = PLANAR; u.idir_c = DM; }
      else c.geo = 1;
    }
    if (u.mmvd) {   // mmvd_merge_idx (:2390)
      int v0 = 0;
      if (ph.maxNumMergeCand > 1) v0 = cab.bin(MmvdMergeIdx);
      int v1 = 0;
      if (cab.bin(MmvdStepMvpIdx)) {
        v1++;
        for (; v1 < 7; v1++)
          if (!cab.ep()) break;
      }
      int v2 = 0;
      if (cab.ep()) { v2 += 2; if (cab.ep()) v2 += 1; }
      else { if (cab.ep()) v2 += 1; }
      s.mmvdMergeIdx = v0 * 32 + v1 * 4 + v2;
      return;
    }
    if (c.geo) {
      u.geodir = (int)truncBin(64);
      const int n2 = ph.maxNumGeoCand - 2;
      u.mergeidx = 0;
      int m0 = 0, m1 = 0;
      if (cab.bin(MergeIdx)) m0 += unary_max_eqprob(n2) + 1;
      if (n2 > 0 && cab.bin(MergeIdx)) m1 += unary_max_eqprob(n2 - 1) + 1;
      m1 += m1 >= m0 ? 1 : 0;
      u.geoi0 = m0;
      u.geoi1 = m1;
      return;
    }
    const int n1 = ph.maxNumMergeCand - 1;
    u.mergeidx = 0;
    if (n1 > 0 && cab.bin(MergeIdx)) {
      u.mergeidx++;
      for (; u.mergeidx < n1; u.mergeidx++)
        if (!cab.ep()) break;
    }
  }
  unsigned unary_max_eqprob(unsigned maxSymbol) {
    for (unsigned k = 0; k < maxSymbol; k++)
      if (!cab.ep()) return k;
    return maxSymbol;
  }
  // imv_mode (:957), CU::hasSubCUNonZeroMVd (UnitTools.cpp:3518)
  void imv_mode(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    if (!sps.amvr) return;
    const vvcr_pu &u = pic.pu[pi];
    const PuSyntax &s = pic.pux[pi];
    bool nz = false;
    if (!u.merge && !c.skip) {
      if (u.interdir != 2) nz |= s.mvd[0][0] != 0 || s.mvd[0][1] != 0;
      if (u.interdir != 1 && (!ph.mvdL1Zero || u.interdir != 3)) nz |= s.mvd[1][0] != 0 || s.mvd[1][1] != 0;
    }
    if (!nz || c.affine) return;
    int v = cab.bin(ImvFlag);
    c.imv = v;
    if (v) {
      v = cab.bin(ImvFlag + 4);
      c.imv = v ? 1 : 3;
      if (v) c.imv = 1 + cab.bin(ImvFlag + 1);
    }
  }
  // affine_amvr_mode (:1007), CU::hasSubCUNonZeroAffineMVd (:3545)
  void affine_amvr_mode(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    if (!sps.affineAmvr || !c.affine) return;
    const vvcr_pu &u = pic.pu[pi];
    const PuSyntax &s = pic.pux[pi];
    if (u.merge) return;
    bool nz = false;
    const int n = c.affinetype ? 3 : 2;
    if (!c.skip) {
      if (u.interdir != 2)
        for (int i = 0; i < n; i++) nz |= s.mvdAffi[0][i][0] != 0 || s.mvdAffi[0][i][1] != 0;
      if (u.interdir != 1 && (!ph.mvdL1Zero || u.interdir != 3))
        for (int i = 0; i < n; i++) nz |= s.mvdAffi[1][i][0] != 0 || s.mvdAffi[1][i][1] != 0;
    }
    if (!nz) return;
    int v = cab.bin(ImvFlag + 2);
    if (v) v = 1 + cab.bin(ImvFlag + 3);
    c.imv = v;
  }
  // cu_bcw_flag (:1197), CU::isBcwIdxCoded (UnitTools.cpp:3715)
  void cu_bcw_flag(int ci, int pi) {
    vvcr_cu &c = pic.cu[ci];
    const vvcr_pu &u = pic.pu[pi];
    if (!sps.bcw || c.predmode == MODE_INTRA || sh.isInterP() || c.w * c.h < 256) return;
    if (u.merge || u.interdir != 3) return;
    for (int k = 0; k < 3; k++)
      if (sh.wp[0][u.ref0][k][0] || sh.wp[1][u.ref1][k][0]) return;
    uint32_t idx = 0;
    if (cab.bin(BcwIdx)) {
      const int numBcw = sh.checkLDC ? 5 : 3;
      idx = 1;
      for (int i = 0; i < numBcw - 2; i++) {
        if (!cab.ep()) break;
        idx++;
      }
    }
    c.bcw = kBcwParsingOrder[idx];
  }

  // ------------------------------------------------------------------------------------------------
  // Residual (cu_residual :1489, transform_tree :2550, transform_unit :2719)
  // ------------------------------------------------------------------------------------------------
  uint8_t sbtAllowed(const vvcr_cu &c, const vvcr_pu &u) const {   // CodingUnit::checkAllowedSbt (Unit.cpp:453)
    if (!sps.sbt || c.predmode != MODE_INTER || u.ciip) return 0;
    if (c.w > maxTb || c.h > maxTb) return 0;
    uint8_t a = 0;
    a |= (c.w >= 8) << SBT_VER_HALF;
    a |= (c.h >= 8) << SBT_HOR_HALF;
    a |= (c.w >= 16) << SBT_VER_QUAD;
    a |= (c.h >= 16) << SBT_HOR_QUAD;
    return a;
  }
  void sbt_mode(int ci, int pi) {   // CABACReader::sbt_mode (:1577)
    vvcr_cu &c = pic.cu[ci];
    const uint8_t allowed = sbtAllowed(c, pic.pu[pi]);
    if (!allowed) return;
    if (!cab.bin(SbtFlag + (c.w * c.h <= 256 ? 1 : 0))) return;
    const bool vh = (allowed >> SBT_VER_HALF) & 1, hh = (allowed >> SBT_HOR_HALF) & 1;
    const bool vq = (allowed >> SBT_VER_QUAD) & 1, hq = (allowed >> SBT_HOR_QUAD) & 1;
    bool quad = false;
    if ((hh || vh) && (hq || vq)) quad = cab.bin(SbtQuadFlag);
    bool hor;
    if ((quad && vq && hq) || (!quad && vh && hh)) hor = cab.bin(SbtHorFlag + (c.w == c.h ? 0 : (c.w < c.h ? 1 : 2)));
    else hor = (quad && hq) || (!quad && hh);
    const int idx = hor ? (quad ? SBT_HOR_QUAD : SBT_HOR_HALF) : (quad ? SBT_VER_QUAD : SBT_VER_HALF);
    const int pos = cab.bin(SbtPosFlag);
    c.sbtinfo = (pos << 4) + idx;
  }

  void cu_residual(Partitioner &p, int ci, int pi, CuCtx &cuCtx) {
    vvcr_cu *c = &pic.cu[ci];
    if (c->predmode != MODE_INTRA) {
      if (!pic.pu[pi].merge) c->rootcbf = cab.bin(QtRootCbf);
      else c->rootcbf = 1;
      if (c->rootcbf) sbt_mode(ci, pi);
      c = &pic.cu[ci];
      if (!c->rootcbf) {
        new_tu(ci, p.area(), p.chType, isSepTree(p.treeType));
        return;
      }
    }
    cuCtx.violatesLfnst[0] = cuCtx.violatesLfnst[1] = false;
    cuCtx.lfnstLastScanPos = false;
    cuCtx.violatesMtsCoeffConstraint = false;
    cuCtx.mtsLastScanPos = false;
    if (c->isp && p.chType == 0) {
      TuState ts;
      ts.trDepth = p.trDepth;
      ts.cuArea = p.area();
      transform_tree_isp(p, ci, cuCtx, p.area(), ts.trDepth, c->isp == 1 ? ISP_H : ISP_V);
    } else {
      transform_tree(p, ci, cuCtx, p.area(), p.trDepth, p.partIdx(), -1);
    }
    residual_lfnst_mode(ci, cuCtx);
    mts_idx(ci, cuCtx);
  }
  struct TuState { int trDepth; Area cuArea; };

  // getMaxTuTiling (UnitPartitioner.cpp:1047)
  static std::vector<Area> maxTuTiling(const Area &a, int maxTbSize) {
    static const int zx[64] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3, 4, 5, 4, 5, 6, 7, 6, 7, 4, 5, 4, 5, 6, 7, 6, 7,
                               0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3, 4, 5, 4, 5, 6, 7, 6, 7, 4, 5, 4, 5, 6, 7, 6, 7};
    static const int zy[64] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3, 0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3,
                               4, 4, 5, 5, 4, 4, 5, 5, 6, 6, 7, 7, 6, 6, 7, 7, 4, 4, 5, 5, 4, 4, 5, 5, 6, 6, 7, 7, 6, 6, 7, 7};
    static const int rs2z[64] = {0, 1, 4, 5, 16, 17, 20, 21, 2, 3, 6, 7, 18, 19, 22, 23, 8, 9, 12, 13, 24, 25, 28, 29,
                                 10, 11, 14, 15, 26, 27, 30, 31, 32, 33, 36, 37, 48, 49, 52, 53, 34, 35, 38, 39, 50, 51, 54, 55,
                                 40, 41, 44, 45, 56, 57, 60, 61, 42, 43, 46, 47, 58, 59, 62, 63};
    const int mt = (a.w > 64 || a.h > 64) ? 64 : maxTbSize;
    const int nh = std::max(1, a.w / mt), nv = std::max(1, a.h / mt);
    std::vector<Area> r;
    for (int i = 0; i < nh * nv; i++) {
      const int rsy = i / nh, rsx = i % nh;
      const int z = rs2z[(rsy << 3) + rsx];
      const int w = a.w / nh, h = a.h / nv;
      r.push_back({a.x + w * zx[z], a.y + h * zy[z], w, h, a.cvalid});
    }
    return r;
  }
  // getSbtTuTiling (:1087)
  static std::vector<Area> sbtTiling(const Area &a, int split) {
    std::vector<Area> r;
    for (int i = 0; i < 2; i++) {
      int wf, hf, xo, yo;
      if (split >= SBT_VQ0) {
        if (split == SBT_HQ0 || split == SBT_HQ1) {
          wf = 4; xo = 0;
          hf = ((i == 0 && split == SBT_HQ0) || (i == 1 && split == SBT_HQ1)) ? 1 : 3;
          yo = i == 0 ? 0 : (split == SBT_HQ0 ? 1 : 3);
        } else {
          wf = ((i == 0 && split == SBT_VQ0) || (i == 1 && split == SBT_VQ1)) ? 1 : 3;
          xo = i == 0 ? 0 : (split == SBT_VQ0 ? 1 : 3);
          hf = 4; yo = 0;
        }
      } else {
        if (split == SBT_HH0 || split == SBT_HH1) { wf = 4; xo = 0; hf = 2; yo = i == 0 ? 0 : 2; }
        else { wf = 2; xo = i == 0 ? 0 : 2; hf = 4; yo = 0; }
      }
      // chroma and luma scale together in 4:2:0 (comp.x += comp.width * xo >> 2 per component)
      r.push_back({a.x + ((a.w * xo) >> 2), a.y + ((a.h * yo) >> 2), (a.w * wf) >> 2, (a.h * hf) >> 2, a.cvalid});
    }
    return r;
  }
  int sbtTuSplit(int sbtinfo) const {   // CodingUnit::getSbtTuSplit (Unit.cpp:505)
    const int idx = sbtinfo & 0xf, pos = (sbtinfo >> 4) & 3;
    switch (idx) {
      case SBT_VER_HALF: return SBT_VH0 + pos;
      case SBT_HOR_HALF: return SBT_HH0 + pos;
      case SBT_VER_QUAD: return SBT_VQ0 + pos;
      case SBT_HOR_QUAD: return SBT_HQ0 + pos;
    }
    return 0;
  }

  // transform_tree (:2550) for the QTBT partitioner path (max-TB and SBT splits)
  void transform_tree(Partitioner &p, int ci, CuCtx &cuCtx, const Area &a, int trDepth, int partIdx, int sbtLevel) {
    const vvcr_cu &c = pic.cu[ci];
    bool split = a.w > maxTb || a.h > maxTb;
    if (c.sbtinfo && trDepth == 0) split = true;
    if (split) {
      std::vector<Area> parts;
      bool isSbt = false;
      if (a.w > maxTb || a.h > maxTb) parts = maxTuTiling(a, maxTb);
      else { parts = sbtTiling(a, sbtTuSplit(c.sbtinfo)); isSbt = true; }
      for (int i = 0; i < (int)parts.size(); i++)
        transform_tree(p, ci, cuCtx, parts[i], trDepth + 1, i, isSbt ? 1 : 0);
      return;
    }
    const int ti = new_tu(ci, a, p.chType, isSepTree(p.treeType));
    vvcr_tu &t = pic.tu[ti];
    t.depth = trDepth;
    // TransformUnit::checkTuNoResidual (Unit.cpp:862)
    if ((c.sbtinfo & 0xf) != SBT_OFF && sbtLevel == 1) {
      const int pos = (c.sbtinfo >> 4) & 3;
      if ((pos == 0 && partIdx == 1) || (pos == 1 && partIdx == 0)) t.noresi = 1;
    }
    transform_unit(p, ci, ti, cuCtx, a, trDepth, -1, false);
  }
  // ISP path (TUIntraSubPartitioner, UnitPartitioner.cpp:660; getTUIntraSubPartitions :956)
  void transform_tree_isp(Partitioner &p, int ci, CuCtx &cuCtx, const Area &cuA, int trDepth, int ispType) {
    const vvcr_cu &c = pic.cu[ci];
    const bool dt = isSepTree(p.treeType);
    // CU::getISPSplitDim (UnitTools.cpp:376)
    const bool rows = ispType == ISP_H;
    const int splitDim = rows ? cuA.h : cuA.w, nonSplit = rows ? cuA.w : cuA.h;
    const int minSamples = 16;
    const int factor = nonSplit < minSamples ? minSamples >> floorLog2(nonSplit) : 1;
    const int part = (splitDim >> 2) < factor ? factor : (splitDim >> 2);
    const int n = splitDim >> floorLog2(part);
    (void)c;
    for (int i = 0; i < n; i++) {
      Area a = cuA;
      if (rows) { a.y = cuA.y + i * part; a.h = part; }
      else { a.x = cuA.x + i * part; a.w = part; }
      a.cvalid = dt ? false : (i == n - 1);
      // the chroma block of the last sub-partition covers the whole CU (chroma is not split)
      const int ti = new_tu(ci, a, p.chType, dt);
      vvcr_tu &t = pic.tu[ti];
      if (!dt && i == n - 1) {
        for (int cc = 1; cc < 3; cc++) { t.b[cc][0] = cuA.x >> 1; t.b[cc][1] = cuA.y >> 1; t.b[cc][2] = cuA.w >> 1; t.b[cc][3] = cuA.h >> 1; }
      }
      t.depth = trDepth + 1;
      transform_unit(p, ci, ti, cuCtx, a, trDepth + 1, i, true);
    }
  }

  unsigned cbf_comp(int ci, int comp, bool prevCbf, bool useISP) {   // CABACReader::cbf_comp (:2625)
    const vvcr_cu &c = pic.cu[ci];
    static const unsigned base[3] = {QtCbf0, QtCbf1, QtCbf2};
    unsigned ctx;
    if (useISP && comp == 0) ctx = 2 + (prevCbf ? 1 : 0);
    else if (comp == 2) ctx = prevCbf ? 1 : 0;
    else ctx = 0;
    if ((comp == 0 && c.bdpcm) || (comp != 0 && c.bdpcmc)) ctx = comp == 2 ? 2 : 1;
    return cab.bin(base[comp] + ctx);
  }

  static bool cbfAt(const vvcr_tu &t, int c, int d) { return (t.b[c][4] >> d) & 1; }
  static void setCbfAt(vvcr_tu &t, int c, int d, bool v) { t.b[c][4] &= ~(1 << d); t.b[c][4] |= (v ? 1 : 0) << d; }

  void transform_unit(Partitioner &p, int ci, int ti, CuCtx &cuCtx, const Area &a, int trDepth, int subTu, bool isp) {
    vvcr_cu &c = pic.cu[ci];
    vvcr_tu &t = pic.tu[ti];
    const bool sep = isSepTree(c.treetype);
    const bool cbValid = tuValid(t, 1);
    const bool chromaCbfISP = cbValid && c.isp;
    bool cbfCb = false, cbfCr = false;
    if (cbValid && (!sep || p.chType == 1) && (!c.isp || chromaCbfISP)) {
      if (!(c.sbtinfo && t.noresi)) cbfCb = cbf_comp(ci, 1, false, false);
      if (!(c.sbtinfo && t.noresi)) cbfCr = cbf_comp(ci, 2, cbfCb, false);
    }
    const bool sigChroma = cbfCb || cbfCr;
    if (p.chType == 0) {
      if (c.predmode != MODE_INTRA && trDepth == 0 && !sigChroma) setCbfAt(t, 0, trDepth, true);
      else if (c.sbtinfo && t.noresi) setCbfAt(t, 0, trDepth, false);
      else if (c.sbtinfo && !sigChroma) setCbfAt(t, 0, trDepth, true);
      else {
        bool lastInferred = false, prevCbf = false;
        if (c.isp) {
          const int nTus = c.isp == 1 ? c.h >> floorLog2(t.b[0][3]) : c.w >> floorLog2(t.b[0][2]);
          if (subTu == nTus - 1) {
            bool rootSoFar = false;
            for (int k = 0; k < nTus - 1; k++) rootSoFar |= cbfAt(pic.tu[c.firsttu + k], 0, trDepth);
            if (!rootSoFar) lastInferred = true;
          }
          if (!lastInferred && ti > c.firsttu) prevCbf = cbfAt(pic.tu[ti - 1], 0, trDepth);
        }
        const bool cbfY = lastInferred ? true : cbf_comp(ci, 0, prevCbf, c.isp != 0) != 0;
        setCbfAt(t, 0, trDepth, cbfY);
      }
    }
    if (!c.isp || chromaCbfISP) {
      if (cbValid) {
        setCbfAt(t, 1, trDepth, cbfCb);
        setCbfAt(t, 2, trDepth, cbfCr);
      }
    }
    const bool lumaOnly = !cbValid;
    const bool cbfLuma = t.b[0][4] != 0;
    const bool cbfChroma = lumaOnly ? false : sigChroma;
    if ((c.w > 64 || c.h > 64 || cbfLuma || cbfChroma) && (!sep || t.chtype == 0)) {
      if (pps.useDQP && !cuCtx.isDQPCoded) {
        c.qp = cu_qp_delta(cuCtx.qp);
        cuCtx.qp = c.qp;
        cuCtx.isDQPCoded = true;
      }
    }
    if (!sep || t.chtype == 1) {
      const int cw = !sep ? c.w : c.cw, chh = !sep ? c.h : c.ch;
      if (sh.chromaQpAdj && (cw > 64 || chh > 64 || cbfChroma) && !cuCtx.isChromaQpAdjCoded) {
        int adj = cab.bin(ChromaQpAdjFlag);
        if (adj && pps.chromaQpOffsetListLen > 1) {
          unsigned ones = 0;
          while (ones < (unsigned)pps.chromaQpOffsetListLen - 1 && cab.bin(ChromaQpAdjIdc)) ++ones;
          adj += ones;
        }
        c.cqpadj = chromaQpAdj = adj;
        cuCtx.isChromaQpAdjCoded = true;
      }
    }
    if (!lumaOnly && sps.jointCbCr) {   // joint_cb_cr (:2904)
      const int mask = (t.b[1][4] ? 2 : 0) + (t.b[2][4] ? 1 : 0);
      if ((c.predmode == MODE_INTRA && mask) || mask == 3) t.jccr = cab.bin(JointCbCrFlag + mask - 1) ? mask : 0;
    }
    (void)isp;
    // coefficient levels: decoded into the zeroed scratch block, then the bounding box of the non-zero
    // levels goes into the picture's pool (a block per coded component, and per chroma component of a
    // joint Cb-Cr TU, in component order); the scratch is zeroed again
    if (pic.box.size() < 3 * (size_t)(ti + 1)) pic.box.resize(3 * (size_t)(ti + 1), 0);
    for (int comp = 0; comp < 3; comp++) {
      vvcr_tu &tt = pic.tu[ti];
      if (!tuValid(tt, comp) || !(tt.b[comp][4] || (comp > 0 && tt.jccr))) continue;
      const int w = tt.b[comp][2];
      const bool coded = comp == 0 ? cbfLuma : (!lumaOnly && tt.b[comp][4]);
      boxR = boxC = 0;
      lvl = scratch;
      lvlStride = w;
      if (coded) residual_coding(ci, ti, comp, cuCtx);
      const size_t off = pic.coef.size();
      tt.b[comp][6] = (int32_t)off;
      pic.box[3 * (size_t)ti + comp] = (uint16_t)(boxR | boxC << 8);
      if (boxR && boxC) {
        // one resize (its zero fill is a memset), then the box's rows copied in (a per-row vector insert runs
        // the allocator's element-wise copy loop: 3 % of an intra picture's parse)
        const size_t need = off + (size_t)boxR * boxC;
        if (need > pic.coef.capacity()) pic.coef.reserve(std::max(need, 2 * pic.coef.capacity()));
        pic.coef.resize(need);
        int32_t *dst = pic.coef.data() + off;
        for (int y = 0; y < boxR; y++, dst += boxC) {
          int32_t *src = lvl + y * lvlStride;
          std::memcpy(dst, src, (size_t)boxC * sizeof(int32_t));
          std::memset(src, 0, (size_t)boxC * sizeof(int32_t));
        }
      }
    }
  }
  alignas(64) int32_t scratch[64 * 64] = {};   // one transform block's levels, zero between blocks
  alignas(64) int32_t pscratch[kPS * kPS] = {}; // the same, padded (regular residual path: kPS)
  int32_t *lvl = scratch;                       // the block the last residual_coding wrote, and its stride
  int lvlStride = 0;
  int boxR = 0, boxC = 0;                      // bounding box of its non-zero levels (rows, columns)

  int cu_qp_delta(int predQP) {   // CABACReader::cu_qp_delta (:2850)
    int dqp = 0;
    while (dqp < 5 && cab.bin(dqp == 0 ? DeltaQP : DeltaQP + 1)) ++dqp;
    if (dqp >= 5) {   // exp_golomb_eqprob(0)
      unsigned sym = 0, bit = 1, count = 0;
      while (bit) { bit = cab.ep(); sym += bit << count++; }
      if (--count) sym += cab.eps(count);
      dqp += (int)sym;
    }
    int qpY = predQP;
    if (dqp > 0) {
      if (cab.ep()) dqp = -dqp;
      const int off = sps.qpBdOffset;
      qpY = ((predQP + dqp + 64 + 2 * off) % (64 + off)) - off;
    }
    return qpY;
  }

  // TU::isTSAllowed (UnitTools.cpp:3897)
  bool tsAllowed(const vvcr_cu &c, const vvcr_tu &t, int comp) const {
    const int tsMax = 1 << pps.log2MaxTs;
    bool ok = sps.transformSkip;
    ok &= !c.isp || comp != 0;
    ok &= !(c.bdpcm && comp == 0);
    ok &= !(c.bdpcmc && comp != 0);
    ok &= t.b[comp][2] <= tsMax && t.b[comp][3] <= tsMax;
    ok &= !c.sbtinfo;
    return ok;
  }

  // residual_coding (:2918)
  void residual_coding(int ci, int ti, int comp, CuCtx &cuCtx) {   // into lvl (zeroed), set here
    const vvcr_cu &c = pic.cu[ci];
    vvcr_tu &t = pic.tu[ti];
    const int w = t.b[comp][2], h = t.b[comp][3];
    if (comp == 2 && t.jccr == 3) return;
    // ts_flag (:3007)
    int ts = ((c.bdpcm && comp == 0) || (c.bdpcmc && comp != 0)) ? 1 : (t.b[comp][5] == MTS_SKIP ? 1 : 0);
    if (tsAllowed(c, t, comp)) ts = cab.bin(TransformSkipFlag + (comp == 0 ? 0 : 1));
    t.b[comp][5] = ts ? MTS_SKIP : MTS_DCT2;
    if (ts) { lvl = scratch; lvlStride = w; residual_codingTS(c, comp, w, h, scratch); boxR = h; boxC = w; return; }
    lvl = pscratch;
    lvlStride = kPS;
    int32_t *coeff = pscratch;
    const bool signHiding = ph.signHiding;
    CoefCtx cc(comp, w, h, signHiding, false);
    CabacLocal cb(cab);   // the engine's registers as locals through the level loops (vvcp_core.h)
    cc.scanPosLast = last_sig_coeff(cb, cc, c, comp, w, h);
    if (h >= 4 && w >= 4) {
      const int maxLfnstPos = ((h == 4 && w == 4) || (h == 8 && w == 8)) ? 7 : 15;
      cuCtx.violatesLfnst[comp ? 1 : 0] |= cc.scanPosLast > maxLfnstPos;
      cuCtx.lfnstLastScanPos |= cc.scanPosLast >= 1;
    }
    if (comp == 0) cuCtx.mtsLastScanPos |= cc.scanPosLast >= 1;
    const int stateTab = ph.depQuant ? 32040 : 0;
    int state = 0;
    int tbW = w, tbH = h;
    if (sps.mts && c.sbtinfo && w <= 32 && h <= 32 && comp == 0) { tbW = w == 32 ? 16 : w; tbH = h == 32 ? 16 : h; }
    tbW = std::min(32, tbW); tbH = std::min(32, tbH);
    cc.regBinLimit = (tbW * tbH * 28) >> 4;
    for (int sub = cc.scanPosLast >> cc.log2CG; sub >= 0; sub--) {
      cc.initSubblock(sub);
      if (sps.mts && c.sbtinfo && h <= 32 && w <= 32 && comp == 0) {
        if ((h == 32 && cc.subSetPosY >= (16 >> cc.log2CGh)) || (w == 32 && cc.subSetPosX >= (16 >> cc.log2CGw))) continue;
      }
      residual_coding_subblock(cb, cc, coeff, stateTab, state);
      if (comp == 0 && cc.isSigGroup() && (cc.subSetPosY > 3 || cc.subSetPosX > 3)) cuCtx.violatesMtsCoeffConstraint = true;
    }
    cb.store(cab);
  }
  int last_sig_coeff(CabacLocal &cab, CoefCtx &cc, const vvcr_cu &c, int comp, int w, int h) {   // :3168
    unsigned px = 0, py = 0;
    unsigned mx = cc.maxLastPosX, my = cc.maxLastPosY;
    if (sps.mts && c.sbtinfo && w <= 32 && h <= 32 && comp == 0) {
      mx = w == 32 ? kGroupIdx[15] : mx;
      my = h == 32 ? kGroupIdx[15] : my;
    }
    for (; px < mx; px++)
      if (!cab.bin(cc.lastXCtx(px))) break;
    for (; py < my; py++)
      if (!cab.bin(cc.lastYCtx(py))) break;
    if (px > 3) {
      uint32_t tmp = 0;
      const int cnt = (px - 2) >> 1;
      for (int i = cnt - 1; i >= 0; i--) tmp += cab.ep() << i;
      px = kMinInGroup[px] + tmp;
    }
    if (py > 3) {
      uint32_t tmp = 0;
      const int cnt = (py - 2) >> 1;
      for (int i = cnt - 1; i >= 0; i--) tmp += cab.ep() << i;
      py = kMinInGroup[py] + tmp;
    }
    return cc.scanInv[px + py * w];   // the scan position of (px, py): first match, else the last position
  }
  void residual_coding_subblock(CabacLocal &cab, CoefCtx &cc, int32_t *coeff, int stateTab, int &state) {   // :3235 (cab: the local engine)
    const int minSubPos = cc.minSubPos;
    const bool isLast = cc.isLast();
    const int firstSigPos = isLast ? cc.scanPosLast : cc.maxSubPos;
    int nextSigPos = firstSigPos;
    bool sigGroup = isLast || !minSubPos;
    if (!sigGroup) sigGroup = cab.bin(cc.sigGroupCtx);
    if (!sigGroup) return;
    cc.setSigGroup();
    uint8_t ctxOffset[16];
    const int inferSigPos = nextSigPos != cc.scanPosLast ? (cc.subSetId != 0 ? minSubPos : -1) : nextSigPos;
    int firstNZPos = nextSigPos, lastNZPos = -1, numNonZero = 0;
    int remRegBins = cc.regBinLimit;
    int sigBlkPos[16];
    for (; nextSigPos >= minSubPos && remRegBins >= 4; nextSigPos--) {
      const int blkPos = cc.pscan[nextSigPos];   // (padded block)
      unsigned sigFlag = (!numNonZero && nextSigPos == inferSigPos);
      if (!sigFlag) {
        const unsigned ctx = cc.sigCtxIdAbs(nextSigPos, coeff, state);
        sigFlag = cab.bin(ctx);
        remRegBins--;
      } else if (nextSigPos != cc.scanPosLast) {
        cc.sigCtxIdAbs(nextSigPos, coeff, state);
      }
      if (sigFlag) {
        uint8_t &off = ctxOffset[nextSigPos - minSubPos];
        off = cc.ctxOffsetAbs();
        sigBlkPos[numNonZero++] = blkPos;
        firstNZPos = nextSigPos;
        lastNZPos = std::max(lastNZPos, nextSigPos);
        const unsigned gt1 = cab.bin(cc.gtxSet[1] + off);
        remRegBins--;
        unsigned par = 0, gt2 = 0;
        if (gt1) {
          par = cab.bin(cc.parSet + off);
          remRegBins--;
          gt2 = cab.bin(cc.gtxSet[0] + off);
          remRegBins--;
        }
        coeff[blkPos] += 1 + par + gt1 + (gt2 << 1);
      }
      state = (stateTab >> ((state << 2) + ((coeff[blkPos] & 1) << 1))) & 3;
    }
    const int firstPosMode2 = nextSigPos;
    cc.regBinLimit = remRegBins;
    for (int sp = firstSigPos; sp > firstPosMode2; sp--) {
      const int sumAll = (int)cc.templateAbsSum(sp, coeff, 4);
      const unsigned rice = kGoRiceParsCoeff[sumAll];
      int32_t &tc = coeff[cc.pscan[sp]];
      if (tc >= 4) {
        const int rem = (int)cab.rem_abs(rice, 5, 15);
        tc += rem << 1;
      }
    }
    for (int sp = firstPosMode2; sp >= minSubPos; sp--) {
      const int sumAll = (int)cc.templateAbsSum(sp, coeff, 0);
      const unsigned rice = kGoRiceParsCoeff[sumAll];
      const int pos0 = (state < 2 ? 1 : 2) << rice;
      const int rem = (int)cab.rem_abs(rice, 5, 15);
      const int tc = rem == pos0 ? 0 : (rem < pos0 ? rem + 1 : rem);
      state = (stateTab >> ((state << 2) + ((tc & 1) << 1))) & 3;
      if (tc) {
        const int blkPos = cc.pscan[sp];
        sigBlkPos[numNonZero++] = blkPos;
        firstNZPos = sp;
        lastNZPos = std::max(lastNZPos, sp);
        coeff[blkPos] = tc;
      }
    }
    for (int k = 0; k < numNonZero; k++) {
      const int r = sigBlkPos[k] / kPS;
      boxR = std::max(boxR, r + 1);
      boxC = std::max(boxC, sigBlkPos[k] - r * kPS + 1);
    }
    const unsigned numSigns = (cc.signHiding && (lastNZPos - firstNZPos >= 4)) ? numNonZero - 1 : numNonZero;
    unsigned signPattern = numSigns ? cab.eps(numSigns) << (32 - numSigns) : 0;
    int sumAbs = 0;
    for (unsigned k = 0; k < numSigns; k++) {
      const int ac = coeff[sigBlkPos[k]];
      sumAbs += ac;
      coeff[sigBlkPos[k]] = (signPattern & (1u << 31)) ? -ac : ac;
      signPattern <<= 1;
    }
    if ((unsigned)numNonZero > numSigns) {
      const int k = numSigns;
      const int ac = coeff[sigBlkPos[k]];
      sumAbs += ac;
      coeff[sigBlkPos[k]] = (sumAbs & 1) ? -ac : ac;
    }
  }
  void residual_codingTS(const vvcr_cu &c, int comp, int w, int h, int32_t *coeff) {   // :3393
    CoefCtx cc(comp, w, h, false, comp == 0 ? c.bdpcm != 0 : c.bdpcmc != 0);
    cc.numCtxBins = (cc.maxNumCoeff * 7) >> 2;
    const int last = (cc.maxNumCoeff - 1) >> cc.log2CG;
    for (int sub = 0; sub <= last; sub++) {
      cc.initSubblock(sub);
      residual_coding_subblockTS(cc, coeff, sub == last);
    }
  }
  void residual_coding_subblockTS(CoefCtx &cc, int32_t *coeff, bool isLastSubSet) {   // :3410
    const int minSubPos = cc.maxSubPos;   // (sic) the reference swaps the names here
    const int firstSigPos = cc.minSubPos;
    int nextSigPos = firstSigPos;
    unsigned signPattern = 0;
    bool sigGroup = isLastSubSet && cc.sigCG == 0;
    if (!sigGroup) sigGroup = cab.bin(cc.sigGroupCtxTS);
    if (!sigGroup) return;
    cc.setSigGroup();
    const int inferSigPos = minSubPos;
    int numNonZero = 0;
    int sigBlkPos[16];
    int lastPass1 = -1, lastPass2 = -1;
    for (; nextSigPos <= minSubPos && cc.numCtxBins >= 4; nextSigPos++) {
      const int blkPos = cc.scan[nextSigPos].idx;
      unsigned sig = (!numNonZero && nextSigPos == inferSigPos);
      if (!sig) {
        sig = cab.bin(cc.sigCtxIdAbsTS(nextSigPos, coeff));
        cc.numCtxBins--;
      }
      if (sig) {
        const int sign = (int)cab.bin(cc.signCtxIdAbsTS(nextSigPos, coeff));
        cc.numCtxBins--;
        signPattern += sign << numNonZero;
        sigBlkPos[numNonZero++] = blkPos;
        const unsigned gt1 = cab.bin(cc.lrg1CtxIdAbsTS(nextSigPos, coeff));
        cc.numCtxBins--;
        unsigned par = 0;
        if (gt1) {
          par = cab.bin(TsParFlag);
          cc.numCtxBins--;
        }
        coeff[blkPos] = (sign ? -1 : 1) * (int)(1 + par + gt1);
      }
      lastPass1 = nextSigPos;
    }
    for (int sp = firstSigPos; sp <= minSubPos && cc.numCtxBins >= 4; sp++) {
      int32_t &tc = coeff[cc.scan[sp].idx];
      int cutoff = 2;
      for (int i = 0; i < 4; i++) {
        if (tc < 0) tc = -tc;
        if (tc >= cutoff) {
          const unsigned g = cab.bin(TsGtxFlag + (cutoff >> 1));
          tc += g << 1;
          cc.numCtxBins--;
        }
        cutoff += 2;
      }
      lastPass2 = sp;
    }
    for (int sp = firstSigPos; sp <= minSubPos; sp++) {
      int32_t &tc = coeff[cc.scan[sp].idx];
      const int cutoff = sp <= lastPass2 ? 10 : (sp <= lastPass1 ? 2 : 0);
      if (tc < 0) tc = -tc;
      if (tc >= cutoff) {
        const int rem = (int)cab.rem_abs(1, 5, 15);
        tc += sp <= lastPass1 ? (rem << 1) : rem;
        if (tc && sp > lastPass1) {
          const int blkPos = cc.scan[sp].idx;
          const int sign = (int)cab.ep();
          signPattern += sign << numNonZero;
          sigBlkPos[numNonZero++] = blkPos;
        }
      }
      if (!cc.bdpcm && cutoff) {
        if (tc > 0) {
          int r, b;
          cc.neighTS(r, b, sp, coeff);
          tc = CoefCtx::decDeriveModCoeff(r, b, tc);
        }
      }
    }
    for (int k = 0; k < numNonZero; k++) {
      const int ac = coeff[sigBlkPos[k]];
      coeff[sigBlkPos[k]] = (signPattern & 1) ? -ac : ac;
      signPattern >>= 1;
    }
  }

  // residual_lfnst_mode (:3106)
  void residual_lfnst_mode(int ci, CuCtx &cuCtx) {
    vvcr_cu &c = pic.cu[ci];
    const bool sep = isSepTree(c.treetype);
    const int chIdx = sep && c.chtype == 1 ? 1 : 0;
    if (c.isp) {   // CU::canUseLfnstWithISP (UnitTools.cpp:354)
      const int part = ispPart(c);
      const int tw = c.isp == 1 ? c.w : part, th = c.isp == 1 ? part : c.h;
      if (!(tw >= 4 && th >= 4)) return;
    }
    if (sps.lfnst && c.predmode == MODE_INTRA && c.mip && !(c.w >= 16 && c.h >= 16)) return;
    if (sep && c.chtype == 1 && std::min(c.cw, c.ch) < 4) return;
    const int bw = chIdx ? c.cw << 1 : c.w, bh = chIdx ? c.ch << 1 : c.h;
    if (bw > maxTb || bh > maxTb) return;
    if (sps.lfnst && c.predmode == MODE_INTRA) {
      const bool lumaFlag = sep ? c.chtype == 0 : true, chromaFlag = sep ? c.chtype == 1 : true;
      const bool nz = (lumaFlag && cuCtx.violatesLfnst[0]) || (chromaFlag && cuCtx.violatesLfnst[1]);
      bool isTrSkip = false;
      for (int k = 0; k < c.ntu && !isTrSkip; k++) {
        const vvcr_tu &t = pic.tu[c.firsttu + k];
        for (int comp = 0; comp < 3; comp++)
          if (tuValid(t, comp) && cbfAt(t, comp, t.depth) && t.b[comp][5] == MTS_SKIP) { isTrSkip = true; break; }
      }
      if ((!cuCtx.lfnstLastScanPos && !c.isp) || nz || isTrSkip) { c.lfnst = 0; return; }
    } else {
      c.lfnst = 0;
      return;
    }
    unsigned ctx = sep ? 1 : 0;
    int idx = cab.bin(LFNSTIdx + ctx);
    if (idx) idx += cab.bin(LFNSTIdx + 2);
    c.lfnst = idx;
  }
  int ispPart(const vvcr_cu &c) const {
    const bool rows = c.isp == 1;
    const int splitDim = rows ? c.h : c.w, nonSplit = rows ? c.w : c.h;
    const int factor = nonSplit < 16 ? 16 >> floorLog2(nonSplit) : 1;
    return (splitDim >> 2) < factor ? factor : (splitDim >> 2);
  }
  // mts_idx (:3023), CU::isMTSAllowed (UnitTools.cpp:3854)
  void mts_idx(int ci, CuCtx &cuCtx) {
    vvcr_cu &c = pic.cu[ci];
    vvcr_tu &t = pic.tu[c.firsttu];
    int mts = t.b[0][5];
    const int tsMax = 1 << pps.log2MaxTs;
    bool allowed = c.chtype == 0;
    allowed &= c.predmode == MODE_INTRA ? sps.intraMts : (sps.interMts && c.predmode == MODE_INTER);
    allowed &= c.w <= 32 && c.h <= 32;
    allowed &= !c.isp;
    allowed &= !c.sbtinfo;
    allowed &= !(c.bdpcm && c.w <= tsMax && c.h <= tsMax);
    if (allowed && !cuCtx.violatesMtsCoeffConstraint && cuCtx.mtsLastScanPos && c.lfnst == 0 && mts != MTS_SKIP) {
      int sym = cab.bin(MTSIdx);
      if (sym) {
        mts = MTS_DST7;
        for (int i = 0, k = 1; i < 3; i++, k++) {
          sym = cab.bin(MTSIdx + k);
          mts += sym;
          if (!sym) break;
        }
      }
    }
    t.b[0][5] = mts;
  }

  // ------------------------------------------------------------------------------------------------
  // CTU level: coding_tree_unit (:136), sao (:318), ALF / CC-ALF CTB flags
  // ------------------------------------------------------------------------------------------------
  void sao(int ctu) {
    vvcr_sao *s = &shp.sao[(size_t)ctu * 3];
    for (int c = 0; c < 3; c++) s[c].mode = 0;
    if (!sps.sao) return;
    const bool lumaF = sh.sao[0], chromaF = sh.sao[1];
    if (!lumaF && !chromaF) return;
    const int ry = ctu / pic.wCtu, rx = ctu - ry * pic.wCtu;
    const int px = rx << pic.ctuLog2, py = ry << pic.ctuLog2;
    int mergeType = -1;
    if (cuRestricted(0, px - pic.ctuSize, py, sc.sliceIdx, curTile) >= 0) mergeType += (int)cab.bin(SaoMergeFlag);
    if (mergeType < 0 && cuRestricted(0, px, py - pic.ctuSize, sc.sliceIdx, curTile) >= 0) mergeType += (int)cab.bin(SaoMergeFlag) << 1;
    if (mergeType >= 0) {
      s[0].mode = 2; s[0].type = mergeType;
      if (chromaF) { s[1].mode = s[2].mode = 2; s[1].type = s[2].type = mergeType; }
      return;
    }
    const int first = lumaF ? 0 : 1, last = chromaF ? 2 : 0;
    const int maxOff = (1 << (std::min(sps.bitDepth, 10) - 5)) - 1;
    for (int comp = first; comp <= last; comp++) {
      vvcr_sao &o = s[comp];
      if (comp != 2) {
        if (cab.bin(SaoTypeIdx)) {
          o.mode = 1;
          o.type = cab.ep() ? 0 : 4;
        }
      } else {
        o.mode = s[1].mode;
        o.type = s[1].type;
      }
      if (o.mode == 0) continue;
      int off[4];
      for (int k = 0; k < 4; k++) off[k] = (int)unary_max_eqprob(maxOff);
      std::memset(o.offset, 0, sizeof(o.offset));
      if (o.type == 4) {
        for (int k = 0; k < 4; k++)
          if (off[k] && cab.ep()) off[k] = -off[k];
        o.band = (int)cab.eps(5);
        for (int k = 0; k < 4; k++) o.offset[(o.band + k) % 32] = off[k];
        continue;
      }
      o.band = 0;
      if (comp != 2) o.type += (int)cab.eps(2);
      else o.type = s[1].type;
      o.offset[0] = off[0];
      o.offset[1] = off[1];
      o.offset[2] = 0;
      o.offset[3] = -off[2];
      o.offset[4] = -off[3];
    }
  }

  void alf_ctb(int ctu) {
    const int ry = ctu / pic.wCtu, rx = ctu - ry * pic.wCtu;
    const int px = rx << pic.ctuLog2, py = ry << pic.ctuLog2;
    if (sps.alf && sh.alf[0]) {
      const bool la = cuRestricted(0, px - pic.ctuSize, py, sc.sliceIdx, curTile) >= 0;
      const bool aa = cuRestricted(0, px, py - pic.ctuSize, sc.sliceIdx, curTile) >= 0;
      const int left = la ? ctu - 1 : -1, above = aa ? ctu - pic.wCtu : -1;
      for (int comp = 0; comp < 3; comp++) {
        if (!sh.alf[comp]) continue;
        std::vector<uint8_t> &en = shp.alfEn[comp];
        int ctx = (left >= 0 && en[left] ? 1 : 0) + (above >= 0 && en[above] ? 1 : 0);
        en[ctu] = (uint8_t)cab.bin(ctbAlfFlag + comp * 3 + ctx);
        if (comp == 0 && en[ctu]) {   // readAlfCtuFilterIndex (:245)
          const unsigned numAps = sh.numAlfAps, avail = numAps + 16;
          uint32_t idx = 0;
          if (avail > 16) {
            if (cab.bin(AlfUseTemporalFilt)) {
              if (numAps > 1) idx = truncBin(avail - 16);
              idx += 16;
            } else idx = truncBin(16);
          } else idx = truncBin(16);
          shp.alfFset[ctu] = (int16_t)idx;
        }
        if (comp > 0) {
          const APS &aps = sc.ps->alfAps[sh.alfApsChroma];
          VVCP_CHECK(!sc.ps->alfValid[sh.alfApsChroma], "chroma ALF APS missing");
          const int numAlts = aps.alf.numAltChroma;
          shp.alfAlt[comp][ctu] = 0;
          if (en[ctu]) {
            uint8_t d = 0;
            while (d < numAlts - 1 && cab.bin(ctbAlfAlternative + comp - 1)) ++d;
            shp.alfAlt[comp][ctu] = d;
          }
        }
      }
    }
    if (sps.ccalf) {
      for (int comp = 1; comp < 3; comp++) {
        if (!sh.ccAlf[comp - 1]) continue;
        VVCP_CHECK(!sc.ps->alfValid[sh.ccAlfApsId[comp - 1]], "CC-ALF APS missing");
        const int count = sc.ps->alfAps[sh.ccAlfApsId[comp - 1]].alf.ccCount[comp - 1];
        const bool la = cuRestricted(0, px - pic.ctuSize, py, sc.sliceIdx, curTile) >= 0;
        const bool aa = cuRestricted(0, px, py - pic.ctuSize, sc.sliceIdx, curTile) >= 0;
        std::vector<uint8_t> &ctl = shp.ccCtl[comp - 1];
        int ctx = 0;
        if (la) ctx += ctl[ctu - 1] ? 1 : 0;
        if (aa) ctx += ctl[ctu - pic.wCtu] ? 1 : 0;
        ctx += comp == 2 ? 3 : 0;
        int v = (int)cab.bin(CcAlfFilterControlF + ctx);
        if (v)
          while (v != count && cab.ep()) v++;
        ctl[ctu] = (uint8_t)v;
      }
    }
  }

  void coding_tree_unit(int ctu, int qps[2]) {
    const int ry = ctu / pic.wCtu, rx = ctu - ry * pic.wCtu;
    Area a{rx << pic.ctuLog2, ry << pic.ctuLog2, pic.ctuSize, pic.ctuSize, true};
    CuCtx cuCtx;
    cuCtx.qp = qps[0];
    Partitioner p;
    p.initCtu(a, 0);
    sao(ctu);
    alf_ctb(ctu);
    if (dualTree && pic.ctuSize > 64) {
      Partitioner pc;
      pc.initCtu(a, 1);
      CuCtx cuCtxC;
      cuCtxC.qp = qps[1];
      coding_tree(p, cuCtx, &pc, &cuCtxC);
      qps[0] = cuCtx.qp;
      qps[1] = cuCtxC.qp;
    } else {
      coding_tree(p, cuCtx);
      qps[0] = cuCtx.qp;
      if (dualTree) {
        CuCtx cuCtxC;
        cuCtxC.qp = qps[1];
        p.initCtu(a, 1);
        coding_tree(p, cuCtxC);
        qps[1] = cuCtxC.qp;
      }
    }
  }

  // CABACReader::initCtxModels (:66)
  void init_ctx() {
    int t = sh.sliceType;   // B 0, P 1, I 2
    if (pps.cabacInitPresent && sh.cabacInit) t = t == 1 ? 0 : (t == 0 ? 1 : t);
    cab.init_contexts(sh.qp, t);
  }

  // DecSlice::decompressSlice (DecSlice.cpp:73) over the slice's CTUs [i0, i1) (indices into sh.ctus),
  // the first of which starts substream ss (a tile start, or the slice's first CTU)
  void run(const uint8_t *data, size_t n, const std::vector<uint32_t> &nal_epb, int i0, int i1, size_t ss) {
    // substream boundaries: entry points count emulation-prevention bytes (VLCReader.cpp:3316-3349)
    std::vector<size_t> starts;
    {
      const size_t d0 = sh.dataOffset;
      size_t endSH = d0 + 2;   // byte location in the NAL (header included)
      for (uint32_t e : nal_epb)
        if (e < endSH) endSH++;
      size_t cur = 0, prev = 0, pos = d0;
      starts.push_back(d0);
      for (uint32_t ep : sh.entryPoints) {
        cur += ep;
        size_t cnt = 0;
        for (uint32_t e : nal_epb)
          if (e >= prev + endSH && e < cur + endSH) cnt++;
        pos += ep - cnt;
        prev = cur;
        starts.push_back(pos);
      }
    }
    VVCP_CHECK(starts.back() > n, "entry point beyond the slice data");
    VVCP_CHECK(ss >= starts.size(), "missing entry point");
    auto substreamEnd = [&](size_t k) { return k + 1 < starts.size() ? starts[k + 1] : n; };
    init_ctx();
    cab.start(data + starts[ss], data + substreamEnd(ss));
    int qps[2] = {sh.qp, sh.qp};
    const int nCtu = (int)sh.ctus.size();
    const bool wpp = pps.entropySync;
    // WPP (entropy_coding_sync): the context state after the first CTU of each CTU row of a tile, which the
    // next row's first CTU starts from when the CTU above it is in the same slice and tile
    // (DecSlice.cpp:160-176, stored at :214-219)
    std::vector<CtxModel> syncCtx;
    for (int i = i0; i < i1; i++) {
      const int ctu = sh.ctus[i];
      const int cx = ctu % pic.wCtu, cy = ctu / pic.wCtu;
      const int tc = pps.ctuToTileCol[cx], tr = pps.ctuToTileRow[cy];
      const int tx0 = pps.colBd[tc], ty0 = pps.rowBd[tr];
      const int tw = pps.colBd[tc + 1] - tx0, th = pps.rowBd[tr + 1] - ty0;
      curTile = pps.tileIdx(cx, cy);
      curCtu = ctu;
      if (cx == tx0 && cy == ty0) {
        if (i != i0) {
          init_ctx();
          cab.start(data + starts[ss], data + substreamEnd(ss));
        }
        qps[0] = qps[1] = sh.qp;
      } else if (cx == tx0 && wpp) {
        if (i != i0) {
          init_ctx();
          cab.start(data + starts[ss], data + substreamEnd(ss));
        }
        // the CTU above in the same slice and tile (CodingStructure::getCURestricted of (x, y - 1))
        if (!syncCtx.empty() && cuRestricted(0, cx << pic.ctuLog2, (cy << pic.ctuLog2) - 1, sc.sliceIdx, curTile) >= 0)
          std::copy(syncCtx.begin(), syncCtx.end(), cab.ctx);
        qps[0] = qps[1] = sh.qp;
      }
      ctuHmvpReset = !sh.isIntra() && cx == tx0;
      firstCuOfCtu = true;
      coding_tree_unit(ctu, qps);
      if (cx == tx0 && wpp) syncCtx.assign(cab.ctx, cab.ctx + vvcp_ctx::NUM_CTX);
      if (i == nCtu - 1) {
        VVCP_CHECK(!cab.trm(), "missing end_of_slice terminating bit");
      } else if (cx + 1 == tx0 + tw && (cy + 1 == ty0 + th || wpp)) {
        // end of a tile, or with WPP of a CTU row of the tile: the substream ends
        VVCP_CHECK(!cab.trm(), "missing end_of_tile / end_of_subset terminating bit");
        ss++;
        VVCP_CHECK(ss >= starts.size(), "missing entry point");
      }
    }
  }
};

}  // namespace

void PictureSyntax::reset(int W_, int H_, int ctuLog2_, bool intra) {
  W = W_; H = H_; ctuLog2 = ctuLog2_; ctuSize = 1 << ctuLog2;
  wCtu = (W + ctuSize - 1) >> ctuLog2;
  hCtu = (H + ctuSize - 1) >> ctuLog2;
  w4 = (W + 3) >> 2;
  h4 = (H + 3) >> 2;
  cu.clear(); cux.clear(); pu.clear(); pux.clear(); tu.clear(); coef.clear(); box.clear();
  // room for a quarter of the samples' levels (the packed boxes of a typical inter picture), three
  // quarters for an intra picture (the 4K QP27 I picture: 4.5 M of 8.3 M); more grows the pool (the blocks come from the
  // large-buffer cache, page-locked once a reconstruction context exists)
  coef.reserve((size_t)W * H / 4 * (intra ? 3 : 1) + 65536);
  // rows: room for a densely coded intra picture (one CU per 64 luma samples), so that the vectors do not
  // grow by reallocation (copying every row) while the CABAC pass appends; larger counts still grow
  const size_t rows = (size_t)W * H / 64 + 1024;
  cu.reserve(rows); cux.reserve(rows); pu.reserve(rows); pux.reserve(rows); tu.reserve(rows + rows / 2);
  map[0].assign((size_t)w4 * h4, -1);
  map[1].clear();
  mapShared = true;
  const size_t n = (size_t)wCtu * hCtu;
  sao.assign(n * 3, vvcr_sao());
  for (int c = 0; c < 3; c++) { alfEn[c].assign(n, 0); alfAlt[c].assign(n, 0); }
  for (int c = 0; c < 2; c++) ccCtl[c].assign(n, 0);
  alfFset.assign(n, 0);
}

void PictureSyntax::reset_rows(const PictureSyntax &o, size_t samples) {
  W = o.W; H = o.H; ctuLog2 = o.ctuLog2; ctuSize = o.ctuSize; wCtu = o.wCtu; hCtu = o.hCtu; w4 = o.w4; h4 = o.h4;
  cu.clear(); cux.clear(); pu.clear(); pux.clear(); tu.clear(); coef.clear(); box.clear();
  coef.reserve(samples / 4 + 4096);
  const size_t rows = samples / 64 + 256;
  cu.reserve(rows); cux.reserve(rows); pu.reserve(rows); pux.reserve(rows); tu.reserve(rows + rows / 2);
}

void PictureSyntax::dense_rows(std::vector<vvcr_tu> &tus, std::vector<int32_t> &pool) const {
  tus.assign(tu.begin(), tu.end());
  size_t n = 0;
  for (const vvcr_tu &t : tu)
    for (int c = 0; c < 3; c++)
      if (t.b[c][6] >= 0) n += (size_t)t.b[c][2] * t.b[c][3];
  pool.assign(n, 0);
  size_t off = 0;
  for (size_t i = 0; i < tu.size(); i++)
    for (int c = 0; c < 3; c++) {
      const int32_t *b = tu[i].b[c];
      if (b[6] < 0) continue;
      const int rows = box[3 * i + c] & 255, cols = box[3 * i + c] >> 8;
      for (int y = 0; y < rows; y++)
        std::memcpy(pool.data() + off + (size_t)y * b[2], coef.data() + b[6] + (size_t)y * cols, (size_t)cols * sizeof(int32_t));
      tus[i].b[c][6] = (int32_t)off;
      off += (size_t)b[2] * b[3];
    }
}

int PictureSyntax::cuAt(int ch, int x, int y) const {
  if (ch) { x <<= 1; y <<= 1; }
  if (x < 0 || y < 0 || x >= W || y >= H) return -1;
  return map[ch && !mapShared ? 1 : 0][(size_t)(y >> 2) * w4 + (x >> 2)];
}

void parse_slice_data(PictureSyntax &pic, const SliceCtx &sc, const uint8_t *rbsp, size_t n, const std::vector<uint32_t> &nal_epb) {
  Parser p(pic, pic, sc);
  p.run(rbsp, n, nal_epb, 0, (int)sc.sh->ctus.size(), 0);
}

namespace {

struct Segment { int slice, i0, i1, ss; };   // the slice's CTUs [i0, i1), starting substream ss

// The slice's CTUs split at tile starts, with the substream each piece starts (the counting of Parser::run)
void slice_segments(const PictureSyntax &pic, const SliceCtx &sc, int s, std::vector<Segment> &out) {
  const PPS &pps = *sc.pps;
  const SliceHeader &sh = *sc.sh;
  const int nCtu = (int)sh.ctus.size();
  int ss = 0;
  for (int i = 0; i < nCtu; i++) {
    const int ctu = sh.ctus[i], cx = ctu % pic.wCtu, cy = ctu / pic.wCtu;
    const int tc = pps.ctuToTileCol[cx], tr = pps.ctuToTileRow[cy];
    const int tx0 = pps.colBd[tc], ty0 = pps.rowBd[tr];
    if (i == 0 || (cx == tx0 && cy == ty0)) {
      if (i) out.back().i1 = i;
      out.push_back({s, i, nCtu, ss});
    }
    if (cx + 1 == pps.colBd[tc + 1] && (cy + 1 == pps.rowBd[tr + 1] || pps.entropySync)) ss++;
  }
}

// Appends a unit's rows to the picture's: CU / PU / TU indices and level offsets move by the rows before
// them, and so do the map entries of the unit's CTUs
void append_rows(PictureSyntax &pic, PictureSyntax &L, const std::vector<SliceData> &slices, const std::vector<Segment> &segs) {
  const int32_t cuOff = (int32_t)pic.cu.size(), puOff = (int32_t)pic.pu.size(), tuOff = (int32_t)pic.tu.size();
  const int32_t coefOff = (int32_t)pic.coef.size();
  VVCP_CHECK(pic.cu.size() + L.cu.size() > (size_t)INT32_MAX / 2 || pic.coef.size() + L.coef.size() > (size_t)INT32_MAX, "picture rows overflow");
  for (vvcr_cu &c : L.cu) {
    if (c.firstpu >= 0) c.firstpu += puOff;
    if (c.firsttu >= 0) c.firsttu += tuOff;
  }
  for (vvcr_pu &u : L.pu) u.cu += cuOff;
  for (vvcr_tu &t : L.tu) {
    t.cu += cuOff;
    for (int c = 0; c < 3; c++)
      if (t.b[c][6] >= 0) t.b[c][6] += coefOff;
  }
  pic.cu.insert(pic.cu.end(), L.cu.begin(), L.cu.end());
  pic.cux.insert(pic.cux.end(), L.cux.begin(), L.cux.end());
  pic.pu.insert(pic.pu.end(), L.pu.begin(), L.pu.end());
  pic.pux.insert(pic.pux.end(), L.pux.begin(), L.pux.end());
  pic.tu.insert(pic.tu.end(), L.tu.begin(), L.tu.end());
  pic.box.resize(3 * (size_t)tuOff, 0);
  L.box.resize(3 * L.tu.size(), 0);
  pic.box.insert(pic.box.end(), L.box.begin(), L.box.end());
  pic.coef.insert(pic.coef.end(), L.coef.begin(), L.coef.end());
  const int s4 = pic.ctuSize >> 2;
  for (const Segment &g : segs)
    for (int i = g.i0; i < g.i1; i++) {
      const int ctu = slices[g.slice].sc.sh->ctus[i];
      const int x0 = (ctu % pic.wCtu) * s4, y0 = (ctu / pic.wCtu) * s4;
      const int x1 = std::min(pic.w4, x0 + s4), y1 = std::min(pic.h4, y0 + s4);
      for (int ch = 0; ch < 2; ch++)
        for (int y = y0; y < y1; y++) {
          int32_t *m = pic.map[ch].data() + (size_t)y * pic.w4;
          for (int x = x0; x < x1; x++)
            if (m[x] >= 0) m[x] += cuOff;
        }
    }
}

}  // namespace

std::pair<int, int> parse_picture_data(PictureSyntax &pic, const std::vector<SliceData> &slices, int threads, int ry0, int ry1) {
  // units of work whose CTUs lie in tiles no other unit touches: each tile of a multi-tile slice (whole tiles,
  // no CABAC or availability dependence between them), or the slices inside one tile together
  struct Unit { std::vector<Segment> segs; int tile; bool whole; size_t ctus; };
  std::vector<Unit> units;
  std::vector<Segment> segs;
  const bool all = ry0 <= 0 && ry1 >= pic.hCtu;
  int r0 = pic.hCtu, r1 = 0;
  for (size_t s = 0; s < slices.size(); s++) {
    const SliceCtx &sc = slices[s].sc;
    if (sc.sh->ctus.empty()) continue;
    segs.clear();
    slice_segments(pic, sc, (int)s, segs);
    for (Segment g : segs) {
      const int ctu = sc.sh->ctus[g.i0];
      const int tile = sc.pps->tileIdx(ctu % pic.wCtu, ctu / pic.wCtu);
      if (!all) {
        // the tiles whose rows reach [ry0, ry1). With one tile column, only the part of a tile before CTU
        // row ry1 (its CTUs come in raster order): the parsed PUs are then a contiguous run of the
        // picture's decoding order (vvcp_dmvr_split); with several, whole tile rows.
        const int tr = sc.pps->ctuToTileRow[ctu / pic.wCtu];
        const int t0 = sc.pps->rowBd[tr], t1 = sc.pps->rowBd[tr + 1];
        if (t1 <= ry0 || t0 >= ry1) continue;
        if (sc.pps->numTileCols() == 1) {
          int e = g.i0;
          while (e < g.i1 && sc.sh->ctus[e] / pic.wCtu < ry1) e++;
          if (e == g.i0) continue;
          g.i1 = e;
          r1 = std::max(r1, std::min(t1, ry1));
        } else {
          r1 = std::max(r1, t1);
        }
        r0 = std::min(r0, t0);
      }
      const bool whole = segs.size() > 1;
      if (!whole && !units.empty() && !units.back().whole && units.back().tile == tile) units.back().segs.push_back(g);
      else units.push_back({{g}, tile, whole, 0});
      units.back().ctus += (size_t)(g.i1 - g.i0);
    }
  }
  auto parse_unit = [&](PictureSyntax &rows, const Unit &u) {
    for (const Segment &g : u.segs) {
      const SliceData &d = slices[g.slice];
      Parser p(rows, pic, d.sc);
      p.run(d.rbsp, d.n, *d.epb, g.i0, g.i1, (size_t)g.ss);
    }
  };
  const std::pair<int, int> covered = all ? std::make_pair(0, pic.hCtu) : std::make_pair(std::min(r0, r1), r1);
  const int nu = (int)units.size();
  if (threads <= 1 || nu <= 1) {
    for (const Unit &u : units) parse_unit(pic, u);
    return covered;
  }
  pic.unshareMap();   // the channels' maps are written by every unit: no unit may copy one while others fill it
  std::vector<std::unique_ptr<PictureSyntax>> loc(nu);
  const size_t ctuArea = (size_t)pic.ctuSize * pic.ctuSize;
  for (int u = 1; u < nu; u++) {
    loc[u].reset(new PictureSyntax());
    loc[u]->reset_rows(pic, units[u].ctus * ctuArea);
  }
  std::vector<std::exception_ptr> err(nu);
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int u; (u = next.fetch_add(1)) < nu;) {
      try {
        parse_unit(u ? *loc[u] : pic, units[u]);
      } catch (...) {
        err[u] = std::current_exception();
      }
    }
  };
  std::vector<std::thread> pool;
  const int nt = std::min(threads, nu);
  for (int t = 1; t < nt; t++) pool.emplace_back(work);
  work();
  for (std::thread &t : pool) t.join();
  for (int u = 0; u < nu; u++)
    if (err[u]) std::rethrow_exception(err[u]);
  for (int u = 1; u < nu; u++) {
    append_rows(pic, *loc[u], slices, units[u].segs);
    loc[u].reset();
  }
  return covered;
}

void finish_picture_syntax(PictureSyntax &pic, int bitDepth) {
  pic.unshareMap();
  pic.box.resize(3 * pic.tu.size(), 0);   // TUs after the last one with levels
  // PU::getFinalIntraMode (UnitTools.cpp:627) of intra PUs, 4:2:0: DM resolves to the co-located luma
  // mode (PU::getCoLocatedIntraLumaMode :642), MIP luma neighbours count as planar
  for (vvcr_pu &u : pic.pu) {
    const vvcr_cu &c = pic.cu[u.cu];
    if (c.predmode != MODE_INTRA) continue;
    if (c.yvalid) u.fidir_l = u.idir_l;
    if (c.cvalid) {
      int m = u.idir_c;
      if (m == DM) {
        const bool sep = c.treetype != TREE_D || !c.yvalid || c.chtype == 1;
        const int lc = sep ? pic.cuAt(0, (c.cx << 1) + c.cw, (c.cy << 1) + c.ch) : u.cu;
        VVCP_CHECK(lc < 0, "co-located luma CU missing");
        m = pic.cu[lc].mip ? PLANAR : pic.pu[pic.cu[lc].firstpu].idir_l;
      }
      u.fidir_c = m;
    }
  }
  const int shift = std::max(bitDepth - 10, 0);
  const int n = pic.wCtu * pic.hCtu;
  for (int ctu = 0; ctu < n; ctu++) {   // raster order: merge targets are already resolved
    const int cx = ctu % pic.wCtu, cy = ctu / pic.wCtu;
    for (int c = 0; c < 3; c++) {
      vvcr_sao &o = pic.sao[(size_t)ctu * 3 + c];
      if (o.mode == 1) {
        int tmp[32];
        std::memcpy(tmp, o.offset, sizeof(tmp));
        std::memset(o.offset, 0, sizeof(o.offset));
        if (o.type == 4) {
          for (int i = 0; i < 4; i++) o.offset[(o.band + i) % 32] = tmp[(o.band + i) % 32] * (1 << shift);
        } else {
          for (int i = 0; i < 5; i++) o.offset[i] = tmp[i] * (1 << shift);
        }
      } else if (o.mode == 2) {
        const int tgt = o.type == 0 ? (cx > 0 ? ctu - 1 : -1) : (cy > 0 ? ctu - pic.wCtu : -1);
        VVCP_CHECK(tgt < 0, "SAO merge target missing");
        o = pic.sao[(size_t)tgt * 3 + c];
      }
    }
  }
}

}  // namespace vvcp
