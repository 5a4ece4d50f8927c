// vvcp_core.h — host-side VVC (VTM-7.3 draft syntax) parser of libvvcr: the descriptor producer that
// feeds the GPU reconstruction path. Bitstream reading, the CABAC engine and
// the data structures shared by the parameter-set, slice-data and motion-derivation stages.
//
// The reference parses with HLSyntaxReader (DecoderLib/VLCReader.cpp), CABACReader / BinDecoder
// (CABACReader.cpp, BinDecoder.cpp) and derives motion in DecCu::xDeriveCUMV (DecCu.cpp:878) over
// CodingStructure objects. This parser keeps flat per-picture arrays instead (CU / TU records, per-4x4
// maps), emits the vvcr_cu / vvcr_pu / vvcr_tu rows of include/vvcr.h directly, and separates the
// CABAC pass of a picture (independent of other pictures) from its motion derivation (which needs the
// collocated picture's motion) so pictures can be parsed on several threads.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "vvcr.h"
#include "vvcp_ctx_tables.h"

namespace vvcp {

struct ParseError : std::runtime_error {
  explicit ParseError(const std::string &m) : std::runtime_error(m) {}
};
#define VVCP_CHECK(c, msg) do { if (c) throw ::vvcp::ParseError(msg); } while (0)

inline int floorLog2(uint32_t v) { return v ? 31 - __builtin_clz(v) : -1; }
inline int ceilLog2(uint32_t v) { return v <= 1 ? 0 : 32 - __builtin_clz(v - 1); }
template <typename T> inline T clip3(T lo, T hi, T v) { return v < lo ? lo : (v > hi ? hi : v); }

// ------------------------------------------------------------------------------------------------
// NAL units: Annex-B start codes, emulation prevention removed (NALread.cpp:59 convertPayloadToRBSP).
// epb = positions (in the original NAL bytes) of the removed 0x03 bytes, for entry-point offsets.
// ------------------------------------------------------------------------------------------------
struct Nal {
  int type = 0, tid = 0, layer = 0;
  std::vector<uint8_t> rbsp;        // payload after the 2-byte NAL header
  std::vector<uint32_t> epb;        // emulation-prevention byte positions, counted from the NAL start
};
std::vector<Nal> split_annexb(const uint8_t *data, size_t n);

// RBSP bit reader (u(n), ue(v), se(v)) over a byte range
struct Bits {
  const uint8_t *p = nullptr;
  size_t nbits = 0, pos = 0;
  Bits() = default;
  Bits(const uint8_t *d, size_t nbytes) : p(d), nbits(nbytes * 8), pos(0) {}
  uint32_t u(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) {
      VVCP_CHECK(pos >= nbits, "bitstream overrun");
      v = (v << 1) | ((p[pos >> 3] >> (7 - (pos & 7))) & 1);
      pos++;
    }
    return v;
  }
  bool flag() { return u(1) != 0; }
  uint32_t ue() {
    int lz = 0;
    while (!u(1)) { lz++; VVCP_CHECK(lz > 31, "bad exp-Golomb code"); }
    return lz ? ((1u << lz) - 1 + u(lz)) : 0;
  }
  int32_t se() {
    uint32_t k = ue();
    return (k & 1) ? (int32_t)((k + 1) >> 1) : -(int32_t)(k >> 1);
  }
  bool aligned() const { return (pos & 7) == 0; }
  void align() { pos = (pos + 7) & ~(size_t)7; }
  size_t left() const { return nbits - pos; }
  size_t byte_pos() const { return pos >> 3; }
  // HLSyntaxReader::xMoreRbspData (VLCReader.cpp:3760)
  bool more_rbsp_data() const {
    const size_t l = left();
    if (l > 8) return true;
    uint32_t last = 0;
    for (size_t i = 0; i < l; i++) last = (last << 1) | ((p[(pos + i) >> 3] >> (7 - ((pos + i) & 7))) & 1);
    int cnt = (int)l;
    while (cnt > 0 && (last & 1) == 0) { last >>= 1; cnt--; }
    cnt--;
    return cnt > 0;
  }
};

// ------------------------------------------------------------------------------------------------
// CABAC: dual-window probability models (Contexts.h BinProbModel_Std) and the arithmetic decoder
// (BinDecoder.cpp). One decoder per substream; contexts are copied for WPP / tile resets.
// ------------------------------------------------------------------------------------------------
struct CtxModel {
  uint16_t s0, s1;
  uint8_t rate;
  static constexpr int MASK0 = ~(~0u << 10) << 5, MASK1 = ~(~0u << 14) << 1;
  void init(int qp, int initId, int log2win) {
    const int slope = (initId >> 3) - 4, offset = ((initId & 7) * 18) + 1;
    int st = ((slope * (qp - 16)) >> 1) + offset;
    st = st < 1 ? 1 : (st > 127 ? 127 : st);
    const int p1 = st << 8;
    s0 = (uint16_t)(p1 & MASK0);
    s1 = (uint16_t)(p1 & MASK1);
    const int r0 = 2 + ((log2win >> 2) & 3), r1 = 3 + r0 + (log2win & 3);
    rate = (uint8_t)(16 * r0 + r1);
  }
  uint8_t state() const { return (uint8_t)((s0 + s1) >> 8); }
  void update(unsigned bin) {   // (no branch on the bin: it is unpredictable)
    const int r0 = rate >> 4, r1 = rate & 15;
    const unsigned m = 0u - bin;
    s0 = (uint16_t)(s0 - ((s0 >> r0) & MASK0) + (((0x7fffu >> r0) & MASK0) & m));
    s1 = (uint16_t)(s1 - ((s1 >> r1) & MASK1) + (((0x7fffu >> r1) & MASK1) & m));
  }
};

// The arithmetic decoder keeps VTM's state (range; value with the stream bits aligned as
// BinDecoderBase keeps them) in a 64-bit window: value64 = VTM's value << 32 plus the next stream bits,
// so a refill reads 4 bytes every 32 bits consumed instead of one byte every 8. The comparisons against
// range << 7 (here << 39) see the same bits: VTM's not-yet-read bits are zeros below its 7 guard bits.
// CabacEngine is the engine's registers; Cabac adds the context models. CabacLocal is a copy of the
// registers with a pointer to the models, for a hot loop (residual coding): as locals the registers stay in
// CPU registers across the loop's level stores, which the compiler must otherwise assume may alias them.
struct CabacEngine {
  const uint8_t *p = nullptr, *end = nullptr;
  uint32_t range = 510;
  uint64_t value = 0;
  int bitsNeeded = -32;   // the lowest valid bit of value is bit bitsNeeded + 32; refill when it passes 32
#ifdef VVCP_TRACE   // bin trace in the format of the reference's D_CABAC channel (BinDecoder.cpp:315)
  int traceCount = 0;
#endif
  uint32_t byte() { return p < end ? *p++ : 0; }
  uint64_t word32() {   // the next 4 stream bytes, big-endian (zeros past the end, as byte())
    if (end - p >= 4) {
      const uint32_t w = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
      p += 4;
      return w;
    }
    uint32_t w = 0;
    for (int k = 0; k < 4; k++) w = w << 8 | byte();
    return w;
  }
  void refill() {
    if (bitsNeeded >= 0) { value += word32() << bitsNeeded; bitsNeeded -= 32; }
  }
  void start(const uint8_t *b, const uint8_t *e) {   // BinDecoderBase::start
    p = b; end = e;
    range = 510;
    value = (uint64_t)byte() << 40;
    value += (uint64_t)byte() << 32;
    value += word32();
    bitsNeeded = -32;
  }
  unsigned decode(CtxModel &m, unsigned id) {   // TBinDecoder::decodeBin, with the LPS / MPS choice as masks
    (void)id;
    const unsigned st = m.state();
    const unsigned mps = st >> 7;
    const unsigned q = st ^ ((0u - mps) & 0xff);   // the LPS probability state
    const uint32_t lps = (((q >> 2) * (range >> 5)) >> 1) + 4;
#ifdef VVCP_TRACE
    fprintf(stderr, "%d %d %d  [%d:%d]  %2d(MPS=%d)    -  ", traceCount++, id, range, range - lps, lps, st, value < ((uint64_t)(range - lps) << 39));
#endif
    range -= lps;
    const uint64_t sr = (uint64_t)range << 39;
    const uint64_t lpsMask = 0 - (uint64_t)(value >= sr);   // all ones when the LPS was decoded
    value -= sr & lpsMask;
    range ^= (range ^ lps) & (uint32_t)lpsMask;
    const unsigned b = mps ^ (unsigned)(lpsMask & 1);
    const int n = __builtin_clz(range) - 23;   // renormalise to 9 bits (range in [256, 510])
    range <<= n;
    value <<= n;
    bitsNeeded += n;
    refill();
    m.update(b);
#ifdef VVCP_TRACE
    fprintf(stderr, "%d\n", b);
#endif
    return b;
  }
  unsigned ep() {   // decodeBinEP
    value += value;
    ++bitsNeeded;
    refill();
    const uint64_t sr = (uint64_t)range << 39;
    const uint64_t mask = 0 - (uint64_t)(value >= sr);
    value -= sr & mask;
#ifdef VVCP_TRACE
    fprintf(stderr, "%d  %d  EP=%d \n", traceCount++, range, (int)(mask & 1));
#endif
    return (unsigned)(mask & 1);
  }
  // decodeBinsEP: n bypass bins, the most significant first, in chunks of up to 8 (one shift and at most
  // one refill per chunk, then a compare-subtract per bin against range << 39..46)
#ifdef VVCP_TRACE
  unsigned eps(unsigned n) {
    unsigned v = 0;
    for (unsigned i = 0; i < n; i++) v = (v << 1) | ep();
    return v;
  }
#else
  unsigned eps(unsigned n) {
    unsigned v = 0;
    while (n) {
      const unsigned k = n < 8 ? n : 8;
      value <<= k;
      bitsNeeded += (int)k;
      refill();
      uint64_t sr = (uint64_t)range << (39 + k);
      for (unsigned i = 0; i < k; i++) {
        sr >>= 1;
        const uint64_t mask = 0 - (uint64_t)(value >= sr);
        value -= sr & mask;
        v = v + v + (unsigned)(mask & 1);
      }
      n -= k;
    }
    return v;
  }
#endif
  unsigned trm() {   // decodeBinTrm
    range -= 2;
    const uint64_t sr = (uint64_t)range << 39;
    if (value >= sr) return 1;
    if (range < 256) {
      range += range; value += value;
      ++bitsNeeded;
      refill();
    }
    return 0;
  }
  // BinDecoderBase::decodeRemAbsEP (BinDecoder.cpp:183)
  unsigned rem_abs(unsigned rice, unsigned cutoff, int maxLog2TrRange) {
    unsigned prefix = 0;
    const unsigned maxPrefix = 32 - maxLog2TrRange;
    unsigned cw;
    do { prefix++; cw = ep(); } while (cw && prefix < maxPrefix);
    prefix -= 1 - cw;
    unsigned length = rice, offset;
    if (prefix < cutoff) offset = prefix << rice;
    else {
      offset = (((1u << (prefix - cutoff)) + cutoff - 1) << rice);
      length += (prefix == 32 - (unsigned)maxLog2TrRange ? maxLog2TrRange - rice : prefix - cutoff);
    }
    return offset + eps(length);
  }
};
struct Cabac : CabacEngine {
  CtxModel ctx[vvcp_ctx::NUM_CTX];
  void init_contexts(int qp, int initType) {   // CtxStore::init (Contexts.cpp:939)
    const int cq = qp < 0 ? 0 : (qp > 63 ? 63 : qp);
    for (int k = 0; k < vvcp_ctx::NUM_CTX; k++) ctx[k].init(cq, vvcp_ctx::kInit[initType][k], vvcp_ctx::kInit[3][k]);
  }
  unsigned bin(unsigned id) { return decode(ctx[id], id); }
};
struct CabacLocal : CabacEngine {
  CtxModel *ctx;
  explicit CabacLocal(Cabac &c) : CabacEngine(c), ctx(c.ctx) {}
  void store(Cabac &c) const { static_cast<CabacEngine &>(c) = *this; }
  unsigned bin(unsigned id) { return decode(ctx[id], id); }
};

// ------------------------------------------------------------------------------------------------
// Parameter sets (SPS / PPS / APS / picture header / slice header), only the fields the VTM-7.3
// syntax needs for this decoder; see vvcp_ps.cpp for the parsing (VLCReader.cpp).
// ------------------------------------------------------------------------------------------------
struct RPL {
  int num = 0, numLT = 0;
  bool ltrpInSH = false;
  int ident[32] = {0};            // delta POC (short term) or poc_lsb_lt (long term)
  bool isLT[32] = {false};
  bool msbPresent[32] = {false};
  int msbCycle[32] = {0};
};

struct SPS {
  int id = -1;
  int chromaFormat = 1, bitDepth = 10, qpBdOffset = 12;
  int width = 0, height = 0, ctuSize = 128, ctuLog2 = 7;
  int log2MinCb = 2;
  int minQT[3] = {0, 0, 0}, maxBTD[3] = {0, 0, 0}, maxBT[3] = {0, 0, 0}, maxTT[3] = {0, 0, 0};   // [I luma, inter, I chroma]
  bool dualTree = false, splitConsOverride = false;
  int log2MaxTb = 6;
  bool jointCbCr = false;
  // chroma QP tables [table][qp + 64]
  bool sameCqpTable = true;
  int cqp[3][128];
  bool sao = false, alf = false, ccalf = false;
  bool transformSkip = false;
  int bdpcm = 0;
  bool wrapAround = false;
  bool tmvp = false, sbtmvp = false, amvr = false, bdof = false, bdofCtrl = false, smvd = false, dmvr = false, dmvrCtrl = false;
  bool mmvd = false, isp = false, mrl = false, mip = false, cclm = false;
  bool mts = false, intraMts = false, interMts = false, sbt = false;
  bool affine = false, affineType = false, affineAmvr = false, prof = false, profCtrl = false;
  bool bcw = false, ibc = false, ciip = false, fpelMmvd = false, geo = false, lmcs = false, lfnst = false;
  bool ladf = false, plt = false, act = false;
  int ladfNum = 0, ladfQpOffset[5] = {0, 0, 0, 0, 0}, ladfLowerBound[5] = {0, 0, 0, 0, 0};   // luma-adaptive deblocking
  int log2ParMrgLevel = 2;
  bool scalingList = false;
  bool vbDisabledPresent = false;   // sps_loop_filter_across_virtual_boundaries_disabled_present_flag
  int numVbVer = 0, numVbHor = 0, vbPosX[3] = {0, 0, 0}, vbPosY[3] = {0, 0, 0};   // luma samples
  int bitsForPoc = 8;
  bool longTermRefs = false, interLayer = false, idrRplPresent = false, rpl1CopyFrom0 = false;
  std::vector<RPL> rpl[2];
  bool useWP = false, useWPBi = false;
  int minQpTsMinus4 = 0;
  int maxTLayers = 1;
  bool subPicPresent = false;
  int numSubPics = 1;
  bool subPicIdPresent = false, subPicIdSignalling = false;
  int subPicIdLen = 0;
  bool horCollocatedChroma = false, verCollocatedChroma = false;
  int mappedChromaQp(int comp, int qp) const {   // comp: 1 Cb, 2 Cr, 3 joint
    return cqp[sameCqpTable ? 0 : comp - 1][qp + 64];
  }
};

struct PPS {
  int id = -1, spsId = -1;
  int width = 0, height = 0;
  int confLeft = 0, confRight = 0, confTop = 0, confBottom = 0;
  bool outputFlagPresent = false;
  bool noPicPartition = true;
  int log2Ctu = 7;
  std::vector<int> tileColW, tileRowH, colBd, rowBd;   // in CTUs; colBd/rowBd have numTiles+1 entries
  std::vector<int> ctuToTileCol, ctuToTileRow;
  bool rectSlice = true, singleSlicePerSubPic = false;
  int numSlicesInPic = 1;
  // explicit rectangular slice layout (PPS::m_rectSlices, VLCReader.cpp:510-575): per slice its first tile,
  // its size in tiles, and for slices inside one tile their count and height in CTUs
  bool tileIdxDeltaPresent = false;
  std::vector<int> rsTileIdx, rsWidthInTiles, rsHeightInTiles, rsNumSlicesInTile, rsHeightInCtu;
  std::vector<std::vector<int>> rectSliceCtus;   // CTU addresses of each rectangular slice
  bool lfAcrossTiles = true, lfAcrossSlices = false;   // PPS constructor defaults (no picture partition)
  bool entropySync = false, cabacInitPresent = false;
  int numRefDefault[2] = {1, 1};
  bool rpl1IdxPresent = false;
  int initQp = 26;
  int log2MaxTs = 2;
  bool useDQP = false;
  int cbQpOffset = 0, crQpOffset = 0, jcQpOffset = 0;
  bool jointCbCrQpOffsetPresent = false, sliceChromaQpFlag = false;
  bool cuChromaQpOffsetEnabled = false;
  int chromaQpOffsetListLen = 0;
  int cqpList[7][3] = {{0}};   // [idx 1..6][cb, cr, jc]
  bool useWP = false, wpBi = false;
  bool dbkCtrlPresent = false, dbkOverrideEnabled = false, dbkDisabled = false;
  int betaOffsetDiv2 = 0, tcOffsetDiv2 = 0;
  bool constantSH = false;
  int depQuantIdc = 0, rplSpsIdc[2] = {0, 0}, mvdL1ZeroIdc = 0, colFromL0Idc = 0, sixMinusMaxMrgPlus1 = 0, maxMrgMinusMaxGeoPlus1 = 0;
  bool phExtPresent = false, shExtPresent = false;
  int numSubPics = 1;
  bool subPicIdSignalling = false;
  int subPicIdLen = 0;
  // derived
  int widthInCtus = 0, heightInCtus = 0;
  int numTiles() const { return (int)(colBd.size() - 1) * (int)(rowBd.size() - 1); }
  int numTileCols() const { return (int)colBd.size() - 1; }
  int tileIdx(int ctuX, int ctuY) const { return ctuToTileRow[ctuY] * numTileCols() + ctuToTileCol[ctuX]; }
};

struct AlfApsParam {
  bool newLuma = false, newChroma = false, ccNew[2] = {false, false};
  bool nonLinear[2] = {false, false};
  int numLumaFilters = 1;
  int deltaIdx[25] = {0};
  int16_t lumaCoeff[25 * 13] = {0};
  int16_t lumaClip[25 * 13] = {0};
  int numAltChroma = 1;
  int16_t chromaCoeff[8][7] = {{0}};
  int16_t chromaClip[8][7] = {{0}};
  int ccCount[2] = {0, 0};
  int16_t ccCoeff[2][4][8] = {{{0}}};
};
struct LmcsApsParam {
  int minBin = 0, maxBin = 15, deltaCwBits = 1;
  int binDelta[16] = {0};
  int chrOffset = 0;
};
struct APS {
  int id = -1, type = -1, tid = 0;
  AlfApsParam alf;
  LmcsApsParam lmcs;
};

struct PicHeader {
  bool valid = false;
  bool nonRef = false, gdr = false, noOutputPrior = false;
  int ppsId = -1;
  bool subPicIdSignalling = false;   // ph_subpic_id_signalling_present_flag
  int subPicIdLen = 0;
  bool vbDisabled = false;          // the picture's virtual boundaries (the SPS's when it carries them)
  int numVbVer = 0, numVbHor = 0, vbPosX[3] = {0, 0, 0}, vbPosY[3] = {0, 0, 0};
  bool picOutput = true;
  bool rplPresent = false;
  int rplIdx[2] = {-1, -1};
  RPL rpl[2];                     // the list in use (copied from the SPS or parsed)
  bool splitOverride = false;
  int minQT[3], maxBTD[3], maxBT[3], maxTT[3];
  int cuQpDeltaSubdivIntra = 0, cuQpDeltaSubdivInter = 0, cuChromaQpOffsetSubdivIntra = 0, cuChromaQpOffsetSubdivInter = 0;
  bool tmvp = false, mvdL1Zero = false;
  int maxNumMergeCand = 6, maxNumAffineMergeCand = 5, maxNumGeoCand = 0, maxNumIbcMergeCand = 0;
  bool disFracMmvd = false, disBdof = false, disDmvr = false, disProf = false;
  bool jointCbCrSign = false;
  bool saoPresent = false, sao[2] = {false, false};
  bool alfPresent = false, alf[3] = {false, false, false};
  int numAlfAps = 0, alfApsLuma[8] = {0}, alfApsChroma = 0;
  bool ccAlf[2] = {false, false};
  int ccAlfApsId[2] = {-1, -1};
  bool depQuant = false, signHiding = false;
  bool dbkOverridePresent = false, dbkOverride = false, dbkDisable = false;
  int betaOffsetDiv2 = 0, tcOffsetDiv2 = 0;
  bool lmcs = false, lmcsChroma = false;
  int lmcsApsId = 0;
  bool scalingListPresent = false;
};

struct SliceHeader {
  int nalType = 0, tid = 0;
  int poc = 0;
  int sliceAddr = 0;
  std::vector<int> ctus;          // CTU raster addresses of the slice in decoding order
  int sliceType = 2;              // 0 B, 1 P, 2 I
  RPL rpl[2];
  int rplIdx[2] = {-1, -1};
  int numRef[2] = {0, 0};
  bool cabacInit = false;
  bool colFromL0 = true;
  int colRefIdx = 0;
  int wp[2][VVCR_MAX_REF][3][4];  // present, log2denom, weight, offset
  int qp = 26;
  int cbQpDelta = 0, crQpDelta = 0, jcQpDelta = 0;
  bool chromaQpAdj = false;
  bool sao[2] = {false, false};
  bool alf[3] = {false, false, false};
  int numAlfAps = 0, alfApsLuma[8] = {0}, alfApsChroma = 0;
  bool ccAlf[2] = {false, false};
  int ccAlfApsId[2] = {-1, -1};
  bool dbkOverride = false, dbkDisable = false;
  int betaOffsetDiv2 = 0, tcOffsetDiv2 = 0;
  std::vector<uint32_t> entryPoints;   // substream sizes in RBSP bytes
  size_t dataOffset = 0;               // RBSP byte position of slice_data
  int indepSliceIdx = 0;
  // reference structure (set by the decoder after RPL construction)
  int refPoc[2][VVCR_MAX_REF];
  bool refLT[2][VVCR_MAX_REF];
  bool checkLDC = false;
  bool biDirPred = false;
  int symRefIdx[2] = {-1, -1};
  bool isIntra() const { return sliceType == 2; }
  bool isInterB() const { return sliceType == 0; }
  bool isInterP() const { return sliceType == 1; }
  bool idr() const { return nalType == 7 || nalType == 8; }
};

}  // namespace vvcp
