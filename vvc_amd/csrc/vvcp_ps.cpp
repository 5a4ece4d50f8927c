// vvcp_ps.cpp — NAL unit splitting and high-level syntax of the host parser: SPS, PPS, APS (ALF,
// LMCS), picture header and slice header in VTM-7.3 draft syntax. Restated from the reference's
// HLSyntaxReader (DecoderLib/VLCReader.cpp; cited per function) — only what this decoder uses is kept,
// and syntax the reconstruction path does not support (palette, ACT, RPR, subpicture IDs in slice
// headers, scaling lists) is rejected with a ParseError instead of being silently misread.
#include "vvcp_ps.h"

#include <algorithm>

namespace vvcp {

// Annex-B byte stream -> NAL units (AnnexBread.cpp / NALread.cpp:59 convertPayloadToRBSP)
std::vector<Nal> split_annexb(const uint8_t *d, size_t n) {
  std::vector<Nal> out;
  size_t i = 0;
  auto is_start = [&](size_t k) { return k + 2 < n && d[k] == 0 && d[k + 1] == 0 && d[k + 2] == 1; };
  while (i < n && !is_start(i)) i++;
  while (i < n) {
    i += 3;
    size_t j = i;
    while (j < n && !is_start(j)) j++;
    size_t e = j;
    while (e > i && d[e - 1] == 0) e--;   // trailing zero bytes belong to the next start code
    if (e - i >= 2) {
      Nal nal;
      nal.layer = d[i] & 0x3f;
      nal.type = (d[i + 1] >> 3) & 0x1f;
      nal.tid = (d[i + 1] & 7) - 1;
      nal.rbsp.reserve(e - i);
      int zeros = 0;
      for (size_t k = i + 2; k < e; k++) {
        if (zeros == 2 && d[k] == 3) {
          nal.epb.push_back((uint32_t)(k - i));
          zeros = 0;
          continue;
        }
        zeros = d[k] == 0 ? zeros + 1 : 0;
        nal.rbsp.push_back(d[k]);
      }
      out.push_back(std::move(nal));
    }
    i = j;
  }
  return out;
}

// parseProfileTierLevel / parseConstraintInfo (VLCReader.cpp:3398-3499): skipped, only sizes matter
static void skip_ptl(Bits &b, int maxSubLayersMinus1) {
  b.u(7); b.u(1);
  // constraint info: 5 flags, u(4), u(2), 35 flags (JVET_Q0795 adds no_ccalf)
  b.u(5); b.u(4); b.u(2);
  for (int i = 0; i < 35; i++) b.u(1);
  b.u(8);
  const int nsub = (int)b.u(8);
  for (int i = 0; i < nsub; i++) b.u(32);
  std::vector<int> present(maxSubLayersMinus1 > 0 ? maxSubLayersMinus1 : 0);
  for (int i = 0; i < maxSubLayersMinus1; i++) present[i] = b.u(1);
  while (!b.aligned()) VVCP_CHECK(b.u(1) != 0, "ptl_alignment_zero_bit");
  for (int i = 0; i < maxSubLayersMinus1; i++)
    if (present[i]) b.u(8);
}

// HLSyntaxReader::parseRefPicList (VLCReader.cpp:318)
static void parse_rpl(Bits &b, const SPS &sps, RPL &r) {
  r = RPL();
  const int n = (int)b.ue();
  VVCP_CHECK(n > 32, "too many reference entries");
  if (sps.longTermRefs) r.ltrpInSH = b.flag();
  bool first = true;
  int prev = 0;
  VVCP_CHECK(sps.interLayer, "inter-layer references are not supported");
  for (int i = 0; i < n; i++) {
    bool lt = false;
    if (sps.longTermRefs) lt = !b.flag();
    if (!lt) {
      uint32_t code = b.ue();
      if (!sps.useWP && !sps.useWPBi) code++;
      int v = (int)code;
      uint32_t sign = 1;
      if (v > 0) sign = b.u(1);
      v = sign ? v : -v;
      int delta = first ? v : prev + v;
      first = false;
      prev = delta;
      r.ident[i] = delta;
      r.isLT[i] = false;
    } else {
      r.ident[i] = r.ltrpInSH ? 0 : (int)b.u(sps.bitsForPoc);
      r.isLT[i] = true;
      r.numLT++;
    }
  }
  r.num = n;
}

// SPS::derivedChromaQPMappingTables (Slice.cpp:1947)
static void derive_cqp(SPS &s, int numTables, const int start[3], const std::vector<int> dIn[3], const std::vector<int> dOut[3]) {
  const int off = s.qpBdOffset;
  for (int t = 0; t < numTables; t++) {
    const int np = (int)dIn[t].size();
    std::vector<int> in(np + 1), outv(np + 1);
    in[0] = start[t] + 26;
    outv[0] = in[0];
    for (int j = 0; j < np; j++) { in[j + 1] = in[j] + dIn[t][j] + 1; outv[j + 1] = outv[j] + dOut[t][j]; }
    int *m = s.cqp[t];
    auto at = [&](int q) -> int & { return m[q + 64]; };
    at(in[0]) = outv[0];
    for (int k = in[0] - 1; k >= -off; k--) at(k) = clip3(-off, 63, at(k + 1) - 1);
    for (int j = 0; j < np; j++) {
      const int sh = (dIn[t][j] + 1) >> 1;
      for (int k = in[j] + 1, mm = 1; k <= in[j + 1]; k++, mm++) at(k) = at(in[j]) + ((outv[j + 1] - outv[j]) * mm + sh) / (dIn[t][j] + 1);
    }
    for (int k = in[np] + 1; k <= 63; k++) at(k) = clip3(-off, 63, at(k - 1) + 1);
  }
}

// HLSyntaxReader::parseSPS (VLCReader.cpp:1129)
void parse_sps(Bits &b, SPS &s) {
  s = SPS();
  b.u(4); b.u(4);                                     // dps id, vps id
  s.maxTLayers = (int)b.u(3) + 1;
  VVCP_CHECK(b.u(5) != 0, "sps_reserved_zero_5bits");
  skip_ptl(b, s.maxTLayers - 1);
  b.u(1);   // gdr_enabled_flag: GDR pictures themselves are rejected at the picture header
  s.id = (int)b.u(4);
  s.chromaFormat = (int)b.u(2);
  VVCP_CHECK(s.chromaFormat != 1, "only 4:2:0 is supported");
  VVCP_CHECK(b.flag(), "reference picture resampling is not supported");
  s.width = (int)b.ue();
  s.height = (int)b.ue();
  const int l2 = (int)b.u(2);
  s.ctuLog2 = l2 + 5;
  s.ctuSize = 1 << s.ctuLog2;
  s.subPicPresent = b.flag();
  if (s.subPicPresent) {
    s.numSubPics = (int)b.u(8) + 1;
    const int wc = (s.width + s.ctuSize - 1) / s.ctuSize, hc = (s.height + s.ctuSize - 1) / s.ctuSize;
    for (int i = 0; i < s.numSubPics; i++) {
      if (s.width > s.ctuSize) b.u(ceilLog2(wc));
      if (s.height > s.ctuSize) b.u(ceilLog2(hc));
      if (s.width > s.ctuSize) b.u(ceilLog2(wc));
      if (s.height > s.ctuSize) b.u(ceilLog2(hc));
      b.u(1); b.u(1);   // subpic_treated_as_pic, loop_filter_across_subpic: not used by VTM 7.3
    }
  }
  s.subPicIdPresent = b.flag();
  if (s.subPicIdPresent) {
    s.subPicIdSignalling = b.flag();
    if (s.subPicIdSignalling) {
      s.subPicIdLen = (int)b.ue() + 1;
      for (int i = 0; i < s.numSubPics; i++) b.u(s.subPicIdLen);
    }
  }
  const int bdm8 = (int)b.ue();
  s.bitDepth = 8 + bdm8;
  s.qpBdOffset = 6 * bdm8;
  VVCP_CHECK(s.bitDepth > 10, "bit depths above 10 are not supported");
  s.minQpTsMinus4 = (int)b.ue();
  s.useWP = b.flag();
  s.useWPBi = b.flag();
  s.bitsForPoc = 4 + (int)b.u(4);
  int sublayerOrdering = s.maxTLayers > 1 ? b.u(1) : 0;
  for (int i = 0; i < s.maxTLayers; i++) {
    b.ue(); b.ue(); b.ue();
    if (!sublayerOrdering) break;
  }
  s.longTermRefs = b.flag();
  s.interLayer = b.flag();
  s.idrRplPresent = b.flag();
  s.rpl1CopyFrom0 = b.flag();
  int n = (int)b.ue();
  s.rpl[0].resize(n);
  for (int i = 0; i < n; i++) parse_rpl(b, s, s.rpl[0][i]);
  if (!s.rpl1CopyFrom0) {
    n = (int)b.ue();
    s.rpl[1].resize(n);
    for (int i = 0; i < n; i++) parse_rpl(b, s, s.rpl[1][i]);
  } else {
    s.rpl[1] = s.rpl[0];   // copyRefPicList (VLCReader.cpp:297): entries and counts
  }
  s.dualTree = b.flag();
  s.log2MinCb = (int)b.ue() + 2;
  s.splitConsOverride = b.flag();
  // JVET_Q0481 ordering: intra luma, inter, intra chroma
  int v = (int)b.ue();
  const int minQtIntraLog2 = v + s.log2MinCb;
  s.minQT[0] = 1 << minQtIntraLog2;
  s.maxBTD[0] = (int)b.ue();
  s.maxBT[0] = s.maxTT[0] = s.minQT[0];
  if (s.maxBTD[0]) { s.maxBT[0] <<= b.ue(); s.maxTT[0] <<= b.ue(); }
  v = (int)b.ue();
  s.minQT[1] = 1 << (v + s.log2MinCb);
  s.maxBTD[1] = (int)b.ue();
  s.maxBT[1] = s.maxTT[1] = s.minQT[1];
  if (s.maxBTD[1]) { s.maxBT[1] <<= b.ue(); s.maxTT[1] <<= b.ue(); }
  if (s.dualTree) {
    s.minQT[2] = 1 << ((int)b.ue() + s.log2MinCb);
    s.maxBTD[2] = (int)b.ue();
    s.maxBT[2] = s.maxTT[2] = s.minQT[2];
    if (s.maxBTD[2]) { s.maxBT[2] <<= b.ue(); s.maxTT[2] <<= b.ue(); }
  }
  s.log2MaxTb = b.flag() ? 6 : 5;
  s.jointCbCr = b.flag();
  {
    s.sameCqpTable = b.flag();
    const int numTables = s.sameCqpTable ? 1 : (s.jointCbCr ? 3 : 2);
    int start[3] = {0, 0, 0};
    std::vector<int> dIn[3], dOut[3];
    for (int t = 0; t < numTables; t++) {
      start[t] = b.se();
      const int np = (int)b.ue() + 1;
      for (int j = 0; j < np; j++) {
        const int in = (int)b.ue();
        const int diff = (int)b.ue();
        dIn[t].push_back(in);
        dOut[t].push_back(diff ^ in);
      }
    }
    for (int t = 0; t < 3; t++)
      for (int q = 0; q < 128; q++) s.cqp[t][q] = 0;
    derive_cqp(s, numTables, start, dIn, dOut);
  }
  s.sao = b.flag();
  s.alf = b.flag();
  if (s.alf) s.ccalf = b.flag();
  s.transformSkip = b.flag();
  if (s.transformSkip) s.bdpcm = b.u(1);
  s.wrapAround = b.flag();
  VVCP_CHECK(s.wrapAround, "wrap-around motion compensation is not supported");
  s.tmvp = b.flag();
  if (s.tmvp) s.sbtmvp = b.flag();
  s.amvr = b.flag();
  s.bdof = b.flag();
  if (s.bdof) s.bdofCtrl = b.flag();
  s.smvd = b.flag();
  s.dmvr = b.flag();
  if (s.dmvr) s.dmvrCtrl = b.flag();
  s.mmvd = b.flag();
  s.isp = b.flag();
  s.mrl = b.flag();
  s.mip = b.flag();
  s.cclm = b.flag();
  s.horCollocatedChroma = b.flag();
  s.verCollocatedChroma = b.flag();
  s.mts = b.flag();
  if (s.mts) { s.intraMts = b.flag(); s.interMts = b.flag(); }
  s.sbt = b.flag();
  s.affine = b.flag();
  if (s.affine) {
    s.affineType = b.flag();
    s.affineAmvr = b.flag();
    s.prof = b.flag();
    if (s.prof) s.profCtrl = b.flag();
  }
  s.bcw = b.flag();
  s.ibc = b.flag();
  VVCP_CHECK(s.ibc, "intra block copy is not supported");
  s.ciip = b.flag();
  if (s.mmvd) s.fpelMmvd = b.flag();
  s.geo = b.flag();
  s.lmcs = b.flag();
  s.lfnst = b.flag();
  s.ladf = b.flag();
  if (s.ladf) {   // VLCReader.cpp:1609-1621: intervals, the lowest one's QP offset, then offset and bound per interval
    s.ladfNum = (int)b.u(2) + 2;
    s.ladfQpOffset[0] = b.se();
    for (int k = 1; k < s.ladfNum; k++) {
      s.ladfQpOffset[k] = b.se();
      const int64_t d = (int64_t)b.ue() + 1;
      VVCP_CHECK(d > (1 << 16), "LADF interval threshold out of range");
      s.ladfLowerBound[k] = s.ladfLowerBound[k - 1] + (int)d;
    }
  }
  s.log2ParMrgLevel = (int)b.ue() + 2;
  s.scalingList = b.flag();
  VVCP_CHECK(s.scalingList, "scaling lists are not supported");
  s.vbDisabledPresent = b.flag();
  if (s.vbDisabledPresent) {   // VLCReader.cpp:1636-1654
    s.numVbVer = (int)b.u(2);
    VVCP_CHECK(s.numVbVer > 3, "too many virtual boundaries");
    for (int i = 0; i < s.numVbVer; i++) s.vbPosX[i] = (int)b.u(13) << 3;
    s.numVbHor = (int)b.u(2);
    VVCP_CHECK(s.numVbHor > 3, "too many virtual boundaries");
    for (int i = 0; i < s.numVbHor; i++) s.vbPosY[i] = (int)b.u(13) << 3;
  }
  // general_hrd_parameters / VUI / extensions follow; nothing after them affects decoding here
}

// PPS::initTiles (Slice.cpp:2164) and the CTU -> tile maps
static void init_tiles(PPS &p) {
  p.colBd.assign(1, 0);
  p.rowBd.assign(1, 0);
  std::vector<int> cw = p.tileColW, rh = p.tileRowH;
  int rem = p.widthInCtus;
  for (int w : cw) { VVCP_CHECK(w <= 0, "tile column width"); rem -= w; }
  VVCP_CHECK(rem < 0, "tile columns wider than the picture");
  int uni = cw.back();
  while (rem > 0) { uni = std::min(rem, uni); cw.push_back(uni); rem -= uni; }
  rem = p.heightInCtus;
  for (int h : rh) { VVCP_CHECK(h <= 0, "tile row height"); rem -= h; }
  VVCP_CHECK(rem < 0, "tile rows taller than the picture");
  uni = rh.back();
  while (rem > 0) { uni = std::min(rem, uni); rh.push_back(uni); rem -= uni; }
  for (int w : cw) p.colBd.push_back(p.colBd.back() + w);
  for (int h : rh) p.rowBd.push_back(p.rowBd.back() + h);
  p.ctuToTileCol.assign(p.widthInCtus, 0);
  p.ctuToTileRow.assign(p.heightInCtus, 0);
  for (int t = 0; t < (int)cw.size(); t++)
    for (int x = p.colBd[t]; x < p.colBd[t + 1]; x++) p.ctuToTileCol[x] = t;
  for (int t = 0; t < (int)rh.size(); t++)
    for (int y = p.rowBd[t]; y < p.rowBd[t + 1]; y++) p.ctuToTileRow[y] = t;
}

static void add_tile_ctus(const PPS &p, std::vector<int> &ctus, int tx, int ty) {
  for (int y = p.rowBd[ty]; y < p.rowBd[ty + 1]; y++)
    for (int x = p.colBd[tx]; x < p.colBd[tx + 1]; x++) ctus.push_back(y * p.widthInCtus + x);
}

// HLSyntaxReader::parsePPS (VLCReader.cpp:408); tile geometry is completed by finalize_pps once the
// SPS (CTU size) is known
void parse_pps(Bits &b, PPS &p) {
  p = PPS();
  p.id = (int)b.ue();
  p.spsId = (int)b.u(4);
  p.width = (int)b.ue();
  p.height = (int)b.ue();
  if (b.flag()) { p.confLeft = b.ue(); p.confRight = b.ue(); p.confTop = b.ue(); p.confBottom = b.ue(); }
  if (b.flag()) { b.ue(); b.ue(); b.ue(); b.ue(); }   // scaling window: RPR only
  p.outputFlagPresent = b.flag();
  p.subPicIdSignalling = b.flag();
  if (p.subPicIdSignalling) {
    p.numSubPics = (int)b.ue() + 1;
    p.subPicIdLen = (int)b.ue() + 1;
    for (int i = 0; i < p.numSubPics; i++) b.u(p.subPicIdLen);
  }
  p.noPicPartition = b.flag();
  if (!p.noPicPartition) {
    p.log2Ctu = (int)b.u(2) + 5;
    const int nc = (int)b.ue() + 1, nr = (int)b.ue() + 1;
    for (int i = 0; i < nc; i++) p.tileColW.push_back((int)b.ue() + 1);
    for (int i = 0; i < nr; i++) p.tileRowH.push_back((int)b.ue() + 1);
    p.rectSlice = b.flag();
    if (p.rectSlice) p.singleSlicePerSubPic = b.flag();
    if (p.rectSlice && !p.singleSlicePerSubPic) {
      // explicit rectangular slices (VLCReader.cpp:510-575); the tile grid is known from the PPS alone
      VVCP_CHECK(p.width <= 0 || p.height <= 0, "PPS picture size");
      p.widthInCtus = (p.width + (1 << p.log2Ctu) - 1) >> p.log2Ctu;
      p.heightInCtus = (p.height + (1 << p.log2Ctu) - 1) >> p.log2Ctu;
      init_tiles(p);
      const int ntc = p.numTileCols(), nt = p.numTiles();
      p.numSlicesInPic = (int)b.ue() + 1;
      VVCP_CHECK(p.numSlicesInPic > 600, "too many slices");   // MAX_SLICES
      p.tileIdxDeltaPresent = b.flag();
      const int n = p.numSlicesInPic;
      p.rsTileIdx.assign(n, 0); p.rsWidthInTiles.assign(n, 1); p.rsHeightInTiles.assign(n, 1);
      p.rsNumSlicesInTile.assign(n, 1); p.rsHeightInCtu.assign(n, 0);
      int tileIdx = 0;
      for (int i = 0; i < n - 1; i++) {
        p.rsTileIdx[i] = tileIdx;
        p.rsWidthInTiles[i] = (int)b.ue() + 1;
        // JVET_Q0480: the height is inferred from the previous slice inside a row of tiles
        if (p.tileIdxDeltaPresent || tileIdx % ntc == 0) p.rsHeightInTiles[i] = (int)b.ue() + 1;
        else p.rsHeightInTiles[i] = i > 0 ? p.rsHeightInTiles[i - 1] : 1;
        if (p.rsWidthInTiles[i] == 1 && p.rsHeightInTiles[i] == 1) {   // slices inside one tile
          const int nst = (int)b.ue() + 1;
          p.rsNumSlicesInTile[i] = nst;
          for (int j = 0; j < nst - 1; j++) {
            p.rsHeightInCtu[i] = (int)b.ue() + 1;
            i++;
            VVCP_CHECK(i >= n, "slices in a tile exceed the picture's slices");
            p.rsWidthInTiles[i] = 1; p.rsHeightInTiles[i] = 1;
            p.rsNumSlicesInTile[i] = nst;
            p.rsTileIdx[i] = tileIdx;
          }
        }
        if (i < n - 1) {
          if (p.tileIdxDeltaPresent) {
            tileIdx += b.se();
            VVCP_CHECK(tileIdx < 0 || tileIdx >= nt, "invalid tile_idx_delta");
          } else {
            tileIdx += p.rsWidthInTiles[i];
            if (tileIdx % ntc == 0) tileIdx += (p.rsHeightInTiles[i] - 1) * ntc;
          }
        }
      }
      VVCP_CHECK(tileIdx >= nt, "rectangular slice outside the tile grid");
      p.rsTileIdx[n - 1] = tileIdx;
    }
    p.lfAcrossTiles = b.flag();
    p.lfAcrossSlices = b.flag();
  }
  p.entropySync = b.flag();
  p.cabacInitPresent = b.flag();
  p.numRefDefault[0] = (int)b.ue() + 1;
  p.numRefDefault[1] = (int)b.ue() + 1;
  p.rpl1IdxPresent = b.flag();
  p.initQp = 26 + b.se();
  p.log2MaxTs = (int)b.ue() + 2;
  p.useDQP = b.flag();
  p.cbQpOffset = b.se();
  p.crQpOffset = b.se();
  p.jointCbCrQpOffsetPresent = b.flag();
  p.jcQpOffset = p.jointCbCrQpOffsetPresent ? b.se() : 0;
  p.sliceChromaQpFlag = b.flag();
  p.cuChromaQpOffsetEnabled = b.flag();
  if (p.cuChromaQpOffsetEnabled) {
    p.chromaQpOffsetListLen = (int)b.ue() + 1;
    VVCP_CHECK(p.chromaQpOffsetListLen > 6, "chroma QP offset list too long");
    for (int i = 1; i <= p.chromaQpOffsetListLen; i++) {
      p.cqpList[i][0] = b.se();
      p.cqpList[i][1] = b.se();
      p.cqpList[i][2] = p.jointCbCrQpOffsetPresent ? b.se() : 0;
    }
  }
  p.useWP = b.flag();
  p.wpBi = b.flag();
  p.dbkCtrlPresent = b.flag();
  if (p.dbkCtrlPresent) {
    p.dbkOverrideEnabled = b.flag();
    p.dbkDisabled = b.flag();
    if (!p.dbkDisabled) { p.betaOffsetDiv2 = b.se(); p.tcOffsetDiv2 = b.se(); }
  }
  p.constantSH = b.flag();
  if (p.constantSH) {
    p.depQuantIdc = (int)b.u(2);
    p.rplSpsIdc[0] = (int)b.u(2);
    p.rplSpsIdc[1] = (int)b.u(2);
    p.mvdL1ZeroIdc = (int)b.u(2);
    p.colFromL0Idc = (int)b.u(2);
    p.sixMinusMaxMrgPlus1 = (int)b.ue();
    p.maxMrgMinusMaxGeoPlus1 = (int)b.ue();
  }
  p.phExtPresent = b.flag();
  p.shExtPresent = b.flag();
  // pps_extension (range extension: cross-component prediction, SAO offset scale) is not used by VTM CTC
}

void finalize_pps(PPS &p, const SPS &s) {
  const int ctu = s.ctuSize;
  p.widthInCtus = (p.width + ctu - 1) / ctu;
  p.heightInCtus = (p.height + ctu - 1) / ctu;
  if (p.noPicPartition) {   // parsePictureHeader (VLCReader.cpp:1917-1936)
    p.tileColW.assign(1, p.widthInCtus);
    p.tileRowH.assign(1, p.heightInCtus);
    p.rectSlice = true;
    p.numSlicesInPic = 1;
  } else {
    VVCP_CHECK(p.log2Ctu != s.ctuLog2, "PPS CTU size does not match the SPS");
  }
  init_tiles(p);
  p.rectSliceCtus.clear();
  if (p.rectSlice && !p.singleSlicePerSubPic && !p.noPicPartition) {
    // PPS::initRectSliceMap (Slice.cpp:2258-2335): the tiles of each slice in raster order, or the CTU
    // rows of the slices inside one tile
    const int ntc = p.numTileCols(), ntr = (int)p.rowBd.size() - 1, n = p.numSlicesInPic;
    p.rectSliceCtus.assign(n, {});
    for (int i = 0; i < n; i++) {
      const int tx = p.rsTileIdx[i] % ntc, ty = p.rsTileIdx[i] / ntc;
      VVCP_CHECK(ty >= ntr, "rectangular slice outside the tile grid");
      if (i == n - 1) { p.rsWidthInTiles[i] = ntc - tx; p.rsHeightInTiles[i] = ntr - ty; p.rsNumSlicesInTile[i] = 1; }
      if (p.rsWidthInTiles[i] > 1 || p.rsHeightInTiles[i] > 1) {
        VVCP_CHECK(tx + p.rsWidthInTiles[i] > ntc || ty + p.rsHeightInTiles[i] > ntr, "rectangular slice outside the tile grid");
        for (int j = 0; j < p.rsHeightInTiles[i]; j++)
          for (int k = 0; k < p.rsWidthInTiles[i]; k++) add_tile_ctus(p, p.rectSliceCtus[i], tx + k, ty + j);
      } else {
        int cy = p.rowBd[ty];
        const int nst = p.rsNumSlicesInTile[i];
        for (int j = 0; j < nst - 1; j++) {
          VVCP_CHECK(p.rsHeightInCtu[i] <= 0 || cy + p.rsHeightInCtu[i] >= p.rowBd[ty + 1], "invalid rectangular slice height");
          for (int y = cy; y < cy + p.rsHeightInCtu[i]; y++)
            for (int x = p.colBd[tx]; x < p.colBd[tx + 1]; x++) p.rectSliceCtus[i].push_back(y * p.widthInCtus + x);
          cy += p.rsHeightInCtu[i];
          i++;
        }
        VVCP_CHECK(cy >= p.rowBd[ty + 1], "invalid rectangular slice signalling");
        for (int y = cy; y < p.rowBd[ty + 1]; y++)
          for (int x = p.colBd[tx]; x < p.colBd[tx + 1]; x++) p.rectSliceCtus[i].push_back(y * p.widthInCtus + x);
      }
    }
    // every CTU in exactly one slice (PPS::checkSliceMap)
    std::vector<uint8_t> seen((size_t)p.widthInCtus * p.heightInCtus, 0);
    for (const auto &c : p.rectSliceCtus)
      for (int a : c) { VVCP_CHECK(seen[a], "a CTU in two rectangular slices"); seen[a] = 1; }
    for (uint8_t v : seen) VVCP_CHECK(!v, "a CTU in no rectangular slice");
  } else if (p.rectSlice) {   // one rectangular slice holding every tile (initRectSliceMap, Slice.cpp:2283)
    VVCP_CHECK(p.singleSlicePerSubPic && s.numSubPics > 1, "one slice per subpicture with several subpictures is not supported");
    std::vector<int> c;
    for (int ty = 0; ty + 1 < (int)p.rowBd.size(); ty++)
      for (int tx = 0; tx + 1 < (int)p.colBd.size(); tx++) add_tile_ctus(p, c, tx, ty);
    p.rectSliceCtus.push_back(c);
  }
}

// HLSyntaxReader::alfGolombDecode / alfFilter (VLCReader.cpp:3789-3872)
static int alf_golomb(Bits &b, int k) {
  int nlb = -1;
  uint32_t bit = 0;
  for (; !bit; nlb++) bit = b.u(1);
  int sym = ((1 << nlb) - 1) << k;
  if (nlb + k > 0) sym += (int)b.u(nlb + k);
  if (sym && b.u(1)) sym = -sym;
  return sym;
}
static void alf_filter(Bits &b, AlfApsParam &a, bool chroma, int alt) {
  const int numCoeff = chroma ? 7 : 13, nf = chroma ? 1 : a.numLumaFilters;
  int16_t *coeff = chroma ? a.chromaCoeff[alt] : a.lumaCoeff;
  int16_t *clip = chroma ? a.chromaClip[alt] : a.lumaClip;
  const int stride = chroma ? 7 : 13;
  for (int f = 0; f < nf; f++)
    for (int i = 0; i < numCoeff - 1; i++) coeff[f * stride + i] = (int16_t)alf_golomb(b, 3);
  if (a.nonLinear[chroma ? 1 : 0]) {
    for (int f = 0; f < nf; f++)
      for (int i = 0; i < numCoeff - 1; i++) clip[f * stride + i] = (int16_t)b.u(2);
  } else {
    for (int f = 0; f < nf; f++)
      for (int i = 0; i < numCoeff; i++) clip[f * stride + i] = 0;
  }
}

// HLSyntaxReader::parseAPS / parseAlfAps / parseLmcsAps (VLCReader.cpp:788-986)
void parse_aps(Bits &b, APS &a) {
  a.id = (int)b.u(5);
  a.type = (int)b.u(3);
  if (a.type == 0) {   // ALF
    AlfApsParam &p = a.alf;
    p = AlfApsParam();
    p.newLuma = b.flag();
    p.newChroma = b.flag();
    p.ccNew[0] = b.flag();
    p.ccNew[1] = b.flag();
    if (p.newLuma) {
      p.nonLinear[0] = b.flag();
      p.numLumaFilters = (int)b.ue() + 1;
      if (p.numLumaFilters > 1) {
        const int len = ceilLog2(p.numLumaFilters);
        for (int i = 0; i < 25; i++) p.deltaIdx[i] = (int)b.u(len);
      }
      alf_filter(b, p, false, 0);
    }
    if (p.newChroma) {
      p.nonLinear[1] = b.flag();
      p.numAltChroma = (int)b.ue() + 1;
      for (int alt = 0; alt < p.numAltChroma; alt++) alf_filter(b, p, true, alt);
    }
    for (int c = 0; c < 2; c++) {
      if (!p.ccNew[c]) continue;
      p.ccCount[c] = (int)b.ue() + 1;
      for (int f = 0; f < p.ccCount[c]; f++)
        for (int i = 0; i < 7; i++) {
          const int code = (int)b.u(3);
          int16_t v = 0;
          if (code) {
            v = (int16_t)(1 << (code - 1));
            if (b.u(1)) v = (int16_t)-v;
          }
          p.ccCoeff[c][f][i] = v;
        }
    }
  } else if (a.type == 1) {   // LMCS
    LmcsApsParam &l = a.lmcs;
    l = LmcsApsParam();
    l.minBin = (int)b.ue();
    l.maxBin = 15 - (int)b.ue();
    l.deltaCwBits = (int)b.ue() + 1;
    for (int i = l.minBin; i <= l.maxBin; i++) {
      const int abs = (int)b.u(l.deltaCwBits);
      const int sign = abs > 0 ? (int)b.u(1) : 0;
      l.binDelta[i] = (1 - 2 * sign) * abs;
    }
    const int abs = (int)b.u(3);
    const int sign = abs > 0 ? (int)b.u(1) : 0;
    l.chrOffset = (1 - 2 * sign) * abs;
  } else {
    VVCP_CHECK(true, "scaling-list APS is not supported");
  }
}

// HLSyntaxReader::parsePictureHeader (VLCReader.cpp:1881); psets gives the SPS/PPS by id
void parse_ph(Bits &b, PicHeader &h, const ParamSets &ps) {
  h = PicHeader();
  h.nonRef = b.flag();
  h.gdr = b.flag();
  h.noOutputPrior = b.flag();
  VVCP_CHECK(h.gdr, "GDR pictures are not supported");
  if (h.gdr) b.ue();   // recovery_poc_cnt
  h.ppsId = (int)b.ue();
  const PPS *pps = ps.pps(h.ppsId);
  VVCP_CHECK(!pps, "picture header references a missing PPS");
  const SPS *sps = ps.sps(pps->spsId);
  VVCP_CHECK(!sps, "PPS references a missing SPS");
  if (sps->subPicIdPresent && !sps->subPicIdSignalling) {
    h.subPicIdSignalling = b.flag();   // ph_subpic_id_signalling_present_flag
    if (h.subPicIdSignalling) {
      h.subPicIdLen = (int)b.ue() + 1;
      for (int i = 0; i < sps->numSubPics; i++) b.u(h.subPicIdLen);
    }
  }
  if (!sps->vbDisabledPresent) {   // VLCReader.cpp:1982-2013
    h.vbDisabled = b.flag();
    if (h.vbDisabled) {
      h.numVbVer = (int)b.u(2);
      VVCP_CHECK(h.numVbVer > 3, "too many virtual boundaries");
      for (int i = 0; i < h.numVbVer; i++) h.vbPosX[i] = (int)b.u(13) << 3;
      h.numVbHor = (int)b.u(2);
      VVCP_CHECK(h.numVbHor > 3, "too many virtual boundaries");
      for (int i = 0; i < h.numVbHor; i++) h.vbPosY[i] = (int)b.u(13) << 3;
    }
  } else {
    h.vbDisabled = true;
    h.numVbVer = sps->numVbVer; h.numVbHor = sps->numVbHor;
    for (int i = 0; i < 3; i++) { h.vbPosX[i] = sps->vbPosX[i]; h.vbPosY[i] = sps->vbPosY[i]; }
  }
  h.picOutput = pps->outputFlagPresent ? b.flag() : true;
  h.rplPresent = b.flag();
  if (h.rplPresent) {
    for (int l = 0; l < 2; l++) {
      uint32_t spsFlag;
      if (l == 1 && !pps->rpl1IdxPresent) {
        h.rplIdx[1] = h.rplIdx[0];
        spsFlag = h.rplIdx[0] != -1;
      } else if (sps->rpl[l].empty()) spsFlag = 0;
      else if (!pps->rplSpsIdc[l]) spsFlag = b.u(1);
      else spsFlag = pps->rplSpsIdc[l] - 1;
      if (!spsFlag) {
        parse_rpl(b, *sps, h.rpl[l]);
        h.rplIdx[l] = -1;
      } else {
        if (l == 1 && !pps->rpl1IdxPresent) {
        } else if (sps->rpl[l].size() > 1) h.rplIdx[l] = (int)b.u(ceilLog2((uint32_t)sps->rpl[l].size()));
        else h.rplIdx[l] = 0;
        // u(ceilLog2(n)) reaches past n - 1 when n is not a power of two; list 1 may inherit list 0's index
        VVCP_CHECK(h.rplIdx[l] < 0 || h.rplIdx[l] >= (int)sps->rpl[l].size(), "picture header: reference picture list index out of range");
        h.rpl[l] = sps->rpl[l][h.rplIdx[l]];
      }
      if (h.rpl[l].numLT) {
        for (int i = 0; i < h.rpl[l].num; i++) {
          if (!h.rpl[l].isLT[i]) continue;
          if (h.rpl[l].ltrpInSH) h.rpl[l].ident[i] = (int)b.u(sps->bitsForPoc);
          h.rpl[l].msbPresent[i] = b.flag();
          if (h.rpl[l].msbPresent[i]) h.rpl[l].msbCycle[i] = (int)b.ue();
        }
      }
    }
  }
  for (int k = 0; k < 3; k++) { h.minQT[k] = sps->minQT[k]; h.maxBTD[k] = sps->maxBTD[k]; h.maxBT[k] = sps->maxBT[k]; h.maxTT[k] = sps->maxTT[k]; }
  if (sps->splitConsOverride) {
    h.splitOverride = b.flag();
    if (h.splitOverride) {
      h.minQT[0] = 1 << ((int)b.ue() + sps->log2MinCb);
      h.maxBTD[0] = (int)b.ue();
      h.maxBT[0] = h.maxTT[0] = h.minQT[0];
      if (h.maxBTD[0]) { h.maxBT[0] <<= b.ue(); h.maxTT[0] <<= b.ue(); }
      h.minQT[1] = 1 << ((int)b.ue() + sps->log2MinCb);
      h.maxBTD[1] = (int)b.ue();
      h.maxBT[1] = h.maxTT[1] = h.minQT[1];
      if (h.maxBTD[1]) { h.maxBT[1] <<= b.ue(); h.maxTT[1] <<= b.ue(); }
      if (sps->dualTree) {
        h.minQT[2] = 1 << ((int)b.ue() + sps->log2MinCb);
        h.maxBTD[2] = (int)b.ue();
        h.maxBT[2] = h.maxTT[2] = h.minQT[2];
        if (h.maxBTD[2]) { h.maxBT[2] <<= b.ue(); h.maxTT[2] <<= b.ue(); }
      }
    }
  }
  if (pps->useDQP) { h.cuQpDeltaSubdivIntra = (int)b.ue(); h.cuQpDeltaSubdivInter = (int)b.ue(); }
  if (pps->cuChromaQpOffsetEnabled) { h.cuChromaQpOffsetSubdivIntra = (int)b.ue(); h.cuChromaQpOffsetSubdivInter = (int)b.ue(); }
  h.tmvp = sps->tmvp ? b.flag() : false;
  h.mvdL1Zero = !pps->mvdL1ZeroIdc ? b.flag() : (pps->mvdL1ZeroIdc - 1) != 0;
  {
    const int v = !pps->sixMinusMaxMrgPlus1 ? (int)b.ue() : pps->sixMinusMaxMrgPlus1 - 1;
    h.maxNumMergeCand = 6 - v;
  }
  if (sps->affine) h.maxNumAffineMergeCand = 5 - (int)b.ue();
  else h.maxNumAffineMergeCand = (sps->sbtmvp && h.tmvp) ? 1 : 0;
  h.disFracMmvd = sps->fpelMmvd ? b.flag() : false;
  h.disBdof = sps->bdofCtrl ? b.flag() : false;
  h.disDmvr = sps->dmvrCtrl ? b.flag() : false;
  h.disProf = sps->profCtrl ? b.flag() : false;
  if (sps->geo && h.maxNumMergeCand >= 2) {
    const int v = !pps->maxMrgMinusMaxGeoPlus1 ? (int)b.ue() : pps->maxMrgMinusMaxGeoPlus1 - 1;
    h.maxNumGeoCand = h.maxNumMergeCand - v;
  }
  h.jointCbCrSign = sps->jointCbCr ? b.flag() : false;
  if (sps->sao) {
    h.saoPresent = b.flag();
    if (h.saoPresent) { h.sao[0] = b.flag(); h.sao[1] = b.flag(); }
    else { h.sao[0] = true; h.sao[1] = true; }
  }
  if (sps->alf) {
    h.alfPresent = b.flag();
    if (h.alfPresent) {
      h.alf[0] = b.flag();
      int chromaIdc = 0;
      if (h.alf[0]) {
        h.numAlfAps = (int)b.u(3);
        for (int i = 0; i < h.numAlfAps; i++) h.alfApsLuma[i] = (int)b.u(3);
        chromaIdc = (int)b.u(2);
        if (chromaIdc) h.alfApsChroma = (int)b.u(3);
        if (sps->ccalf) {
          for (int c = 0; c < 2; c++) {
            h.ccAlf[c] = b.flag();
            h.ccAlfApsId[c] = -1;
            if (h.ccAlf[c]) h.ccAlfApsId[c] = (int)b.u(3);
          }
        }
      }
      h.alf[1] = chromaIdc & 1;
      h.alf[2] = chromaIdc >> 1;
    } else {
      h.alf[0] = h.alf[1] = h.alf[2] = true;
    }
  }
  h.depQuant = !pps->depQuantIdc ? b.flag() : (pps->depQuantIdc - 1) != 0;
  h.signHiding = !h.depQuant ? b.flag() : false;
  if (pps->dbkCtrlPresent) {
    if (pps->dbkOverrideEnabled) {
      h.dbkOverridePresent = b.flag();
      if (h.dbkOverridePresent) h.dbkOverride = b.flag();
    }
    if (h.dbkOverride) {
      h.dbkDisable = b.flag();
      if (!h.dbkDisable) { h.betaOffsetDiv2 = b.se(); h.tcOffsetDiv2 = b.se(); }
    } else {
      h.dbkDisable = pps->dbkDisabled;
      h.betaOffsetDiv2 = pps->betaOffsetDiv2;
      h.tcOffsetDiv2 = pps->tcOffsetDiv2;
    }
  }
  if (sps->lmcs) {
    h.lmcs = b.flag();
    if (h.lmcs) {
      h.lmcsApsId = (int)b.u(2);
      h.lmcsChroma = b.flag();
    }
  }
  if (pps->phExtPresent) {
    const int n = (int)b.ue();
    for (int i = 0; i < n; i++) b.u(8);
  }
  h.valid = true;
}

// HLSyntaxReader::parseSliceHeader (VLCReader.cpp:2636). prevTid0Poc: POC of the previous TemporalId-0
// picture (DecLib::xUpdatePreviousTid0POC) for the POC MSB.
void parse_sh(Bits &b, SliceHeader &s, PicHeader &ph, const ParamSets &ps, int prevTid0Poc) {
  if (b.flag()) parse_ph(b, ph, ps);   // picture_header_in_slice_header_flag (JVET_Q0775)
  VVCP_CHECK(!ph.valid, "slice without a picture header");
  const PPS *pps = ps.pps(ph.ppsId);
  const SPS *sps = ps.sps(pps->spsId);
  const int lsb = (int)b.u(sps->bitsForPoc);
  if (s.idr()) s.poc = lsb;
  else {
    const int maxLsb = 1 << sps->bitsForPoc;
    const int prevLsb = prevTid0Poc & (maxLsb - 1), prevMsb = prevTid0Poc - prevLsb;
    int msb;
    if (lsb < prevLsb && prevLsb - lsb >= maxLsb / 2) msb = prevMsb + maxLsb;
    else if (lsb > prevLsb && lsb - prevLsb > maxLsb / 2) msb = prevMsb - maxLsb;
    else msb = prevMsb;
    s.poc = msb + lsb;
  }
  if (sps->subPicPresent) {   // slice_subpic_id (VLCReader.cpp:2696-2716); VTM 7.3 decodes a subpicture's
    // slices through the PPS slice map, the subpicture itself changes nothing else in the decoding
    int bits = sps->subPicIdSignalling ? sps->subPicIdLen
             : (ph.subPicIdSignalling ? ph.subPicIdLen : (pps->subPicIdSignalling ? pps->subPicIdLen : ceilLog2(sps->numSubPics)));
    if (bits) b.u(bits);
  }
  s.ctus.clear();
  if (!pps->rectSlice) {   // raster-scan slices: tiles in raster order
    int addr = 0, ntiles = 1;
    if (pps->numTiles() > 1) {
      addr = (int)b.u(ceilLog2(pps->numTiles()));
      ntiles = (int)b.ue() + 1;
    }
    s.sliceAddr = addr;
    for (int t = addr; t < addr + ntiles; t++) {
      const int tx = t % pps->numTileCols(), ty = t / pps->numTileCols();
      VVCP_CHECK(ty + 1 >= (int)pps->rowBd.size(), "slice extends past the last tile");
      add_tile_ctus(*pps, s.ctus, tx, ty);
    }
  } else {
    s.sliceAddr = 0;
    if (pps->numSlicesInPic > 1) s.sliceAddr = (int)b.u(ceilLog2(pps->numSlicesInPic));
    s.ctus = pps->rectSliceCtus[s.sliceAddr];
  }
  s.sliceType = (int)b.ue();
  VVCP_CHECK(s.sliceType > 2, "bad slice type");
  // inheritFromPicHeader (Slice.cpp:197)
  s.dbkDisable = ph.dbkDisable; s.betaOffsetDiv2 = ph.betaOffsetDiv2; s.tcOffsetDiv2 = ph.tcOffsetDiv2;
  s.sao[0] = ph.sao[0]; s.sao[1] = ph.sao[1];
  for (int c = 0; c < 3; c++) s.alf[c] = ph.alf[c];
  s.numAlfAps = ph.numAlfAps;
  for (int i = 0; i < 8; i++) s.alfApsLuma[i] = ph.alfApsLuma[i];
  s.alfApsChroma = ph.alfApsChroma;
  for (int c = 0; c < 2; c++) { s.ccAlf[c] = ph.ccAlf[c]; s.ccAlfApsId[c] = ph.ccAlfApsId[c]; }

  if (ph.rplPresent) {
    s.rpl[0] = ph.rpl[0]; s.rpl[1] = ph.rpl[1];
    s.rplIdx[0] = ph.rplIdx[0]; s.rplIdx[1] = ph.rplIdx[1];
  } else if (s.idr() && !sps->idrRplPresent) {
    s.rpl[0] = RPL(); s.rpl[1] = RPL();
  } else {
    for (int l = 0; l < 2; l++) {
      if (l == 1 && !pps->rpl1IdxPresent) {
        s.rplIdx[1] = s.rplIdx[0];
        if (s.rplIdx[1] != -1) {
          VVCP_CHECK(s.rplIdx[1] >= (int)sps->rpl[1].size(), "slice header: inherited list-1 RPL index out of range");
          s.rpl[1] = sps->rpl[1][s.rplIdx[1]];
        }
      } else {
        uint32_t spsFlag = 0;
        if (!sps->rpl[l].empty()) spsFlag = !pps->rplSpsIdc[l] ? b.u(1) : (uint32_t)(pps->rplSpsIdc[l] - 1);
        if (l == 0 || spsFlag) {
          if (!spsFlag) {
            parse_rpl(b, *sps, s.rpl[l]);
            s.rplIdx[l] = -1;
          } else {
            s.rplIdx[l] = sps->rpl[l].size() > 1 ? (int)b.u(ceilLog2((uint32_t)sps->rpl[l].size())) : 0;
            VVCP_CHECK(s.rplIdx[l] >= (int)sps->rpl[l].size(), "slice header: reference picture list index out of range");
            s.rpl[l] = sps->rpl[l][s.rplIdx[l]];
          }
        } else {
          s.rplIdx[1] = -1;
        }
      }
      if (l == 1 && s.rplIdx[1] == -1 && pps->rpl1IdxPresent) {
        // explicitly carried in the slice header (VLCReader.cpp:2918)
      }
      if (l == 1 && s.rplIdx[1] == -1) parse_rpl(b, *sps, s.rpl[1]);
      if (s.rpl[l].numLT) {
        for (int i = 0; i < s.rpl[l].num; i++) {
          if (!s.rpl[l].isLT[i]) continue;
          if (s.rpl[l].ltrpInSH) s.rpl[l].ident[i] = (int)b.u(sps->bitsForPoc);
          s.rpl[l].msbPresent[i] = b.flag();
          if (s.rpl[l].msbPresent[i]) s.rpl[l].msbCycle[i] = (int)b.ue();
        }
      }
    }
  }
  if (!ph.rplPresent && s.idr() && !sps->idrRplPresent) {
    s.numRef[0] = s.numRef[1] = 0;
  } else {
    if ((!s.isIntra() && s.rpl[0].num > 1) || (s.isInterB() && s.rpl[1].num > 1)) {
      if (b.flag()) {
        s.numRef[0] = (s.rpl[0].num > 1 ? (int)b.ue() : 0) + 1;
        if (s.isInterB()) s.numRef[1] = (s.rpl[1].num > 1 ? (int)b.ue() : 0) + 1;
        else s.numRef[1] = 0;
      } else {
        s.numRef[0] = std::min(s.rpl[0].num, pps->numRefDefault[0]);
        s.numRef[1] = s.isInterB() ? std::min(s.rpl[1].num, pps->numRefDefault[1]) : 0;
      }
    } else {
      s.numRef[0] = s.isIntra() ? 0 : 1;
      s.numRef[1] = s.isInterB() ? 1 : 0;
    }
  }
  if (s.isIntra()) s.numRef[0] = s.numRef[1] = 0;   // constructRefPicList (Slice.cpp:417)
  VVCP_CHECK(s.numRef[0] > VVCR_MAX_REF || s.numRef[1] > VVCR_MAX_REF, "too many active references");
  VVCP_CHECK(s.numRef[0] > s.rpl[0].num || s.numRef[1] > s.rpl[1].num, "more active references than list entries");
  s.cabacInit = false;
  if (pps->cabacInitPresent && !s.isIntra()) s.cabacInit = b.flag();
  s.colFromL0 = true;
  s.colRefIdx = 0;
  if (ph.tmvp) {
    if (s.isInterB()) s.colFromL0 = !pps->colFromL0Idc ? b.flag() : (pps->colFromL0Idc - 1) != 0;
    if (!s.isIntra() && ((s.colFromL0 && s.numRef[0] > 1) || (!s.colFromL0 && s.numRef[1] > 1))) s.colRefIdx = (int)b.ue();
    // indexes refPoc[colList] in the motion derivation (vvcp_mv.cpp)
    VVCP_CHECK(!s.isIntra() && s.colRefIdx >= s.numRef[s.colFromL0 ? 0 : 1], "slice header: collocated_ref_idx out of range");
  }
  std::memset(s.wp, 0, sizeof(s.wp));
  if ((pps->useWP && s.isInterP()) || (pps->wpBi && s.isInterB())) {   // parsePredWeightTable (VLCReader.cpp:3545)
    const int denomL = (int)b.ue();
    const int denomC = denomL + b.se();
    const int nl = s.isInterB() ? 2 : 1;
    for (int l = 0; l < nl; l++) {
      for (int r = 0; r < s.numRef[l]; r++) {
        s.wp[l][r][0][1] = denomL;
        s.wp[l][r][1][1] = s.wp[l][r][2][1] = denomC;
        s.wp[l][r][0][0] = b.u(1);
      }
      for (int r = 0; r < s.numRef[l]; r++) {
        const int f = (int)b.u(1);
        s.wp[l][r][1][0] = s.wp[l][r][2][0] = f;
      }
      for (int r = 0; r < s.numRef[l]; r++) {
        int (*w)[4] = s.wp[l][r];
        if (w[0][0]) {
          w[0][2] = b.se() + (1 << w[0][1]);
          w[0][3] = b.se();
        } else {
          w[0][2] = 1 << w[0][1];
          w[0][3] = 0;
        }
        if (w[1][0]) {
          const int range = 128;
          for (int c = 1; c < 3; c++) {
            w[c][2] = b.se() + (1 << w[c][1]);
            const int dOff = b.se();
            const int pred = range - ((range * w[c][2]) >> w[c][1]);
            w[c][3] = clip3(-range, range - 1, dOff + pred);
          }
        } else {
          for (int c = 1; c < 3; c++) { w[c][2] = 1 << w[c][1]; w[c][3] = 0; }
        }
      }
    }
  }
  s.qp = pps->initQp + b.se();
  s.cbQpDelta = s.crQpDelta = s.jcQpDelta = 0;
  if (pps->sliceChromaQpFlag) {
    s.cbQpDelta = b.se();
    s.crQpDelta = b.se();
    if (sps->jointCbCr) s.jcQpDelta = b.se();
  }
  s.chromaQpAdj = pps->cuChromaQpOffsetEnabled ? b.flag() : false;
  if (sps->sao && !ph.saoPresent) { s.sao[0] = b.flag(); s.sao[1] = b.flag(); }
  if (sps->alf && !ph.alfPresent) {
    s.alf[0] = b.flag();
    int chromaIdc = 0;
    if (s.alf[0]) {
      s.numAlfAps = (int)b.u(3);
      for (int i = 0; i < s.numAlfAps; i++) s.alfApsLuma[i] = (int)b.u(3);
      chromaIdc = (int)b.u(2);
      if (chromaIdc) s.alfApsChroma = (int)b.u(3);
    } else {
      s.numAlfAps = 0;
    }
    s.alf[1] = chromaIdc & 1;
    s.alf[2] = chromaIdc >> 1;
    if (sps->ccalf && s.alf[0]) {
      for (int c = 0; c < 2; c++) {
        s.ccAlf[c] = b.flag();
        s.ccAlfApsId[c] = -1;
        if (s.ccAlf[c]) s.ccAlfApsId[c] = (int)b.u(3);
      }
    } else {
      s.ccAlf[0] = s.ccAlf[1] = false;
      s.ccAlfApsId[0] = s.ccAlfApsId[1] = -1;
    }
  }
  if (pps->dbkCtrlPresent) {
    s.dbkOverride = (pps->dbkOverrideEnabled && !ph.dbkOverridePresent) ? b.flag() : false;
    if (s.dbkOverride) {
      s.dbkDisable = b.flag();
      if (!s.dbkDisable) { s.betaOffsetDiv2 = b.se(); s.tcOffsetDiv2 = b.se(); }
    } else {
      s.dbkDisable = ph.dbkDisable; s.betaOffsetDiv2 = ph.betaOffsetDiv2; s.tcOffsetDiv2 = ph.tcOffsetDiv2;
    }
  } else {
    s.dbkDisable = false; s.betaOffsetDiv2 = 0; s.tcOffsetDiv2 = 0;
  }
  if (pps->shExtPresent) {
    const int n = (int)b.ue();
    for (int i = 0; i < n; i++) b.u(8);
  }
  // entry points: one per tile start after the first CTU, and with entropy coding sync (WPP) one per CTU row
  // start of a tile (Slice::setNumEntryPoints, Slice.cpp:247)
  int nEntry = 0;
  for (size_t i = 1; i < s.ctus.size(); i++) {
    const int cx = s.ctus[i] % pps->widthInCtus, cy = s.ctus[i] / pps->widthInCtus;
    if (pps->colBd[pps->ctuToTileCol[cx]] == cx && (pps->rowBd[pps->ctuToTileRow[cy]] == cy || pps->entropySync)) nEntry++;
  }
  s.entryPoints.clear();
  if (nEntry > 0) {
    const int len = (int)b.ue() + 1;
    for (int i = 0; i < nEntry; i++) s.entryPoints.push_back(b.u(len) + 1);
  }
  // byte_alignment(): alignment_bit_equal_to_one, then zero bits up to the byte boundary
  VVCP_CHECK(b.u(1) != 1, "byte_alignment bit is not 1");
  while (!b.aligned()) VVCP_CHECK(b.u(1) != 0, "byte_alignment zero bit is not 0");
  s.dataOffset = b.byte_pos();
}

}  // namespace vvcp
