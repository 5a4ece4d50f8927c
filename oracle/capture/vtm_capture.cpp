// vtm_capture — TEST INFRASTRUCTURE (never shipped, never on the product path).
//
// Runs the reference decoder (VTM 7.3 DecApp/DecLib, compiled from /root/reference by oracle/ref.mk)
// and records, per decoded picture, everything the MI355X reconstruction path consumes plus golden
// intermediate results of the reference:
//   * descriptors  — CU / PU / TU tables with derived MVs, coefficient levels, QPs, motion field,
//                    SAO / ALF / CC-ALF / LMCS / WP parameters (what a host parser hands to vvcr_submit)
//   * golden planes — prediction (MC-only and final), residual, pre-loop-filter reconstruction,
//                    deblocking input/output, SAO output, ALF output (= the decoded picture)
// Interposition is link-time only (GNU ld --wrap, list in wraps.txt): each __wrap_X calls __real_X
// and copies the reference result out. No reference source is copied or modified.
//
// Usage: VVCR_CAPTURE_DIR=<dir> vtm_capture -b stream.bin [-o out.yuv]   (DecoderApp options)
// Output: <dir>/pic_<decodeidx>.cap  — chunk format read by vvc_amd/capfile.py
//
// Built with -DVVCR_DROPIN (oracle/ref.mk: oracle/_ref/vtm_vvcr) the same source is the drop-in of
// DecoderApp (DecApp / DecLib / DecCu unchanged, linked against libvvcr.so) whose
// reconstruction and loop filters are REPLACED by libvvcr. DecCu still parses and derives motion; its
// calls into the reference's prediction, transforms and LMCS mapping return without running (the
// wrappers below only record what the descriptors need: TU QPs, GEO candidates), and
// DecLib::executeLoopFilters (DecLib.cpp:560) is replaced: the picture's descriptors go to
// vvcr_begin_picture / vvcr_submit / vvcr_set_loop_filter_params / vvcr_end_picture, libvvcr's final
// picture (vvcr_read_picture) fills the reference's picture buffer (which the reference never wrote)
// before DecLib's MD5 check, DecApp::xWriteOutput and later pictures' parsing read it, and libvvcr's
// DMVR refinements (vvcr_get_dmvr_deltas) feed CS::setRefinedMotionField (DecLib.cpp:579), so later
// pictures' temporal candidates come from libvvcr too. The calls into the reference's reconstruction
// that ran are counted and reported (zero).

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <map>
#include <fstream>
#include <iostream>
#include <list>
#include <algorithm>
#include <array>
#include <sstream>
#include <functional>
#include <memory>
#include <utility>

// white-box access to the reference's private state (layout is unaffected by access specifiers)
#define private public
#define protected public
#include "DecApp.h"
#include "DecoderLib/DecLib.h"
#include "CommonLib/CodingStructure.h"
#include "CommonLib/Picture.h"
#include "CommonLib/UnitTools.h"
#include "CommonLib/InterPrediction.h"
#include "CommonLib/IntraPrediction.h"
#include "CommonLib/TrQuant.h"
#include "CommonLib/LoopFilter.h"
#include "CommonLib/SampleAdaptiveOffset.h"
#include "CommonLib/AdaptiveLoopFilter.h"
#include "CommonLib/Reshape.h"
#include "CommonLib/dtrace_next.h"
namespace vtm_mip {
#include "CommonLib/MipData.h"
}
#undef private
#undef protected

// ---------------------------------------------------------------------------------------------
// chunk writer
// ---------------------------------------------------------------------------------------------
struct Chunk { char dtype; std::vector<uint64_t> dims; std::vector<uint8_t> bytes; };
struct CapFile {
  FILE *f = nullptr;
  std::map<std::string, Chunk> *mem = nullptr;   // in-memory chunks instead of a file (drop-in mode)
  void open(const std::string &p) {
    f = fopen(p.c_str(), "wb");
    if (!f) { perror(p.c_str()); exit(3); }
    fwrite("VVCRCAP1", 1, 8, f);
  }
  void close() { if (f) fclose(f); f = nullptr; }
  // dtype: 'b' int8, 'B' uint8, 'h' int16, 'H' uint16, 'i' int32, 'q' int64
  void put(const char *name, char dtype, std::vector<uint64_t> dims, const void *data, size_t elsz) {
    if (mem) {
      uint64_t n = 1;
      for (auto d : dims) n *= d;
      Chunk &c = (*mem)[name];
      c.dtype = dtype;
      c.dims = dims;
      c.bytes.assign((const uint8_t *)data, (const uint8_t *)data + n * elsz);
      return;
    }
    char nm[24] = {0};
    strncpy(nm, name, 23);
    fwrite(nm, 1, 24, f);
    uint32_t dt = (uint32_t)dtype, nd = (uint32_t)dims.size();
    fwrite(&dt, 4, 1, f); fwrite(&nd, 4, 1, f);
    uint64_t n = 1;
    for (auto d : dims) { fwrite(&d, 8, 1, f); n *= d; }
    uint64_t nb = n * elsz;
    fwrite(&nb, 8, 1, f);
    if (nb) fwrite(data, 1, nb, f);
  }
  void i32(const char *name, const std::vector<int32_t> &v, std::vector<uint64_t> dims) { put(name, 'i', dims, v.data(), 4); }
  void i16(const char *name, const std::vector<int16_t> &v, std::vector<uint64_t> dims) { put(name, 'h', dims, v.data(), 2); }
  void u8 (const char *name, const std::vector<uint8_t> &v, std::vector<uint64_t> dims) { put(name, 'B', dims, v.data(), 1); }
};

// ---------------------------------------------------------------------------------------------
// per-picture capture state
// ---------------------------------------------------------------------------------------------
struct Plane { int w = 0, h = 0; std::vector<int16_t> d; void init(int W, int H, int16_t v) { w = W; h = H; d.assign((size_t)W * H, v); } };

struct PicCapture {
  const CodingStructure *cs = nullptr;
  Plane pmc[3], pfin[3], resi[3];      // MC-only prediction, final prediction, final residual
  Plane stage[6][3];                   // prelf, dbkin, dbk, sao, alf  (index by enum)
  bool  haveStage[6] = {false};
  std::map<const CodingUnit *, std::array<int32_t, 12>> geo;   // per GEO CU: two uni candidates
  std::map<const TransformUnit *, std::array<int32_t, 6>> tuqp; // per TU: Qp non-TS / TS per comp
  bool active = false;
};
enum { ST_PRELF = 0, ST_DBKIN, ST_DBK, ST_SAO, ST_ALF, ST_N };
static const char *kStageName[ST_N] = {"prelf", "dbkin", "dbk", "sao", "alf"};

static std::string g_dir;
static bool g_trace = getenv("VVCR_CAPTURE_TRACE") != nullptr;
#define TR(x) do { if (g_trace) fprintf(stderr, "[cap] %s\n", x); } while (0)
static int g_picCounter = 0;
static PicCapture g_cap;
// calls into the reference's reconstruction and loop filters that actually ran (__real_*): the drop-in
// build runs none of them (main reports the counts, tests/test_dropin_gpu.py checks they are zero)
enum { RC_FILTER_HOR, RC_MC, RC_MC_GEO, RC_INTRA, RC_ITX, RC_DBK, RC_SAO, RC_N };
static const char *kRcName[RC_N] = {"InterpolationFilter::filterHor", "InterPrediction::motionCompensation",
                                    "InterPrediction::motionCompensationGeo", "IntraPrediction::predIntra*",
                                    "TrQuant::invTransformNxN", "LoopFilter::loopFilterPic", "SampleAdaptiveOffset::SAOProcess"};
static long g_refCalls[RC_N] = {};
#ifdef VVCR_DROPIN
static const bool g_replace = true;    // the reference's reconstruction is replaced, not run
#else
static const bool g_replace = false;
#endif

static void initPlanes(const CodingStructure &cs) {
  if (g_dir.empty()) return;   // not capturing: wrappers only forward
  g_cap = PicCapture();
  g_cap.cs = &cs;
  g_cap.active = true;
  const Picture &pic = *cs.picture;
  for (int c = 0; c < 3; c++) {
    const CompArea &a = pic.blocks[c];
    g_cap.pmc[c].init(a.width, a.height, (int16_t)-32768);
    g_cap.pfin[c].init(a.width, a.height, (int16_t)-32768);
    g_cap.resi[c].init(a.width, a.height, 0);
  }
}

// locate a buffer that views the CodingStructure pred / resi storage. Without KEEP_PRED_AND_RESI_SIGNALS
// those buffers are CTU-sized and indexed with CTU-local coordinates (Picture::getBuf Picture.cpp:841-850),
// so the absolute position is the current CTU origin (set by every wrapper that knows its unit) + offset.
static int g_ctuX = 0, g_ctuY = 0;
static void setCtu(const CodingStructure &cs, int lumaX, int lumaY) {
  const int m = ~(int)(cs.pcv->maxCUWidth - 1);
  g_ctuX = lumaX & m; g_ctuY = lumaY & m;
}
static bool locate(const CodingStructure &cs, PictureType type, int comp, const Pel *p, int &x, int &y) {
  const PelStorage *st = type == PIC_PREDICTION ? &cs.m_pred : &cs.m_resi;
  if (st->bufs.size() <= (size_t)comp) return false;
  const PelBuf &b = st->bufs[comp];
  ptrdiff_t off = p - b.buf;
  if (off < 0 || off >= (ptrdiff_t)b.stride * (ptrdiff_t)b.height) return false;
  const int sc = comp ? 1 : 0;
  y = (int)(off / b.stride) + (g_ctuY >> sc);
  x = (int)(off % b.stride) + (g_ctuX >> sc);
  return true;
}

static void copyBlock(Plane &dst, const PelBuf &src, int x0, int y0) {
  for (int y = 0; y < (int)src.height; y++)
    for (int x = 0; x < (int)src.width; x++) {
      int X = x0 + x, Y = y0 + y;
      if (X < dst.w && Y < dst.h) dst.d[(size_t)Y * dst.w + X] = src.buf[y * src.stride + x];
    }
}

static void snapBuf(Plane *dst, const CPelUnitBuf &buf) {
  for (int c = 0; c < 3; c++) {
    const CPelBuf &b = buf.bufs[c];
    dst[c].init(b.width, b.height, 0);
    for (int y = 0; y < (int)b.height; y++) memcpy(&dst[c].d[(size_t)y * b.width], b.buf + y * b.stride, b.width * 2);
  }
}

static void snapStage(int st) {
  if (!g_cap.active) return;
  snapBuf(g_cap.stage[st], g_cap.cs->picture->getRecoBuf());
  g_cap.haveStage[st] = true;
}

// ---------------------------------------------------------------------------------------------
// descriptor dump
// ---------------------------------------------------------------------------------------------
struct Hdr {
  std::vector<std::string> k;
  std::vector<int64_t> v;
  void add(const std::string &key, int64_t val) { k.push_back(key); v.push_back(val); }
};

static void dumpDescriptors(CapFile &F, DecLib &dec, const CodingStructure &cs) {
  const Slice &sl = *cs.slice;
  const SPS &sps = *cs.sps;
  const PPS &pps = *cs.pps;
  const PicHeader &ph = *cs.picHeader;
  const PreCalcValues &pcv = *cs.pcv;
  Hdr H;
  H.add("poc", sl.getPOC());
  H.add("decode_idx", g_picCounter);
  H.add("width", pps.getPicWidthInLumaSamples());
  H.add("height", pps.getPicHeightInLumaSamples());
  H.add("chroma_format", (int)sps.getChromaFormatIdc());
  H.add("bitdepth_y", sps.getBitDepth(CHANNEL_TYPE_LUMA));
  H.add("bitdepth_c", sps.getBitDepth(CHANNEL_TYPE_CHROMA));
  H.add("ctu_size", sps.getMaxCUWidth());
  H.add("ctu_log2", pcv.maxCUWidthLog2);
  H.add("width_in_ctus", pcv.widthInCtus);
  H.add("height_in_ctus", pcv.heightInCtus);
  H.add("slice_type", (int)sl.getSliceType());
  H.add("slice_qp", sl.getSliceQp());
  H.add("tid", sl.getTLayer());
  H.add("num_slices", (int)cs.picture->slices.size());
  H.add("dual_tree", CS::isDualITree(cs) ? 1 : 0);
  H.add("num_ref_l0", sl.getNumRefIdx(REF_PIC_LIST_0));
  H.add("num_ref_l1", sl.getNumRefIdx(REF_PIC_LIST_1));
  H.add("check_ldc", sl.getCheckLDC() ? 1 : 0);
  H.add("col_from_l0", sl.getColFromL0Flag() ? 1 : 0);
  H.add("dep_quant", ph.getDepQuantEnabledFlag() ? 1 : 0);
  H.add("sign_hiding", ph.getSignDataHidingEnabledFlag() ? 1 : 0);
  H.add("dbk_disable", sl.getDeblockingFilterDisable() ? 1 : 0);
  H.add("dbk_beta_offset_div2", sl.getDeblockingFilterBetaOffsetDiv2());
  H.add("dbk_tc_offset_div2", sl.getDeblockingFilterTcOffsetDiv2());
  H.add("lf_across_slices", pps.getLoopFilterAcrossSlicesEnabledFlag() ? 1 : 0);
  H.add("lf_across_tiles", pps.getLoopFilterAcrossTilesEnabledFlag() ? 1 : 0);
  H.add("num_tiles", pps.getNumTiles());
  H.add("entropy_sync", pps.getEntropyCodingSyncEnabledFlag() ? 1 : 0);
  // virtual boundaries (only when loop filtering across them is disabled do they change decoding)
  H.add("vb_disabled", ph.getLoopFilterAcrossVirtualBoundariesDisabledFlag() ? 1 : 0);
  H.add("num_vb_ver", ph.getNumVerVirtualBoundaries());
  H.add("num_vb_hor", ph.getNumHorVirtualBoundaries());
  for (int i = 0; i < 3; i++) {
    H.add(std::string("vb_ver") + char('0' + i), i < (int)ph.getNumVerVirtualBoundaries() ? ph.getVirtualBoundariesPosX(i) : 0);
    H.add(std::string("vb_hor") + char('0' + i), i < (int)ph.getNumHorVirtualBoundaries() ? ph.getVirtualBoundariesPosY(i) : 0);
  }
  // luma-adaptive deblocking (SPS)
  H.add("ladf_num", sps.getLadfEnabled() ? sps.getLadfNumIntervals() : 0);
  for (int k = 0; k < 5; k++) {
    const bool on = sps.getLadfEnabled() && k < sps.getLadfNumIntervals();
    H.add(std::string("ladf_qp_offset") + char('0' + k), on ? sps.getLadfQpOffset(k) : 0);
    H.add(std::string("ladf_lower_bound") + char('0' + k), on && k > 0 ? sps.getLadfIntervalLowerBound(k) : 0);
  }
  H.add("sao_enabled", sps.getSAOEnabledFlag() ? 1 : 0);
  H.add("sao_luma", sl.getSaoEnabledFlag(CHANNEL_TYPE_LUMA) ? 1 : 0);
  H.add("sao_chroma", sl.getSaoEnabledFlag(CHANNEL_TYPE_CHROMA) ? 1 : 0);
  H.add("alf_enabled", sps.getALFEnabledFlag() ? 1 : 0);
  for (int c = 0; c < 3; c++) H.add(std::string("alf_slice_en") + char('0' + c), sl.getTileGroupAlfEnabledFlag((ComponentID)c) ? 1 : 0);
  H.add("alf_num_aps", sl.getTileGroupNumAps());
  H.add("alf_aps_chroma", sl.getTileGroupApsIdChroma());
  H.add("ccalf_en_cb", sl.m_ccAlfFilterParam.ccAlfFilterEnabled[0] ? 1 : 0);
  H.add("ccalf_en_cr", sl.m_ccAlfFilterParam.ccAlfFilterEnabled[1] ? 1 : 0);
  H.add("lmcs_enabled", (sps.getUseLmcs() && ph.getLmcsEnabledFlag()) ? 1 : 0);
  H.add("lmcs_chroma_scale", ph.getLmcsChromaResidualScaleFlag() ? 1 : 0);
  H.add("lmcs_ctu_flag", dec.m_cReshaper.getCTUFlag() ? 1 : 0);
  H.add("lmcs_slice_flag", dec.m_cReshaper.getSliceReshaperInfo().getUseSliceReshaper() ? 1 : 0);
  H.add("lmcs_min_bin", dec.m_cReshaper.getSliceReshaperInfo().reshaperModelMinBinIdx);
  H.add("lmcs_max_bin", dec.m_cReshaper.getSliceReshaperInfo().reshaperModelMaxBinIdx);
  H.add("bdof_enabled", (sps.getBDOFEnabledFlag() && !ph.getDisBdofFlag()) ? 1 : 0);
  H.add("dmvr_enabled", (sps.getUseDMVR() && !ph.getDisDmvrFlag()) ? 1 : 0);
  H.add("prof_enabled", (sps.getUsePROF() && !ph.getDisProfFlag()) ? 1 : 0);
  H.add("lfnst_enabled", sps.getUseLFNST() ? 1 : 0);
  H.add("mts_intra", sps.getUseIntraMTS() ? 1 : 0);
  H.add("mts_inter", sps.getUseInterMTS() ? 1 : 0);
  H.add("sbt", sps.getUseSBT() ? 1 : 0);
  H.add("wp_p", pps.getUseWP() ? 1 : 0);
  H.add("wp_b", pps.getWPBiPred() ? 1 : 0);
  H.add("scaling_list", sps.getScalingListFlag() ? 1 : 0);
  H.add("wrap_around", sps.getWrapAroundEnabledFlag() ? 1 : 0);
  H.add("max_tb_size", sps.getMaxTbSize());
  H.add("log2_max_ts", pps.getLog2MaxTransformSkipBlockSize());
  H.add("joint_cbcr", sps.getJointCbCrEnabledFlag() ? 1 : 0);
  H.add("joint_cbcr_sign", ph.getJointCbCrSignFlag() ? 1 : 0);
  H.add("use_mts", sps.getUseMTS() ? 1 : 0);
  H.add("implicit_mts", sps.getUseImplicitMTS() ? 1 : 0);
  H.add("bdpcm_enabled", sps.m_BDPCMEnabled);
  H.add("isp_enabled", sps.getUseISP() ? 1 : 0);
  H.add("mip_enabled", sps.getUseMIP() ? 1 : 0);
  H.add("lm_chroma", sps.getUseLMChroma() ? 1 : 0);
  H.add("ciip_enabled", sps.getUseCiip() ? 1 : 0);
  H.add("bcw_enabled", sps.getUseBcw() ? 1 : 0);
  H.add("min_qp_ts", 4 + sps.getMinQpPrimeTsMinus4(CHANNEL_TYPE_LUMA));
  H.add("chroma_qp_off_cb", pps.getQpOffset(COMPONENT_Cb) + sl.getSliceChromaQpDelta(COMPONENT_Cb));
  H.add("chroma_qp_off_cr", pps.getQpOffset(COMPONENT_Cr) + sl.getSliceChromaQpDelta(COMPONENT_Cr));
  H.add("chroma_qp_off_jc", pps.getQpOffset(JOINT_CbCr) + sl.getSliceChromaQpDelta(JOINT_CbCr));
  H.add("ladf_enabled", sps.getLadfEnabled() ? 1 : 0);
  H.add("plt_enabled", sps.getPLTMode() ? 1 : 0);
  H.add("cu_chroma_qp_adj", sl.getUseChromaQpAdj() ? 1 : 0);
  H.add("pps_cb_qp_offset", pps.getQpOffset(COMPONENT_Cb));
  H.add("pps_cr_qp_offset", pps.getQpOffset(COMPONENT_Cr));
  H.add("picture_output", ph.getPicOutputFlag() ? 1 : 0);
  H.add("alf_vb_luma", dec.m_cALF.m_alfVBLumaPos);
  H.add("alf_vb_chroma", dec.m_cALF.m_alfVBChmaPos);
  H.add("virtual_bnd", ph.getLoopFilterAcrossVirtualBoundariesDisabledFlag() ? 1 : 0);
  H.add("mmvd_fpel", ph.getDisFracMMVD() ? 1 : 0);
  {
    std::string keys;
    for (size_t i = 0; i < H.k.size(); i++) keys += (i ? "," : "") + H.k[i];
    F.put("hdr_keys", 'B', {keys.size()}, keys.data(), 1);
    F.put("hdr_vals", 'q', {H.v.size()}, H.v.data(), 8);
  }

  // reference lists (POCs; the decoded picture with that POC is the reference)
  {
    std::vector<int32_t> r(2 * MAX_NUM_REF, -1), lt(2 * MAX_NUM_REF, 0);
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < sl.getNumRefIdx((RefPicList)l); i++) {
        r[l * MAX_NUM_REF + i] = sl.getRefPOC((RefPicList)l, i);
        lt[l * MAX_NUM_REF + i] = sl.getRefPic((RefPicList)l, i)->longTerm ? 1 : 0;
      }
    F.i32("ref_poc", r, {2, (uint64_t)MAX_NUM_REF});
    F.i32("ref_lt", lt, {2, (uint64_t)MAX_NUM_REF});
    // weighted prediction tables: [list][ref][comp][present, log2denom, weight, offset, w, o, offset(shifted)]
    std::vector<int32_t> wp(2 * MAX_NUM_REF * 3 * 7, 0);
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < sl.getNumRefIdx((RefPicList)l); i++) {
        WPScalingParam *p = nullptr;
        sl.getWpScaling((RefPicList)l, i, p);
        if (!p) continue;
        for (int c = 0; c < 3; c++) {
          int32_t *o = &wp[((l * MAX_NUM_REF + i) * 3 + c) * 7];
          o[0] = p[c].bPresentFlag; o[1] = p[c].uiLog2WeightDenom; o[2] = p[c].iWeight; o[3] = p[c].iOffset;
          o[4] = p[c].w; o[5] = p[c].o; o[6] = p[c].offset;
        }
      }
    F.i32("wp", wp, {2, (uint64_t)MAX_NUM_REF, 3, 7});
  }

  // tile layout in CTUs (PPS::getTileColumnBd / getTileRowBd); bd[n] = picture size in CTUs
  {
    std::vector<int32_t> cb, rb;
    for (uint32_t i = 0; i < pps.getNumTileColumns(); i++) cb.push_back((int32_t)pps.getTileColumnBd(i));
    cb.push_back((int32_t)pcv.widthInCtus);
    for (uint32_t i = 0; i < pps.getNumTileRows(); i++) rb.push_back((int32_t)pps.getTileRowBd(i));
    rb.push_back((int32_t)pcv.heightInCtus);
    F.i32("tile_col_bd", cb, {(uint64_t)cb.size()});
    F.i32("tile_row_bd", rb, {(uint64_t)rb.size()});
  }

  // chroma QP mapping: mapped[c][qp + 64] for qp in [-64, 63]
  {
    std::vector<int32_t> m(3 * 128, 0);
    for (int c = 1; c < 3; c++)
      for (int q = -sps.getQpBDOffset(CHANNEL_TYPE_CHROMA); q < 64; q++) m[c * 128 + q + 64] = sps.getMappedChromaQpValue((ComponentID)c, q);
    F.i32("chroma_qp_map", m, {3, 128});
    std::vector<int32_t> j(128, 0);   // JOINT_CbCr mapping (QpParam with useJQP, Quant.cpp:121)
    for (int q = -sps.getQpBDOffset(CHANNEL_TYPE_CHROMA); q < 64; q++) j[q + 64] = sps.getMappedChromaQpValue(JOINT_CbCr, q);
    F.i32("chroma_qp_map_jc", j, {128});
  }

  TR("hdr+ref+qp done");
  // index maps
  std::map<const CodingUnit *, int> cuIdx;
  std::map<const PredictionUnit *, int> puIdx;
  std::map<const TransformUnit *, int> tuIdx;
  for (size_t i = 0; i < cs.cus.size(); i++) cuIdx[cs.cus[i]] = (int)i;
  for (size_t i = 0; i < cs.pus.size(); i++) puIdx[cs.pus[i]] = (int)i;
  for (size_t i = 0; i < cs.tus.size(); i++) tuIdx[cs.tus[i]] = (int)i;

  // ---- CU table
  enum { CU_X, CU_Y, CU_W, CU_H, CU_CX, CU_CY, CU_CW, CU_CH, CU_CHTYPE, CU_PREDMODE, CU_QP, CU_TREETYPE, CU_MODETYPE,
         CU_SKIP, CU_MMVDSKIP, CU_AFFINE, CU_AFFINETYPE, CU_GEO, CU_BDPCM, CU_BDPCMC, CU_IMV, CU_ROOTCBF, CU_SBTINFO,
         CU_MTSFLAG, CU_LFNST, CU_BCW, CU_MIP, CU_ISP, CU_SMVD, CU_ACT, CU_CQPADJ, CU_DEPTH, CU_QTDEPTH, CU_FIRSTPU,
         CU_NPU, CU_FIRSTTU, CU_NTU, CU_SLICE, CU_YVALID, CU_CVALID, CU_NF };
  std::vector<int32_t> cut(cs.cus.size() * CU_NF, 0);
  for (size_t i = 0; i < cs.cus.size(); i++) {
    const CodingUnit &cu = *cs.cus[i];
    int32_t *o = &cut[i * CU_NF];
    Position lp = cu.lumaPos(); Size ls = cu.lumaSize();
    o[CU_X] = lp.x; o[CU_Y] = lp.y; o[CU_W] = ls.width; o[CU_H] = ls.height;
    if (cu.chromaFormat != CHROMA_400 && cu.blocks.size() > 1 && cu.blocks[1].valid()) {
      o[CU_CX] = cu.blocks[1].x; o[CU_CY] = cu.blocks[1].y; o[CU_CW] = cu.blocks[1].width; o[CU_CH] = cu.blocks[1].height;
    }
    o[CU_CHTYPE] = cu.chType; o[CU_PREDMODE] = cu.predMode; o[CU_QP] = cu.qp; o[CU_TREETYPE] = cu.treeType;
    o[CU_MODETYPE] = cu.modeType; o[CU_SKIP] = cu.skip; o[CU_MMVDSKIP] = cu.mmvdSkip; o[CU_AFFINE] = cu.affine;
    o[CU_AFFINETYPE] = cu.affineType; o[CU_GEO] = cu.geoFlag; o[CU_BDPCM] = cu.bdpcmMode; o[CU_BDPCMC] = cu.bdpcmModeChroma;
    o[CU_IMV] = cu.imv; o[CU_ROOTCBF] = cu.rootCbf; o[CU_SBTINFO] = cu.sbtInfo; o[CU_MTSFLAG] = cu.mtsFlag;
    o[CU_LFNST] = cu.lfnstIdx; o[CU_BCW] = cu.BcwIdx; o[CU_MIP] = cu.mipFlag; o[CU_ISP] = cu.ispMode; o[CU_SMVD] = cu.smvdMode;
    o[CU_ACT] = cu.colorTransform; o[CU_CQPADJ] = cu.chromaQpAdj; o[CU_DEPTH] = cu.depth; o[CU_QTDEPTH] = cu.qtDepth;
    o[CU_FIRSTPU] = cu.firstPU ? puIdx[cu.firstPU] : -1;
    int np = 0; for (const PredictionUnit *p = cu.firstPU; p; p = (p == cu.lastPU) ? nullptr : p->next) np++;
    o[CU_NPU] = np;
    o[CU_FIRSTTU] = cu.firstTU ? tuIdx[cu.firstTU] : -1;
    int nt = 0; for (const TransformUnit *t = cu.firstTU; t; t = (t == cu.lastTU) ? nullptr : t->next) nt++;
    o[CU_NTU] = nt;
    o[CU_SLICE] = cu.slice ? (int)cu.slice->getSliceID() : 0;
    o[CU_YVALID] = cu.Y().valid(); o[CU_CVALID] = (cu.chromaFormat != CHROMA_400 && cu.Cb().valid());
  }
  TR("cu table");
  F.i32("cu", cut, {cs.cus.size(), (uint64_t)CU_NF});

  // ---- PU table
  enum { PU_CU, PU_X, PU_Y, PU_W, PU_H, PU_CX, PU_CY, PU_CW, PU_CH, PU_CHTYPE, PU_IDIR_L, PU_IDIR_C, PU_FIDIR_L, PU_FIDIR_C,
         PU_MIPT, PU_MRL, PU_MERGE, PU_REGMERGE, PU_MERGEIDX, PU_GEODIR, PU_GEOI0, PU_GEOI1, PU_MMVD, PU_INTERDIR,
         PU_MV0X, PU_MV0Y, PU_MV1X, PU_MV1Y, PU_REF0, PU_REF1, PU_MRGTYPE, PU_MVREFINE, PU_CIIP,
         PU_AFF0, /* 12 ints: mvAffi[l][k].hor/ver */ PU_DMVR_OFF = PU_AFF0 + 12, PU_BDOF, PU_DMVR, PU_NF };
  std::vector<int32_t> put(cs.pus.size() * PU_NF, 0);
  std::vector<int32_t> dmvrPool;
  for (size_t i = 0; i < cs.pus.size(); i++) {
    const PredictionUnit &pu = *cs.pus[i];
    int32_t *o = &put[i * PU_NF];
    o[PU_CU] = cuIdx[pu.cu];
    Position lp = pu.lumaPos(); Size ls = pu.lumaSize();
    o[PU_X] = lp.x; o[PU_Y] = lp.y; o[PU_W] = ls.width; o[PU_H] = ls.height;
    if (pu.chromaFormat != CHROMA_400 && pu.blocks.size() > 1 && pu.blocks[1].valid()) {
      o[PU_CX] = pu.blocks[1].x; o[PU_CY] = pu.blocks[1].y; o[PU_CW] = pu.blocks[1].width; o[PU_CH] = pu.blocks[1].height;
    }
    o[PU_CHTYPE] = pu.chType;
    o[PU_IDIR_L] = pu.intraDir[0]; o[PU_IDIR_C] = pu.intraDir[1];
    o[PU_FIDIR_L] = (CU::isIntra(*pu.cu) && pu.Y().valid()) ? PU::getFinalIntraMode(pu, CHANNEL_TYPE_LUMA) : -1;
    o[PU_FIDIR_C] = (CU::isIntra(*pu.cu) && pu.chromaFormat != CHROMA_400 && pu.Cb().valid()) ? PU::getFinalIntraMode(pu, CHANNEL_TYPE_CHROMA) : -1;
    o[PU_MIPT] = pu.mipTransposedFlag; o[PU_MRL] = pu.multiRefIdx;
    o[PU_MERGE] = pu.mergeFlag; o[PU_REGMERGE] = pu.regularMergeFlag; o[PU_MERGEIDX] = pu.mergeIdx;
    o[PU_GEODIR] = pu.geoSplitDir; o[PU_GEOI0] = pu.geoMergeIdx0; o[PU_GEOI1] = pu.geoMergeIdx1;
    o[PU_MMVD] = pu.mmvdMergeFlag; o[PU_INTERDIR] = pu.interDir;
    o[PU_MV0X] = pu.mv[0].hor; o[PU_MV0Y] = pu.mv[0].ver; o[PU_MV1X] = pu.mv[1].hor; o[PU_MV1Y] = pu.mv[1].ver;
    o[PU_REF0] = pu.refIdx[0]; o[PU_REF1] = pu.refIdx[1];
    o[PU_MRGTYPE] = pu.mergeType; o[PU_MVREFINE] = pu.mvRefine; o[PU_CIIP] = pu.ciipFlag;
    for (int l = 0; l < 2; l++)
      for (int k = 0; k < 3; k++) { o[PU_AFF0 + (l * 3 + k) * 2] = pu.mvAffi[l][k].hor; o[PU_AFF0 + (l * 3 + k) * 2 + 1] = pu.mvAffi[l][k].ver; }
    o[PU_DMVR_OFF] = -1;
    bool isInterPU = CU::isInter(*pu.cu);
    // reference decisions (InterPrediction.cpp:1584-1638): motionCompensation(cu) sets mvRefine=true around MC
    if (isInterPU && pu.interDir == 3 && !pu.cu->geoFlag) {
      PredictionUnit &mp = const_cast<PredictionUnit &>(pu);
      bool saved = mp.mvRefine; mp.mvRefine = true;
      o[PU_DMVR] = PU::checkDMVRCondition(pu) ? 1 : 0;
      mp.mvRefine = saved;
      WPScalingParam *wp0, *wp1;
      sl.getWpScaling(REF_PIC_LIST_0, pu.refIdx[0], wp0);
      sl.getWpScaling(REF_PIC_LIST_1, pu.refIdx[1], wp1);
      bool bio = false;
      if (sps.getBDOFEnabledFlag() && !ph.getDisBdofFlag() && !pu.cu->affine && pu.mergeType == MRG_TYPE_DEFAULT_N) {
        bool c0 = !((wp0[0].bPresentFlag || wp0[1].bPresentFlag || wp0[2].bPresentFlag || wp1[0].bPresentFlag || wp1[1].bPresentFlag || wp1[2].bPresentFlag) && sl.getSliceType() == B_SLICE);
        bool c1 = !(pps.getUseWP() && sl.getSliceType() == P_SLICE);
        bio = c0 && c1 && PU::isBiPredFromDifferentDirEqDistPoc(pu) && pu.Y().height >= 8 && pu.Y().width >= 8 && pu.Y().height * pu.Y().width >= 128;
        if (pu.ciipFlag || pu.cu->smvdMode || (sps.getUseBcw() && pu.cu->BcwIdx != BCW_DEFAULT)) bio = false;
      }
      o[PU_BDOF] = bio ? 1 : 0;
    }
    // DMVR refinement deltas per 16x16 sub-block (still held in mvdL0SubPu until CS::setRefinedMotionField,
    // which runs after deblocking: DecLib.cpp:579-580), in xProcessDMVR raster order
    if (o[PU_DMVR]) {
      o[PU_DMVR_OFF] = (int32_t)(dmvrPool.size() / 2);
      const int dy = std::min<int>(pu.lumaSize().height, DMVR_SUBCU_HEIGHT), dx = std::min<int>(pu.lumaSize().width, DMVR_SUBCU_WIDTH);
      const int n = (pu.lumaSize().height / dy) * (pu.lumaSize().width / dx);
      for (int k = 0; k < n; k++) { dmvrPool.push_back(pu.mvdL0SubPu[k].hor); dmvrPool.push_back(pu.mvdL0SubPu[k].ver); }
    }
  }
  TR("pu table");
  F.i32("pu", put, {cs.pus.size(), (uint64_t)PU_NF});
  F.i32("dmvr_delta", dmvrPool, {dmvrPool.size() / 2, 2});

  // ---- TU table + coefficient pool
  enum { TU_CU, TU_CHTYPE, TU_DEPTH, TU_NORESI, TU_JCCR, TU_CADJ,
         TU_B0 /* per comp: x,y,w,h,cbf,mts,coefoff,qp,qpts,(9) */, TU_NF = TU_B0 + 27 };
  std::vector<int32_t> tut(cs.tus.size() * TU_NF, 0);
  std::vector<int32_t> coef;
  for (size_t i = 0; i < cs.tus.size(); i++) {
    const TransformUnit &tu = *cs.tus[i];
    int32_t *o = &tut[i * TU_NF];
    o[TU_CU] = cuIdx[tu.cu]; o[TU_CHTYPE] = tu.chType; o[TU_DEPTH] = tu.depth; o[TU_NORESI] = tu.noResidual;
    o[TU_JCCR] = tu.jointCbCr; o[TU_CADJ] = tu.m_chromaResScaleInv;
    auto q = g_cap.tuqp.find(&tu);
    for (int c = 0; c < 3; c++) {
      int32_t *b = &o[TU_B0 + c * 9];
      b[6] = -1; b[7] = -1000; b[8] = -1000;
      if ((size_t)c >= tu.blocks.size() || !tu.blocks[c].valid()) continue;
      const CompArea &a = tu.blocks[c];
      b[0] = a.x; b[1] = a.y; b[2] = a.width; b[3] = a.height; b[4] = tu.cbf[c]; b[5] = tu.mtsIdx[c];
      if (q != g_cap.tuqp.end()) { b[7] = q->second[c * 2]; b[8] = q->second[c * 2 + 1]; }
      if (tu.cbf[c] || (c > 0 && tu.jointCbCr)) {
        b[6] = (int32_t)coef.size();
        const CCoeffBuf cb = tu.getCoeffs((ComponentID)c);
        for (int y = 0; y < (int)a.height; y++)
          for (int x = 0; x < (int)a.width; x++) coef.push_back(cb.buf[y * cb.stride + x]);
      }
    }
  }
  TR("tu table");
  F.i32("tu", tut, {cs.tus.size(), (uint64_t)TU_NF});
  F.i32("coef", coef, {coef.size()});

  // ---- GEO candidates: cu, (interDir, ref0, ref1, mv0x, mv0y, mv1x, mv1y) x... flattened 12: per cand (dir, refL, mvx, mvy, ?, ?)
  {
    std::vector<int32_t> g;
    for (auto &kv : g_cap.geo) { g.push_back(cuIdx[kv.first]); for (int k = 0; k < 12; k++) g.push_back(kv.second[k]); }
    F.i32("geo", g, {g.size() / 13, 13});
  }

  TR("geo");
  // ---- motion field (4x4), before DMVR refinement write-back (what deblocking sees)
  {
    const int W4 = pcv.lumaWidth >> 2, H4 = pcv.lumaHeight >> 2;
    const int NF = 10;
    std::vector<int32_t> mf((size_t)W4 * H4 * NF, 0);
    for (int y = 0; y < H4; y++)
      for (int x = 0; x < W4; x++) {
        const MotionInfo &mi = cs.getMotionInfo(Position(x << 2, y << 2));
        int32_t *o = &mf[((size_t)y * W4 + x) * NF];
        o[0] = mi.isInter; o[1] = mi.interDir; o[2] = mi.refIdx[0]; o[3] = mi.refIdx[1];
        o[4] = mi.mv[0].hor; o[5] = mi.mv[0].ver; o[6] = mi.mv[1].hor; o[7] = mi.mv[1].ver; o[8] = mi.BcwIdx; o[9] = mi.useAltHpelIf;
      }
    F.i32("motion", mf, {(uint64_t)H4, (uint64_t)W4, (uint64_t)NF});
  }

  TR("motion");
  // ---- LMCS
  {
    Reshape &r = dec.m_cReshaper;
    std::vector<int16_t> fwd(r.m_fwdLUT.begin(), r.m_fwdLUT.end()), inv(r.m_invLUT.begin(), r.m_invLUT.end());
    std::vector<int16_t> piv(r.m_reshapePivot.begin(), r.m_reshapePivot.end()), ipiv(r.m_inputPivot.begin(), r.m_inputPivot.end());
    std::vector<int32_t> cadj(r.m_chromaAdjHelpLUT.begin(), r.m_chromaAdjHelpLUT.end());
    std::vector<int32_t> fsc(r.m_fwdScaleCoef.begin(), r.m_fwdScaleCoef.end()), isc(r.m_invScaleCoef.begin(), r.m_invScaleCoef.end());
    F.i16("lmcs_fwd", fwd, {fwd.size()});
    F.i16("lmcs_inv", inv, {inv.size()});
    F.i16("lmcs_pivot", piv, {piv.size()});
    F.i16("lmcs_inpivot", ipiv, {ipiv.size()});
    F.i32("lmcs_cadj", cadj, {cadj.size()});
    F.i32("lmcs_fwdscale", fsc, {fsc.size()});
    F.i32("lmcs_invscale", isc, {isc.size()});
  }
}

static void dumpSao(CapFile &F, const CodingStructure &cs) {
  const int n = cs.pcv->sizeInCtus;
  std::vector<int32_t> s((size_t)n * 3 * 35, 0);
  SAOBlkParam *p = cs.picture->getSAO();
  for (int i = 0; i < n; i++)
    for (int c = 0; c < 3; c++) {
      const SAOOffset &o = p[i][c];
      int32_t *d = &s[((size_t)i * 3 + c) * 35];
      d[0] = o.modeIdc; d[1] = o.typeIdc; d[2] = o.typeAuxInfo;
      for (int k = 0; k < 32; k++) d[3 + k] = o.offset[k];
    }
  F.i32("sao", s, {(uint64_t)n, 3, 35});
}

static void dumpAlf(CapFile &F, DecLib &dec, const CodingStructure &cs) {
  AdaptiveLoopFilter &A = dec.m_cALF;
  const int n = cs.pcv->sizeInCtus;
  Picture &pic = *cs.picture;
  std::vector<uint8_t> en(3 * n), alt(3 * n), cc(2 * n, 0);
  for (int c = 0; c < 3; c++)
    for (int i = 0; i < n; i++) {
      const uint8_t *e = pic.getAlfCtuEnableFlag(c), *a = pic.getAlfCtuAlternativeData(c);
      en[c * n + i] = (e && pic.m_alfCtuEnableFlag[c].size() > (size_t)i) ? e[i] : 0;
      alt[c * n + i] = (a && pic.m_alfCtuAlternative[c].size() > (size_t)i) ? a[i] : 0;
    }
  for (int c = 0; c < 2; c++)
    if (A.m_ccAlfFilterControl[c])
      for (int i = 0; i < n; i++) cc[c * n + i] = A.m_ccAlfFilterControl[c][i];
  std::vector<int16_t> fidx(n, 0);
  for (int i = 0; i < n && i < (int)pic.m_alfCtbFilterIndex.size(); i++) fidx[i] = pic.m_alfCtbFilterIndex[i];
  F.u8("alf_ctb_en", en, {3, (uint64_t)n});
  F.u8("alf_ctb_alt", alt, {3, (uint64_t)n});
  F.i16("alf_ctb_fidx", fidx, {(uint64_t)n});
  F.u8("ccalf_ctl", cc, {2, (uint64_t)n});
  const int L = MAX_NUM_ALF_CLASSES * MAX_NUM_ALF_LUMA_COEFF;
  std::vector<int16_t> ca(&A.m_coeffApsLuma[0][0], &A.m_coeffApsLuma[0][0] + ALF_CTB_MAX_NUM_APS * L);
  std::vector<int16_t> cl(&A.m_clippApsLuma[0][0], &A.m_clippApsLuma[0][0] + ALF_CTB_MAX_NUM_APS * L);
  std::vector<int16_t> fx(&A.m_fixedFilterSetCoeffDec[0][0], &A.m_fixedFilterSetCoeffDec[0][0] + NUM_FIXED_FILTER_SETS * L);
  std::vector<int16_t> cdef(A.m_clipDefault, A.m_clipDefault + L);
  F.i16("alf_coef_aps", ca, {(uint64_t)ALF_CTB_MAX_NUM_APS, (uint64_t)MAX_NUM_ALF_CLASSES, (uint64_t)MAX_NUM_ALF_LUMA_COEFF});
  F.i16("alf_clip_aps", cl, {(uint64_t)ALF_CTB_MAX_NUM_APS, (uint64_t)MAX_NUM_ALF_CLASSES, (uint64_t)MAX_NUM_ALF_LUMA_COEFF});
  F.i16("alf_fixed", fx, {(uint64_t)NUM_FIXED_FILTER_SETS, (uint64_t)MAX_NUM_ALF_CLASSES, (uint64_t)MAX_NUM_ALF_LUMA_COEFF});
  F.i16("alf_clip_default", cdef, {(uint64_t)MAX_NUM_ALF_CLASSES, (uint64_t)MAX_NUM_ALF_LUMA_COEFF});
  const int C = MAX_NUM_ALF_ALTERNATIVES_CHROMA * MAX_NUM_ALF_CHROMA_COEFF;
  std::vector<int16_t> cc2(&A.m_chromaCoeffFinal[0][0], &A.m_chromaCoeffFinal[0][0] + C);
  std::vector<int16_t> cl2(&A.m_chromaClippFinal[0][0], &A.m_chromaClippFinal[0][0] + C);
  F.i16("alf_chroma_coef", cc2, {(uint64_t)MAX_NUM_ALF_ALTERNATIVES_CHROMA, (uint64_t)MAX_NUM_ALF_CHROMA_COEFF});
  F.i16("alf_chroma_clip", cl2, {(uint64_t)MAX_NUM_ALF_ALTERNATIVES_CHROMA, (uint64_t)MAX_NUM_ALF_CHROMA_COEFF});
  std::vector<int16_t> cv(&A.m_alfClippingValues[0][0], &A.m_alfClippingValues[0][0] + MAX_NUM_CHANNEL_TYPE * AdaptiveLoopFilter::MaxAlfNumClippingValues);
  F.i16("alf_clip_values", cv, {(uint64_t)MAX_NUM_CHANNEL_TYPE, (uint64_t)AdaptiveLoopFilter::MaxAlfNumClippingValues});
  // APS ids used by the slice for luma (order = filter set index - NUM_FIXED_FILTER_SETS)
  std::vector<int32_t> aps;
  for (int i = 0; i < cs.slice->getTileGroupNumAps(); i++) aps.push_back(cs.slice->getTileGroupApsIdLuma()[i]);
  F.i32("alf_aps_ids", aps, {aps.size()});
  // CC-ALF filters: [comp][filter][coef]
  const CcAlfFilterParam &p = cs.slice->m_ccAlfFilterParam;
  std::vector<int16_t> ccf(2 * MAX_NUM_CC_ALF_FILTERS * MAX_NUM_CC_ALF_CHROMA_COEFF);
  std::vector<int32_t> ccn(2 * (1 + MAX_NUM_CC_ALF_FILTERS));
  for (int c = 0; c < 2; c++) {
    ccn[c * (1 + MAX_NUM_CC_ALF_FILTERS)] = p.ccAlfFilterCount[c];
    for (int f = 0; f < MAX_NUM_CC_ALF_FILTERS; f++) {
      ccn[c * (1 + MAX_NUM_CC_ALF_FILTERS) + 1 + f] = p.ccAlfFilterIdxEnabled[c][f];
      for (int k = 0; k < MAX_NUM_CC_ALF_CHROMA_COEFF; k++) ccf[(c * MAX_NUM_CC_ALF_FILTERS + f) * MAX_NUM_CC_ALF_CHROMA_COEFF + k] = p.ccAlfCoeff[c][f][k];
    }
  }
  F.i16("ccalf_coef", ccf, {2, (uint64_t)MAX_NUM_CC_ALF_FILTERS, (uint64_t)MAX_NUM_CC_ALF_CHROMA_COEFF});
  F.i32("ccalf_info", ccn, {2, (uint64_t)(1 + MAX_NUM_CC_ALF_FILTERS)});
}

// ---------------------------------------------------------------------------------------------
// constant tables of the reference (transform / LFNST / MIP / deblocking / GEO), dumped once from the
// running reference so the kernels' generated tables can be pinned against them (tests/golden/tables.cap)
// ---------------------------------------------------------------------------------------------
static void dumpTables(const char *path) {
  CapFile T;
  T.open(path);
  auto m = [&](const char *n, const TMatrixCoeff *p, int N) { std::vector<int16_t> v(p, p + N * N); T.i16(n, v, {(uint64_t)N, (uint64_t)N}); };
  m("dct2_2", &g_trCoreDCT2P2[0][0][0], 2); m("dct2_4", &g_trCoreDCT2P4[0][0][0], 4); m("dct2_8", &g_trCoreDCT2P8[0][0][0], 8);
  m("dct2_16", &g_trCoreDCT2P16[0][0][0], 16); m("dct2_32", &g_trCoreDCT2P32[0][0][0], 32); m("dct2_64", &g_trCoreDCT2P64[0][0][0], 64);
  m("dst7_4", &g_trCoreDST7P4[0][0][0], 4); m("dst7_8", &g_trCoreDST7P8[0][0][0], 8); m("dst7_16", &g_trCoreDST7P16[0][0][0], 16); m("dst7_32", &g_trCoreDST7P32[0][0][0], 32);
  m("dct8_4", &g_trCoreDCT8P4[0][0][0], 4); m("dct8_8", &g_trCoreDCT8P8[0][0][0], 8); m("dct8_16", &g_trCoreDCT8P16[0][0][0], 16); m("dct8_32", &g_trCoreDCT8P32[0][0][0], 32);
  { std::vector<int16_t> v(&g_lfnst8x8[0][0][0][0], &g_lfnst8x8[0][0][0][0] + 4 * 2 * 16 * 48); T.i16("lfnst8x8", v, {4, 2, 16, 48}); }
  { std::vector<int16_t> v(&g_lfnst4x4[0][0][0][0], &g_lfnst4x4[0][0][0][0] + 4 * 2 * 16 * 16); T.i16("lfnst4x4", v, {4, 2, 16, 16}); }
  { std::vector<int16_t> v(g_lfnstLut, g_lfnstLut + NUM_INTRA_MODE + NUM_EXT_LUMA_MODE - 1); T.i16("lfnst_lut", v, {v.size()}); }
  { std::vector<int16_t> v(&vtm_mip::mipMatrix4x4[0][0][0], &vtm_mip::mipMatrix4x4[0][0][0] + 16 * 16 * 4); T.i16("mip4x4", v, {16, 16, 4}); }
  { std::vector<int16_t> v(&vtm_mip::mipMatrix8x8[0][0][0], &vtm_mip::mipMatrix8x8[0][0][0] + 8 * 16 * 8); T.i16("mip8x8", v, {8, 16, 8}); }
  { std::vector<int16_t> v(&vtm_mip::mipMatrix16x16[0][0][0], &vtm_mip::mipMatrix16x16[0][0][0] + 6 * 64 * 7); T.i16("mip16x16", v, {6, 64, 7}); }
  { std::vector<int16_t> v(LoopFilter::sm_tcTable, LoopFilter::sm_tcTable + MAX_QP + 1 + 2); T.i16("dbk_tc", v, {v.size()}); }
  { std::vector<int16_t> v(LoopFilter::sm_betaTable, LoopFilter::sm_betaTable + MAX_QP + 1); T.i16("dbk_beta", v, {v.size()}); }
  { std::vector<int16_t> v(&g_invQuantScales[0][0], &g_invQuantScales[0][0] + 2 * SCALING_LIST_REM_NUM); T.i16("inv_quant_scales", v, {2, (uint64_t)SCALING_LIST_REM_NUM}); }
  { std::vector<int16_t> v; for (int i = 0; i < GEO_NUM_PARTITION_MODE; i++) { v.push_back(g_GeoParams[i][0]); v.push_back(g_GeoParams[i][1]); } T.i16("geo_params", v, {(uint64_t)GEO_NUM_PARTITION_MODE, 2}); }
  { std::vector<int16_t> v(g_angle2mask, g_angle2mask + GEO_NUM_ANGLES); T.i16("geo_angle2mask", v, {v.size()}); }
  { std::vector<int16_t> v(g_Dis, g_Dis + GEO_NUM_ANGLES); T.i16("geo_dis", v, {v.size()}); }
  { std::vector<int16_t> v(g_angle2mirror, g_angle2mirror + GEO_NUM_ANGLES); T.i16("geo_angle2mirror", v, {v.size()}); }
  { std::vector<int16_t> v(&g_weightOffset[0][0][0][0], &g_weightOffset[0][0][0][0] + GEO_NUM_PARTITION_MODE * GEO_NUM_CU_SIZE * GEO_NUM_CU_SIZE * 2);
    T.i16("geo_weight_offset", v, {(uint64_t)GEO_NUM_PARTITION_MODE, (uint64_t)GEO_NUM_CU_SIZE, (uint64_t)GEO_NUM_CU_SIZE, 2}); }
  { std::vector<int16_t> v; for (int i = 0; i < GEO_NUM_PRESTORED_MASK; i++) v.insert(v.end(), g_globalGeoWeights[i], g_globalGeoWeights[i] + GEO_WEIGHT_MASK_SIZE * GEO_WEIGHT_MASK_SIZE);
    T.i16("geo_weights", v, {(uint64_t)GEO_NUM_PRESTORED_MASK, (uint64_t)GEO_WEIGHT_MASK_SIZE, (uint64_t)GEO_WEIGHT_MASK_SIZE}); }
  // CABAC context sets (Contexts.cpp:188-908): offset/size of every set and the four init tables
  // (B, P, I init values and the log2 window sizes, ContextSetCfg::getInitTable 0..3)
#define VVCR_CS(n) { const CtxSet &s = ContextSetCfg::n; std::vector<int32_t> v{(int32_t)s.Offset, (int32_t)s.Size}; T.i32("ctx_" #n, v, {2}); }
#define VVCR_CSA(n, k) { const CtxSet &s = ContextSetCfg::n[k]; std::vector<int32_t> v{(int32_t)s.Offset, (int32_t)s.Size}; T.i32("ctx_" #n #k, v, {2}); }
  VVCR_CS(SplitFlag) VVCR_CS(SplitQtFlag) VVCR_CS(SplitHvFlag) VVCR_CS(Split12Flag) VVCR_CS(ModeConsFlag) VVCR_CS(SkipFlag)
  VVCR_CS(MergeFlag) VVCR_CS(RegularMergeFlag) VVCR_CS(MergeIdx) VVCR_CS(PredMode) VVCR_CS(MultiRefLineIdx)
  VVCR_CS(IntraLumaMpmFlag) VVCR_CS(IntraLumaPlanarFlag) VVCR_CS(CclmModeFlag) VVCR_CS(CclmModeIdx) VVCR_CS(IntraChromaPredMode)
  VVCR_CS(MipFlag) VVCR_CS(DeltaQP) VVCR_CS(InterDir) VVCR_CS(RefPic) VVCR_CS(MmvdFlag) VVCR_CS(MmvdMergeIdx) VVCR_CS(MmvdStepMvpIdx)
  VVCR_CS(SubblockMergeFlag) VVCR_CS(AffineFlag) VVCR_CS(AffineType) VVCR_CS(AffMergeIdx) VVCR_CS(Mvd) VVCR_CS(BDPCMMode)
  VVCR_CS(QtRootCbf) VVCR_CS(ACTFlag) VVCR_CSA(QtCbf, 0) VVCR_CSA(QtCbf, 1) VVCR_CSA(QtCbf, 2)
  VVCR_CSA(SigCoeffGroup, 0) VVCR_CSA(SigCoeffGroup, 1) VVCR_CSA(LastX, 0) VVCR_CSA(LastX, 1) VVCR_CSA(LastY, 0) VVCR_CSA(LastY, 1)
  VVCR_CSA(SigFlag, 0) VVCR_CSA(SigFlag, 1) VVCR_CSA(SigFlag, 2) VVCR_CSA(SigFlag, 3) VVCR_CSA(SigFlag, 4) VVCR_CSA(SigFlag, 5)
  VVCR_CSA(ParFlag, 0) VVCR_CSA(ParFlag, 1) VVCR_CSA(GtxFlag, 0) VVCR_CSA(GtxFlag, 1) VVCR_CSA(GtxFlag, 2) VVCR_CSA(GtxFlag, 3)
  VVCR_CS(TsSigCoeffGroup) VVCR_CS(TsSigFlag) VVCR_CS(TsParFlag) VVCR_CS(TsGtxFlag) VVCR_CS(TsLrg1Flag) VVCR_CS(TsResidualSign)
  VVCR_CS(MVPIdx) VVCR_CS(SaoMergeFlag) VVCR_CS(SaoTypeIdx) VVCR_CS(TransformSkipFlag) VVCR_CS(MTSIdx) VVCR_CS(LFNSTIdx)
  VVCR_CS(PLTFlag) VVCR_CS(RdpcmFlag) VVCR_CS(RdpcmDir) VVCR_CS(SbtFlag) VVCR_CS(SbtQuadFlag) VVCR_CS(SbtHorFlag) VVCR_CS(SbtPosFlag)
  VVCR_CS(CrossCompPred) VVCR_CS(ChromaQpAdjFlag) VVCR_CS(ChromaQpAdjIdc) VVCR_CS(ImvFlag) VVCR_CS(BcwIdx) VVCR_CS(ctbAlfFlag)
  VVCR_CS(ctbAlfAlternative) VVCR_CS(AlfUseTemporalFilt) VVCR_CS(CcAlfFilterControlFlag) VVCR_CS(CiipFlag) VVCR_CS(SmvdFlag)
  VVCR_CS(IBCFlag) VVCR_CS(ISPMode) VVCR_CS(JointCbCrFlag)
#undef VVCR_CS
#undef VVCR_CSA
  for (int k = 0; k < 4; k++) {
    const std::vector<uint8_t> &t = ContextSetCfg::getInitTable(k);
    char nm[24]; snprintf(nm, sizeof nm, "ctx_init%d", k);
    T.u8(nm, t, {t.size()});
  }
  T.close();
}

static DecLib *g_dec = nullptr;
static CapFile g_file;

#ifdef VVCR_DROPIN
// ---------------------------------------------------------------------------------------------
// drop-in: the picture through libvvcr (include/vvcr.h), its result back into the reference's buffers
// ---------------------------------------------------------------------------------------------
#include "vvcr.h"
static std::map<std::string, Chunk> g_mem;
static vvcr_ctx *g_vvcr = nullptr;
static const int kSlots = 24;
static std::map<int, int> g_slotOfPoc;   // POC -> DPB slot of libvvcr (slot = decode index mod kSlots)

template <class T> static const T *chunk(const char *name, size_t *n = nullptr) {
  auto it = g_mem.find(name);
  if (it == g_mem.end()) { if (n) *n = 0; return nullptr; }
  if (n) *n = it->second.bytes.size() / sizeof(T);
  return (const T *)it->second.bytes.data();
}
static int64_t hdr(const char *key) {
  size_t nk = 0, nv = 0;
  const char *k = chunk<char>("hdr_keys", &nk);
  const int64_t *v = chunk<int64_t>("hdr_vals", &nv);
  std::string keys(k, nk), want(key);
  size_t i = 0, pos = 0;
  while (pos <= keys.size()) {
    size_t e = keys.find(',', pos);
    if (e == std::string::npos) e = keys.size();
    if (keys.compare(pos, e - pos, want) == 0 && e - pos == want.size()) return v[i];
    pos = e + 1;
    i++;
  }
  fprintf(stderr, "vtm_vvcr: header field %s missing\n", key);
  exit(4);
}
static void vcheck(int rc, const char *what) {
  if (rc < 0) { fprintf(stderr, "vtm_vvcr: %s: %s\n", what, vvcr_last_error(g_vvcr)); exit(5); }
}

// vvcr_pic_params from the descriptors (the C++ form of vvc_amd/stream.py pic_params)
static void picParams(vvcr_pic_params &pp, int slot) {
  std::memset(&pp, 0, sizeof pp);
  pp.poc = (int32_t)hdr("poc"); pp.slot = slot; pp.slice_type = (int32_t)hdr("slice_type"); pp.slice_qp = (int32_t)hdr("slice_qp");
  const int32_t *rp = chunk<int32_t>("ref_poc"), *rl = chunk<int32_t>("ref_lt");
  for (int l = 0; l < 2; l++) {
    pp.num_ref[l] = (int32_t)hdr(l ? "num_ref_l1" : "num_ref_l0");
    for (int r = 0; r < pp.num_ref[l]; r++) {
      const int poc = rp[l * MAX_NUM_REF + r];
      auto it = g_slotOfPoc.find(poc);
      if (it == g_slotOfPoc.end()) { fprintf(stderr, "vtm_vvcr: POC %d: reference POC %d not in libvvcr's DPB\n", pp.poc, poc); exit(6); }
      pp.ref_poc[l][r] = poc; pp.ref_slot[l][r] = it->second; pp.ref_lt[l][r] = rl[l * MAX_NUM_REF + r];
    }
  }
#define F(k) pp.k = (int32_t)hdr(#k)
  F(dual_tree); F(dep_quant); F(sign_hiding); F(joint_cbcr); F(bdof_enabled); F(dmvr_enabled); F(prof_enabled);
  F(lfnst_enabled); F(mts_intra); F(mts_inter); F(sbt); F(wp_p); F(wp_b); F(dbk_disable); F(dbk_beta_offset_div2);
  F(dbk_tc_offset_div2); F(lf_across_slices); F(lf_across_tiles); F(sao_luma); F(sao_chroma); F(alf_vb_luma);
  F(alf_vb_chroma); F(lmcs_chroma_scale); F(lmcs_min_bin); F(lmcs_max_bin); F(log2_max_ts); F(use_mts);
  F(implicit_mts); F(joint_cbcr_sign); F(entropy_sync); F(vb_disabled); F(num_vb_ver); F(num_vb_hor);
#undef F
  for (int i = 0; i < 3; i++) {
    pp.vb_ver[i] = (int32_t)hdr((std::string("vb_ver") + char('0' + i)).c_str());
    pp.vb_hor[i] = (int32_t)hdr((std::string("vb_hor") + char('0' + i)).c_str());
  }
  if (!pp.num_vb_ver && !pp.num_vb_hor) pp.vb_disabled = 0;
  pp.ladf_num = (int32_t)hdr("ladf_num");
  for (int k = 0; k < 5; k++) {
    pp.ladf_qp_offset[k] = (int32_t)hdr((std::string("ladf_qp_offset") + char('0' + k)).c_str());
    pp.ladf_lower_bound[k] = (int32_t)hdr((std::string("ladf_lower_bound") + char('0' + k)).c_str());
  }
  pp.lmcs_enabled = hdr("lmcs_enabled") && hdr("lmcs_slice_flag");
  int tb = 0;
  while ((1 << (tb + 1)) <= hdr("max_tb_size")) tb++;
  pp.max_tb_log2 = tb;
  pp.chroma_qp_off[0] = (int32_t)hdr("chroma_qp_off_jc");
  pp.chroma_qp_off[1] = (int32_t)hdr("chroma_qp_off_cb");
  pp.chroma_qp_off[2] = (int32_t)hdr("chroma_qp_off_cr");
  std::memcpy(pp.wp, chunk<int32_t>("wp"), sizeof pp.wp);
  std::memcpy(pp.chroma_qp_map, chunk<int32_t>("chroma_qp_map"), sizeof pp.chroma_qp_map);
  std::memcpy(pp.chroma_qp_map[0], chunk<int32_t>("chroma_qp_map_jc"), sizeof pp.chroma_qp_map[0]);   // row 0: joint Cb-Cr
  for (int c = 0; c < 3; c++) pp.alf_en[c] = (int32_t)hdr(c == 0 ? "alf_slice_en0" : c == 1 ? "alf_slice_en1" : "alf_slice_en2");
  pp.ccalf_en[0] = (int32_t)hdr("ccalf_en_cb"); pp.ccalf_en[1] = (int32_t)hdr("ccalf_en_cr");
  size_t n;
  const int16_t *t = chunk<int16_t>("lmcs_fwd", &n);
  std::memcpy(pp.lmcs_fwd, t, std::min<size_t>(n, 1024) * 2);
  t = chunk<int16_t>("lmcs_inv", &n);
  std::memcpy(pp.lmcs_inv, t, std::min<size_t>(n, 1024) * 2);
  t = chunk<int16_t>("lmcs_pivot", &n);
  std::memcpy(pp.lmcs_pivot, t, std::min<size_t>(n, 17) * 2);
  const int32_t *ca = chunk<int32_t>("lmcs_cadj", &n);
  std::memcpy(pp.lmcs_cadj, ca, std::min<size_t>(n, 16) * 4);
  size_t nc, nr;
  const int32_t *cb = chunk<int32_t>("tile_col_bd", &nc), *rb = chunk<int32_t>("tile_row_bd", &nr);
  pp.num_tile_cols = (int32_t)nc - 1; pp.num_tile_rows = (int32_t)nr - 1;
  std::memcpy(pp.tile_col_bd, cb, nc * 4);
  std::memcpy(pp.tile_row_bd, rb, nr * 4);
}

static void dropinPicture(CodingStructure &cs) {
  const int W = (int)hdr("width"), H = (int)hdr("height");
  if (!g_vvcr) {
    vvcr_seq_params sp{W, H, 1, (int32_t)hdr("bitdepth_y"), (int32_t)hdr("ctu_log2"), kSlots, 0};
    if (vvcr_create(&sp, &g_vvcr) < 0) { fprintf(stderr, "vtm_vvcr: vvcr_create failed\n"); exit(5); }
  }
  const int slot = g_picCounter % kSlots, poc = (int)hdr("poc");
  for (auto it = g_slotOfPoc.begin(); it != g_slotOfPoc.end();)
    it = it->second == slot ? g_slotOfPoc.erase(it) : std::next(it);
  vvcr_pic_params pp;
  picParams(pp, slot);
  vcheck(vvcr_begin_picture(g_vvcr, &pp), "vvcr_begin_picture");
  size_t ncu, npu, ntu, ncoef, nmo, ngeo;
  const vvcr_cu *cu = chunk<vvcr_cu>("cu", &ncu);
  const vvcr_pu *pu = chunk<vvcr_pu>("pu", &npu);
  const vvcr_tu *tu = chunk<vvcr_tu>("tu", &ntu);
  const int32_t *coef = chunk<int32_t>("coef", &ncoef);
  const vvcr_motion *mo = chunk<vvcr_motion>("motion", &nmo);
  const vvcr_geo *geo = chunk<vvcr_geo>("geo", &ngeo);
  vcheck(vvcr_submit(g_vvcr, cu, (int32_t)ncu, pu, (int32_t)npu, tu, (int32_t)ntu, coef, (int64_t)ncoef, mo, geo, (int32_t)ngeo),
         "vvcr_submit");
  // SAO / ALF parameters (vvc_amd/stream.py set_loop_filter_params)
  const vvcr_sao *sao = chunk<vvcr_sao>("sao");
  vvcr_alf alf{}, *palf = nullptr;
  std::vector<int16_t> coefL, clipL;
  std::vector<uint8_t> ccCtl, alt;
  if (hdr("alf_enabled") && g_mem.count("alf_ctb_en")) {
    size_t naps, nfx, nca, nctb;
    chunk<int32_t>("alf_aps_ids", &naps);
    const int16_t *fx = chunk<int16_t>("alf_fixed", &nfx), *ca2 = chunk<int16_t>("alf_coef_aps", &nca);
    const int16_t *cl = chunk<int16_t>("alf_clip_aps"), *cdef = chunk<int16_t>("alf_clip_default");
    const int L = MAX_NUM_ALF_CLASSES * MAX_NUM_ALF_LUMA_COEFF;
    coefL.assign(fx, fx + nfx);
    coefL.insert(coefL.end(), ca2, ca2 + naps * L);
    for (size_t k = 0; k < nfx / L; k++) clipL.insert(clipL.end(), cdef, cdef + L);
    clipL.insert(clipL.end(), cl, cl + naps * L);
    const uint8_t *cc = chunk<uint8_t>("ccalf_ctl", &nctb);
    nctb /= 2;
    ccCtl.assign(cc, cc + 2 * nctb);
    for (size_t i = 0; i < nctb; i++) {
      if (!hdr("ccalf_en_cb")) ccCtl[i] = 0;   // control words of a disabled component are not coded
      if (!hdr("ccalf_en_cr")) ccCtl[nctb + i] = 0;
    }
    const uint8_t *a = chunk<uint8_t>("alf_ctb_alt");
    alt.assign(a, a + 3 * nctb);
    std::fill(alt.begin(), alt.begin() + nctb, 0);
    alf.num_luma_sets = (int32_t)(nfx / L + naps);
    alf.luma_coef = coefL.data(); alf.luma_clip = clipL.data();
    alf.chroma_coef = chunk<int16_t>("alf_chroma_coef"); alf.chroma_clip = chunk<int16_t>("alf_chroma_clip");
    alf.cc_coef = chunk<int16_t>("ccalf_coef"); alf.ctb_en = chunk<uint8_t>("alf_ctb_en"); alf.ctb_alt = alt.data();
    alf.ctb_filter_set = chunk<int16_t>("alf_ctb_fidx"); alf.cc_ctl = ccCtl.data();
    palf = &alf;
  }
  vcheck(vvcr_set_loop_filter_params(g_vvcr, sao, palf), "vvcr_set_loop_filter_params");
  vcheck(vvcr_end_picture(g_vvcr), "vvcr_end_picture");
  g_slotOfPoc[poc] = slot;
  // the decoded picture: libvvcr's replaces the reference's (DecApp writes and later pictures read it)
  PelUnitBuf reco = cs.picture->getRecoBuf();
  std::vector<uint16_t> planes[3];
  uint16_t *ptr[3];
  int32_t stride[3];
  for (int c = 0; c < 3; c++) {
    planes[c].resize((size_t)reco.bufs[c].width * reco.bufs[c].height);
    ptr[c] = planes[c].data();
    stride[c] = (int32_t)reco.bufs[c].width;
  }
  vcheck(vvcr_read_picture(g_vvcr, slot, ptr, stride), "vvcr_read_picture");
  // the reference never reconstructed this picture: its buffer holds libvvcr's samples only (DecLib's MD5
  // check of the decoded-picture-hash SEI and DecApp's output read them)
  for (int c = 0; c < 3; c++) {
    PelBuf &b = reco.bufs[c];
    for (int y = 0; y < (int)b.height; y++) {
      Pel *row = b.buf + (size_t)y * b.stride;
      const uint16_t *src = planes[c].data() + (size_t)y * b.width;
      for (int x = 0; x < (int)b.width; x++) row[x] = (Pel)src[x];
    }
  }
  // DMVR: libvvcr's refinements replace the reference's before CS::setRefinedMotionField
  size_t nd;
  chunk<int32_t>("dmvr_delta", &nd);
  if (nd) {
    std::vector<int32_t> d(nd);
    const int got = vvcr_get_dmvr_deltas(g_vvcr, d.data(), (int64_t)nd / 2);
    vcheck(got, "vvcr_get_dmvr_deltas");
    enum { PU_DMVR_OFF = 45, PU_DMVR = 47 };
    const int32_t *prow = chunk<int32_t>("pu");
    for (size_t i = 0; i < cs.pus.size(); i++) {
      const int32_t *o = prow + i * 48;
      if (!o[PU_DMVR]) continue;
      PredictionUnit &u = *cs.pus[i];
      const int dy = std::min<int>(u.lumaSize().height, DMVR_SUBCU_HEIGHT), dx = std::min<int>(u.lumaSize().width, DMVR_SUBCU_WIDTH);
      const int n = (u.lumaSize().height / dy) * (u.lumaSize().width / dx);
      for (int k = 0; k < n; k++) {
        const int64_t j = (int64_t)o[PU_DMVR_OFF] + k;
        if (j >= got) { fprintf(stderr, "vtm_vvcr: DMVR deltas short\n"); exit(7); }
        u.mvdL0SubPu[k].hor = d[2 * j];
        u.mvdL0SubPu[k].ver = d[2 * j + 1];
      }
    }
  }
}
#endif

static void planeOut(const char *pfx, Plane *p) {
  for (int c = 0; c < 3; c++) {
    char nm[32];
    snprintf(nm, sizeof nm, "%s_%c", pfx, "yuv"[c]);
    g_file.i16(nm, p[c].d, {(uint64_t)p[c].h, (uint64_t)p[c].w});
  }
}

static void finishCapture() {
  if (!g_cap.active) return;
  for (int s = 0; s < ST_N; s++) if (g_cap.haveStage[s]) planeOut(kStageName[s], g_cap.stage[s]);
  planeOut("pmc", g_cap.pmc);
  planeOut("pfin", g_cap.pfin);
  planeOut("resi", g_cap.resi);
  g_file.close();
  g_cap.active = false;
  g_picCounter++;
}

// ---------------------------------------------------------------------------------------------
// link-time wrappers (see wraps.txt)
// ---------------------------------------------------------------------------------------------
extern "C" {

// DecLib::executeLoopFilters()
void __real__ZN6DecLib18executeLoopFiltersEv(DecLib *self);
void __wrap__ZN6DecLib18executeLoopFiltersEv(DecLib *self) {
  g_dec = self;
  static bool tablesDumped = false;
  if (!tablesDumped && getenv("VVCR_DUMP_TABLES")) { dumpTables(getenv("VVCR_DUMP_TABLES")); tablesDumped = true; }
  if (!self->m_pcPic || g_dir.empty()) { __real__ZN6DecLib18executeLoopFiltersEv(self); return; }
  CodingStructure &cs = *self->m_pcPic->cs;
#ifdef VVCR_DROPIN
  // DecLib::executeLoopFilters (DecLib.cpp:560-623) REPLACED: the reference's deblocking, SAO and ALF do
  // not run. What the decoder state needs from it is kept: the reshaper's flag (:570-576), the SAO
  // parameters with merges resolved (SAOProcess's first step, SampleAdaptiveOffset.cpp:623) and the ALF
  // filters of the slice's APSs (ALFProcess's reconstructCoeffAPSs, AdaptiveLoopFilter.cpp:439) as
  // libvvcr's parameters, and CS::setRefinedMotionField (:579) with libvvcr's DMVR refinements.
  g_mem.clear();
  g_file.mem = &g_mem;
  if (!g_cap.active) initPlanes(cs);   // an intra picture without inter CUs
  dumpDescriptors(g_file, *self, cs);
  if (cs.sps->getUseLmcs() && self->m_cReshaper.getSliceReshaperInfo().getUseSliceReshaper()) self->m_cReshaper.setRecReshaped(false);
  if (cs.sps->getSAOEnabledFlag()) {
    self->m_cSAO.xReconstructBlkSAOParams(cs, cs.picture->getSAO());
    dumpSao(g_file, cs);
  }
  if (cs.sps->getALFEnabledFlag()) {
    Slice &sl = *cs.slice;
    if (sl.getTileGroupAlfEnabledFlag(COMPONENT_Y) || sl.getTileGroupAlfEnabledFlag(COMPONENT_Cb) || sl.getTileGroupAlfEnabledFlag(COMPONENT_Cr))
      self->m_cALF.reconstructCoeffAPSs(cs, true, sl.getTileGroupAlfEnabledFlag(COMPONENT_Cb) || sl.getTileGroupAlfEnabledFlag(COMPONENT_Cr), false);
    dumpAlf(g_file, *self, cs);
  }
  dropinPicture(cs);
  CS::setRefinedMotionField(cs);
  g_cap.active = false;
  g_picCounter++;
#else
  char path[512];
  snprintf(path, sizeof path, "%s/pic_%03d.cap", g_dir.c_str(), g_picCounter);
  g_file.open(path);
  snapStage(ST_PRELF);
  dumpDescriptors(g_file, *self, cs);
  __real__ZN6DecLib18executeLoopFiltersEv(self);
  if (!g_cap.haveStage[ST_SAO]) { g_cap.stage[ST_SAO][0] = g_cap.stage[ST_DBK][0]; g_cap.stage[ST_SAO][1] = g_cap.stage[ST_DBK][1]; g_cap.stage[ST_SAO][2] = g_cap.stage[ST_DBK][2]; g_cap.haveStage[ST_SAO] = true; }
  TR("real LF done");
  snapStage(ST_ALF);
  if (cs.sps->getALFEnabledFlag()) dumpAlf(g_file, *self, cs);
  TR("alf dumped");
  finishCapture();
#endif
}

// LoopFilter::loopFilterPic(CodingStructure&)
void __real__ZN10LoopFilter13loopFilterPicER15CodingStructure(LoopFilter *self, CodingStructure &cs);
void __wrap__ZN10LoopFilter13loopFilterPicER15CodingStructure(LoopFilter *self, CodingStructure &cs) {
  snapStage(ST_DBKIN);
  g_refCalls[RC_DBK]++;
  __real__ZN10LoopFilter13loopFilterPicER15CodingStructure(self, cs);
  snapStage(ST_DBK);
}

// SampleAdaptiveOffset::SAOProcess(CodingStructure&, SAOBlkParam*)
void __real__ZN20SampleAdaptiveOffset10SAOProcessER15CodingStructureP11SAOBlkParam(SampleAdaptiveOffset *self, CodingStructure &cs, SAOBlkParam *p);
void __wrap__ZN20SampleAdaptiveOffset10SAOProcessER15CodingStructureP11SAOBlkParam(SampleAdaptiveOffset *self, CodingStructure &cs, SAOBlkParam *p) {
  g_refCalls[RC_SAO]++;
  __real__ZN20SampleAdaptiveOffset10SAOProcessER15CodingStructureP11SAOBlkParam(self, cs, p);
  snapStage(ST_SAO);
  if (g_cap.active) dumpSao(g_file, cs);   // parameters are merge-resolved in place by SAOProcess
}

// InterPrediction::motionCompensation(CodingUnit&, RefPicList const&, bool, bool)
void __real__ZN15InterPrediction18motionCompensationER10CodingUnitRK10RefPicListbb(InterPrediction *self, CodingUnit &cu, const RefPicList &l, bool luma, bool chroma);
void __wrap__ZN15InterPrediction18motionCompensationER10CodingUnitRK10RefPicListbb(InterPrediction *self, CodingUnit &cu, const RefPicList &l, bool luma, bool chroma) {
  if (g_replace) { if (!g_cap.active) initPlanes(*cu.cs); return; }   // libvvcr predicts (k_mc, DMVR / BDOF, affine)
  g_refCalls[RC_MC]++;
  __real__ZN15InterPrediction18motionCompensationER10CodingUnitRK10RefPicListbb(self, cu, l, luma, chroma);
  if (!g_cap.active || g_cap.cs != cu.cs) { if (!g_cap.active) initPlanes(*cu.cs); }
  setCtu(*cu.cs, cu.lumaPos().x, cu.lumaPos().y);
  PelUnitBuf pb = cu.cs->getPredBuf(cu);
  for (int c = 0; c < 3; c++) {
    if ((c == 0 && !luma) || (c > 0 && !chroma) || !cu.blocks[c].valid()) continue;
    copyBlock(g_cap.pmc[c], pb.bufs[c], cu.blocks[c].x, cu.blocks[c].y);
    copyBlock(g_cap.pfin[c], pb.bufs[c], cu.blocks[c].x, cu.blocks[c].y);
  }
}

// InterPrediction::motionCompensationGeo(CodingUnit&, MergeCtx&)
void __real__ZN15InterPrediction21motionCompensationGeoER10CodingUnitR8MergeCtx(InterPrediction *self, CodingUnit &cu, MergeCtx &m);
void __wrap__ZN15InterPrediction21motionCompensationGeoER10CodingUnitR8MergeCtx(InterPrediction *self, CodingUnit &cu, MergeCtx &m) {
  if (!g_cap.active) initPlanes(*cu.cs);
  std::array<int32_t, 12> g{};
  int idx[2] = {cu.firstPU->geoMergeIdx0, cu.firstPU->geoMergeIdx1};
  for (int k = 0; k < 2; k++) {
    int i = idx[k];
    int32_t *o = &g[k * 6];
    o[0] = m.interDirNeighbours[i];
    const MvField &f0 = m.mvFieldNeighbours[2 * i], &f1 = m.mvFieldNeighbours[2 * i + 1];
    // GEO candidates are uni-predicted: store the used list's ref and MV
    const MvField &f = (o[0] == 2) ? f1 : f0;
    o[1] = (o[0] == 2) ? 1 : 0; o[2] = f.refIdx; o[3] = f.mv.hor; o[4] = f.mv.ver; o[5] = m.useAltHpelIf[i];
  }
  g_cap.geo[&cu] = g;   // the candidates are descriptor rows (vvcr_geo); the blend is libvvcr's in the drop-in
  if (g_replace) {
    // the PU state motionCompensationGeo leaves behind (InterPrediction.cpp:1761-1770): each candidate's
    // merge info set and spanned in turn, the second one last; the two MCs and the blend do not run
    for (auto &pu : CU::traversePUs(cu)) {
      m.setMergeInfo(pu, idx[0]);
      PU::spanMotionInfo(pu);
      m.setMergeInfo(pu, idx[1]);
      PU::spanMotionInfo(pu);
    }
    return;
  }
  g_refCalls[RC_MC_GEO]++;
  __real__ZN15InterPrediction21motionCompensationGeoER10CodingUnitR8MergeCtx(self, cu, m);
  setCtu(*cu.cs, cu.lumaPos().x, cu.lumaPos().y);
  PelUnitBuf pb = cu.cs->getPredBuf(cu);
  for (int c = 0; c < 3; c++) {
    if (!cu.blocks[c].valid()) continue;
    copyBlock(g_cap.pmc[c], pb.bufs[c], cu.blocks[c].x, cu.blocks[c].y);
    copyBlock(g_cap.pfin[c], pb.bufs[c], cu.blocks[c].x, cu.blocks[c].y);
  }
}

// IntraPrediction::geneWeightedPred(ComponentID, PelBuf&, PU const&, Pel*)   (CIIP blend -> final pred)
void __real__ZN15IntraPrediction16geneWeightedPredE11ComponentIDR7AreaBufIsERK14PredictionUnitPs(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu, Pel *src);
void __wrap__ZN15IntraPrediction16geneWeightedPredE11ComponentIDR7AreaBufIsERK14PredictionUnitPs(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu, Pel *src) {
  if (g_replace) return;
  g_refCalls[RC_INTRA]++;
  __real__ZN15IntraPrediction16geneWeightedPredE11ComponentIDR7AreaBufIsERK14PredictionUnitPs(self, c, pred, pu, src);
  if (!g_cap.active) return;
  setCtu(*pu.cs, pu.lumaPos().x, pu.lumaPos().y);
  int x, y;
  if (locate(*pu.cs, PIC_PREDICTION, c, pred.buf, x, y)) copyBlock(g_cap.pfin[c], pred, x, y);
}

static void recordIntra(const PredictionUnit &pu, ComponentID c, const PelBuf &pred) {
  if (!g_cap.active) initPlanes(*pu.cs);
  { const CompArea &a = pu.blocks[pu.chType]; setCtu(*pu.cs, a.x << (pu.chType ? 1 : 0), a.y << (pu.chType ? 1 : 0)); }
  int x, y;
  if (locate(*pu.cs, PIC_PREDICTION, c, pred.buf, x, y)) copyBlock(g_cap.pfin[c], pred, x, y);
}

// IntraPrediction::predIntraAng(ComponentID, PelBuf&, PU const&)
void __real__ZN15IntraPrediction12predIntraAngE11ComponentIDR7AreaBufIsERK14PredictionUnit(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu);
void __wrap__ZN15IntraPrediction12predIntraAngE11ComponentIDR7AreaBufIsERK14PredictionUnit(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu) {
  if (g_replace) { if (!g_cap.active) initPlanes(*pu.cs); return; }
  g_refCalls[RC_INTRA]++;
  __real__ZN15IntraPrediction12predIntraAngE11ComponentIDR7AreaBufIsERK14PredictionUnit(self, c, pred, pu);
  recordIntra(pu, c, pred);
}
// IntraPrediction::predIntraMip(ComponentID, PelBuf&, PU const&)
void __real__ZN15IntraPrediction12predIntraMipE11ComponentIDR7AreaBufIsERK14PredictionUnit(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu);
void __wrap__ZN15IntraPrediction12predIntraMipE11ComponentIDR7AreaBufIsERK14PredictionUnit(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu) {
  if (g_replace) { if (!g_cap.active) initPlanes(*pu.cs); return; }
  g_refCalls[RC_INTRA]++;
  __real__ZN15IntraPrediction12predIntraMipE11ComponentIDR7AreaBufIsERK14PredictionUnit(self, c, pred, pu);
  recordIntra(pu, c, pred);
}
// IntraPrediction::predIntraChromaLM(ComponentID, PelBuf&, PU const&, CompArea const&, int)
void __real__ZN15IntraPrediction17predIntraChromaLME11ComponentIDR7AreaBufIsERK14PredictionUnitRK8CompAreai(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu, const CompArea &a, int mode);
void __wrap__ZN15IntraPrediction17predIntraChromaLME11ComponentIDR7AreaBufIsERK14PredictionUnitRK8CompAreai(IntraPrediction *self, ComponentID c, PelBuf &pred, const PredictionUnit &pu, const CompArea &a, int mode) {
  if (g_replace) { if (!g_cap.active) initPlanes(*pu.cs); return; }
  g_refCalls[RC_INTRA]++;
  __real__ZN15IntraPrediction17predIntraChromaLME11ComponentIDR7AreaBufIsERK14PredictionUnitRK8CompAreai(self, c, pred, pu, a, mode);
  recordIntra(pu, c, pred);
}

// TrQuant::invTransformNxN(TransformUnit&, ComponentID const&, PelBuf&, QpParam const&)
void __real__ZN7TrQuant15invTransformNxNER13TransformUnitRK11ComponentIDR7AreaBufIsERK7QpParam(TrQuant *self, TransformUnit &tu, const ComponentID &c, PelBuf &resi, const QpParam &q);
void __wrap__ZN7TrQuant15invTransformNxNER13TransformUnitRK11ComponentIDR7AreaBufIsERK7QpParam(TrQuant *self, TransformUnit &tu, const ComponentID &c, PelBuf &resi, const QpParam &q) {
  if (!g_replace) {
    g_refCalls[RC_ITX]++;
    __real__ZN7TrQuant15invTransformNxNER13TransformUnitRK11ComponentIDR7AreaBufIsERK7QpParam(self, tu, c, resi, q);
  }
  if (!g_cap.active) initPlanes(*tu.cs);
  { const CompArea &a = tu.blocks[c]; setCtu(*tu.cs, a.x << (c ? 1 : 0), a.y << (c ? 1 : 0)); }
  auto &e = g_cap.tuqp[&tu];   // the block's QPs (QpParam, Quant.h:68) are descriptor fields
  e[c * 2] = q.Qps[0]; e[c * 2 + 1] = q.Qps[1];
  if (g_replace) return;
  int x, y;
  if (locate(*tu.cs, PIC_RESIDUAL, c, resi.buf, x, y)) copyBlock(g_cap.resi[c], resi, x, y);
}

// TrQuant::invTransformICT(TransformUnit const&, PelBuf&, PelBuf&)
void __real__ZN7TrQuant15invTransformICTERK13TransformUnitR7AreaBufIsES5_(TrQuant *self, const TransformUnit &tu, PelBuf &cb, PelBuf &cr);
void __wrap__ZN7TrQuant15invTransformICTERK13TransformUnitR7AreaBufIsES5_(TrQuant *self, const TransformUnit &tu, PelBuf &cb, PelBuf &cr) {
  if (g_replace) return;
  __real__ZN7TrQuant15invTransformICTERK13TransformUnitR7AreaBufIsES5_(self, tu, cb, cr);
  if (!g_cap.active) return;
  { const CompArea &a = tu.blocks[1]; setCtu(*tu.cs, a.x << 1, a.y << 1); }
  int x, y;
  if (locate(*tu.cs, PIC_RESIDUAL, 1, cb.buf, x, y)) copyBlock(g_cap.resi[1], cb, x, y);
  if (locate(*tu.cs, PIC_RESIDUAL, 2, cr.buf, x, y)) copyBlock(g_cap.resi[2], cr, x, y);
}

// AreaBuf<Pel>::scaleSignal(int, bool, ClpRng const&)  (LMCS chroma residual scaling -> final residual)
void __real__ZN7AreaBufIsE11scaleSignalEibRK6ClpRng(PelBuf *self, int scale, bool dir, const ClpRng &r);
void __wrap__ZN7AreaBufIsE11scaleSignalEibRK6ClpRng(PelBuf *self, int scale, bool dir, const ClpRng &r) {
  if (g_replace) return;
  __real__ZN7AreaBufIsE11scaleSignalEibRK6ClpRng(self, scale, dir, r);
  if (!g_cap.active) return;
  for (int c = 1; c < 3; c++) {
    int x, y;
    if (locate(*g_cap.cs, PIC_RESIDUAL, c, self->buf, x, y)) { copyBlock(g_cap.resi[c], *self, x, y); return; }
  }
}

// AreaBuf<Pel>::rspSignal(std::vector<Pel>&)  (LMCS forward map of an inter prediction -> final prediction)
void __real__ZN7AreaBufIsE9rspSignalERSt6vectorIsSaIsEE(PelBuf *self, std::vector<Pel> &lut);
void __wrap__ZN7AreaBufIsE9rspSignalERSt6vectorIsSaIsEE(PelBuf *self, std::vector<Pel> &lut) {
  if (g_replace) return;
  __real__ZN7AreaBufIsE9rspSignalERSt6vectorIsSaIsEE(self, lut);
  if (!g_cap.active) return;
  int x, y;
  if (locate(*g_cap.cs, PIC_PREDICTION, 0, self->buf, x, y)) copyBlock(g_cap.pfin[0], *self, x, y);
}

// InterpolationFilter::filterHor (InterpolationFilter.cpp:743): counted only, to show that nothing of the
// reference's motion compensation runs in the drop-in
void __real__ZN19InterpolationFilter9filterHorE11ComponentIDPKsiPsiiiib12ChromaFormatRK6ClpRngibb(InterpolationFilter *self, ComponentID c, const Pel *src, int ss, Pel *dst, int ds, int w, int h, int frac, bool last, ChromaFormat f, const ClpRng &r, int idx, bool dmvr, bool alt);
void __wrap__ZN19InterpolationFilter9filterHorE11ComponentIDPKsiPsiiiib12ChromaFormatRK6ClpRngibb(InterpolationFilter *self, ComponentID c, const Pel *src, int ss, Pel *dst, int ds, int w, int h, int frac, bool last, ChromaFormat f, const ClpRng &r, int idx, bool dmvr, bool alt) {
  g_refCalls[RC_FILTER_HOR]++;
  __real__ZN19InterpolationFilter9filterHorE11ComponentIDPKsiPsiiiib12ChromaFormatRK6ClpRngibb(self, c, src, ss, dst, ds, w, h, frac, last, f, r, idx, dmvr, alt);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
int main(int argc, char *argv[]) {
#ifdef VVCR_DROPIN
  g_dir = "<libvvcr>";   // every picture goes through the capture hooks (in memory) and libvvcr
#else
  const char *d = getenv("VVCR_CAPTURE_DIR");
  g_dir = d ? d : "";
#endif
  DecApp *app = new DecApp;
  if (!app->parseCfg(argc, argv)) { delete app; return 1; }
  uint32_t ret = app->decode();
  delete app;
#ifdef VVCR_DROPIN
  long ran = 0;
  for (int k = 0; k < RC_N; k++) ran += g_refCalls[k];
  fprintf(stderr, "vtm_vvcr: %d pictures decoded through libvvcr, %ld calls into the reference's reconstruction and loop filters\n",
          g_picCounter, ran);
  for (int k = 0; k < RC_N; k++) fprintf(stderr, "vtm_vvcr:   %s %ld\n", kRcName[k], g_refCalls[k]);
  if (g_vvcr) vvcr_destroy(g_vvcr);
  if (ran) return 2;
#endif
  return ret != 0 ? 1 : 0;
}
