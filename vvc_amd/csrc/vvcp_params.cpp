// vvcp_params.cpp — see vvcp_params.h.
#include "vvcp_params.h"

#include <cstring>

#include "vvcp_alf_fixed.h"

namespace vvcp {

namespace {
constexpr int FP_PREC = 11, CSCALE_FP_PREC = 11, CW_BINS = 16;   // CommonDef.h:483-486
constexpr int ALF_VB_POS_ABOVE_CTUROW_LUMA = 4, ALF_VB_POS_ABOVE_CTUROW_CHMA = 2;

// Reshape::constructReshaper (Reshape.cpp:241) for the model of an LMCS APS
void construct_reshaper(const LmcsApsParam &m, int bitDepth, vvcr_pic_params &pp) {
  const int lutSize = 1 << bitDepth, initCW = lutSize / CW_BINS;
  int binCW[CW_BINS], pivot[CW_BINS + 1], inPivot[CW_BINS + 1], fwdScale[CW_BINS], invScale[CW_BINS];
  for (int i = 0; i < CW_BINS; i++) binCW[i] = (i < m.minBin || i > m.maxBin) ? 0 : (uint16_t)(m.binDelta[i] + initCW);
  pivot[0] = inPivot[0] = 0;
  const int binLenLog2 = floorLog2((uint32_t)initCW);
  for (int i = 0; i < CW_BINS; i++) {
    pivot[i + 1] = pivot[i] + binCW[i];
    inPivot[i + 1] = inPivot[i] + initCW;
    fwdScale[i] = (binCW[i] * (1 << FP_PREC) + (1 << (binLenLog2 - 1))) >> binLenLog2;
    if (binCW[i] == 0) {
      invScale[i] = 0;
      pp.lmcs_cadj[i] = 1 << CSCALE_FP_PREC;
    } else {
      invScale[i] = initCW * (1 << FP_PREC) / binCW[i];
      pp.lmcs_cadj[i] = initCW * (1 << FP_PREC) / (binCW[i] + m.chrOffset);
    }
  }
  auto pwlIdxInv = [&](int v) {   // Reshape::getPWLIdxInv (:204)
    int i = m.minBin;
    for (; i <= m.maxBin; i++)
      if (v < pivot[i + 1]) break;
    return std::min(i, CW_BINS - 1);
  };
  const int maxV = lutSize - 1;
  VVCP_CHECK(lutSize > 1024, "LMCS tables above 10 bits are not supported");
  for (int s = 0; s < lutSize; s++) {
    const int iy = s / initCW;
    const int f = pivot[iy] + ((fwdScale[iy] * (s - inPivot[iy]) + (1 << (FP_PREC - 1))) >> FP_PREC);
    pp.lmcs_fwd[s] = (int16_t)clip3(0, maxV, f);
    const int ii = pwlIdxInv(s);
    const int v = inPivot[ii] + ((invScale[ii] * (s - pivot[ii]) + (1 << (FP_PREC - 1))) >> FP_PREC);
    pp.lmcs_inv[s] = (int16_t)clip3(0, maxV, v);
  }
  for (int i = 0; i <= CW_BINS; i++) pp.lmcs_pivot[i] = (int16_t)pivot[i];
  pp.lmcs_min_bin = m.minBin;
  pp.lmcs_max_bin = m.maxBin;
}
}  // namespace

void build_pic_params(const PictureUnit &p, vvcr_pic_params &pp) {
  std::memset(&pp, 0, sizeof(pp));
  VVCP_CHECK(p.slices.empty(), "picture without slices");
  const SPS &sps = p.sps;
  const PPS &pps = p.pps;
  const PicHeader &ph = p.ph;
  const SliceHeader &sh = p.slices.back();
  for (const SliceHeader &s : p.slices) {   // vvcr_pic_params carries one reference structure per picture
    bool same = s.numRef[0] == sh.numRef[0] && s.numRef[1] == sh.numRef[1];
    for (int l = 0; l < 2 && same; l++)
      for (int r = 0; r < sh.numRef[l]; r++) same &= s.refPoc[l][r] == sh.refPoc[l][r];
    VVCP_CHECK(!same, "slices of one picture with different reference lists are not supported");
  }
  pp.poc = p.poc;
  pp.slice_type = sh.sliceType;
  pp.slice_qp = sh.qp;
  for (int l = 0; l < 2; l++) {
    pp.num_ref[l] = sh.numRef[l];
    for (int r = 0; r < VVCR_MAX_REF; r++) {
      pp.ref_poc[l][r] = r < sh.numRef[l] ? sh.refPoc[l][r] : -1;
      pp.ref_lt[l][r] = r < sh.numRef[l] ? sh.refLT[l][r] : 0;
    }
  }
  pp.dual_tree = sh.isIntra() && sps.dualTree;
  pp.dep_quant = ph.depQuant;
  pp.sign_hiding = ph.signHiding;
  pp.joint_cbcr = sps.jointCbCr;
  pp.bdof_enabled = sps.bdof && !ph.disBdof;
  pp.dmvr_enabled = sps.dmvr && !ph.disDmvr;
  pp.prof_enabled = sps.prof && !ph.disProf;
  pp.lfnst_enabled = sps.lfnst;
  pp.mts_intra = sps.intraMts;
  pp.mts_inter = sps.interMts;
  pp.sbt = sps.sbt;
  pp.wp_p = pps.useWP;
  pp.wp_b = pps.wpBi;
  // weighted prediction after Slice::initWpScaling (Slice.cpp:1489): weight 1 << denom and offset 0
  // when absent; the library scales offsets to the bit depth itself
  for (int l = 0; l < 2; l++)
    for (int r = 0; r < sh.numRef[l]; r++)
      for (int c = 0; c < 3; c++) {
        const int *w = sh.wp[l][r][c];
        int32_t *o = pp.wp[l][r][c];
        o[0] = w[0]; o[1] = w[1];
        o[2] = w[0] ? w[2] : 1 << w[1];
        o[3] = w[0] ? w[3] : 0;
        o[4] = o[2]; o[5] = o[3] * (1 << (sps.bitDepth - 8));
      }
  pp.dbk_disable = sh.dbkDisable;
  pp.dbk_beta_offset_div2 = sh.betaOffsetDiv2;
  pp.dbk_tc_offset_div2 = sh.tcOffsetDiv2;
  pp.lf_across_slices = pps.lfAcrossSlices;
  pp.lf_across_tiles = pps.lfAcrossTiles;
  pp.vb_disabled = ph.vbDisabled && (ph.numVbVer + ph.numVbHor) > 0;
  pp.num_vb_ver = pp.vb_disabled ? ph.numVbVer : 0;
  pp.num_vb_hor = pp.vb_disabled ? ph.numVbHor : 0;
  for (int i = 0; i < 3; i++) { pp.vb_ver[i] = ph.vbPosX[i]; pp.vb_hor[i] = ph.vbPosY[i]; }
  pp.ladf_num = sps.ladf ? sps.ladfNum : 0;
  for (int k = 0; k < 5; k++) { pp.ladf_qp_offset[k] = sps.ladfQpOffset[k]; pp.ladf_lower_bound[k] = sps.ladfLowerBound[k]; }
  pp.chroma_qp_off[1] = pps.cbQpOffset + sh.cbQpDelta;
  pp.chroma_qp_off[2] = pps.crQpOffset + sh.crQpDelta;
  pp.chroma_qp_off[0] = pps.jcQpOffset + sh.jcQpDelta;
  for (int q = -sps.qpBdOffset; q < 64; q++) {   // SPS::getMappedChromaQpValue; row 0 = JOINT_CbCr
    pp.chroma_qp_map[0][q + 64] = sps.mappedChromaQp(3, q);
    pp.chroma_qp_map[1][q + 64] = sps.mappedChromaQp(1, q);
    pp.chroma_qp_map[2][q + 64] = sps.mappedChromaQp(2, q);
  }
  pp.sao_luma = sh.sao[0];
  pp.sao_chroma = sh.sao[1];
  for (int c = 0; c < 3; c++) pp.alf_en[c] = sh.alf[c];
  pp.ccalf_en[0] = sh.ccAlf[0];
  pp.ccalf_en[1] = sh.ccAlf[1];
  // AdaptiveLoopFilter::create (AdaptiveLoopFilter.cpp:735)
  pp.alf_vb_luma = sps.ctuSize - ALF_VB_POS_ABOVE_CTUROW_LUMA;
  pp.alf_vb_chroma = (sps.ctuSize >> 1) - ALF_VB_POS_ABOVE_CTUROW_CHMA;
  pp.lmcs_enabled = sps.lmcs && ph.lmcs;
  pp.lmcs_chroma_scale = ph.lmcs && ph.lmcsChroma;
  if (pp.lmcs_enabled) {
    VVCP_CHECK(ph.lmcsApsId < 0 || ph.lmcsApsId > 3 || !p.lmcsValid[ph.lmcsApsId], "LMCS APS missing");
    construct_reshaper(p.lmcsAps[ph.lmcsApsId].lmcs, sps.bitDepth, pp);
  }
  pp.max_tb_log2 = sps.log2MaxTb;
  pp.log2_max_ts = pps.log2MaxTs;
  pp.use_mts = sps.mts;
  pp.implicit_mts = sps.mts && !sps.intraMts;
  pp.joint_cbcr_sign = ph.jointCbCrSign;
  pp.num_tile_cols = pps.numTileCols();
  pp.num_tile_rows = (int)pps.rowBd.size() - 1;
  VVCP_CHECK(pp.num_tile_cols > VVCR_MAX_TILE_LINES || pp.num_tile_rows > VVCR_MAX_TILE_LINES, "too many tiles");
  for (size_t i = 0; i < pps.colBd.size(); i++) pp.tile_col_bd[i] = pps.colBd[i];
  for (size_t i = 0; i < pps.rowBd.size(); i++) pp.tile_row_bd[i] = pps.rowBd[i];
  pp.entropy_sync = pps.entropySync;
}

// AdaptiveLoopFilter::reconstructCoeffAPSs / reconstructCoeff (AdaptiveLoopFilter.cpp:620-713) with the
// clipping table of AdaptiveLoopFilter::create (:743-762, JVET_Q0495)
void build_alf(const PictureUnit &p, AlfFilters &f) {
  const SliceHeader &sh = p.slices.back();
  const int bd = p.sps.bitDepth;
  int clipVal[4];
  clipVal[0] = 1 << bd;
  for (int i = 1; i < 4; i++) clipVal[i] = 1 << (7 - 2 * i + bd - 8);
  const int factor = 1 << (8 - 1);   // m_NUM_BITS = 8
  const int nAps = sh.alf[0] ? sh.numAlfAps : 0;
  f.numLumaSets = 16 + nAps;
  f.lumaCoef.assign((size_t)f.numLumaSets * 25 * 13, 0);
  f.lumaClip.assign((size_t)f.numLumaSets * 25 * 13, 0);
  for (int s = 0; s < 16; s++)
    for (int c = 0; c < 25; c++)
      for (int k = 0; k < 13; k++) {
        f.lumaCoef[((size_t)s * 25 + c) * 13 + k] = vvcp_alf::kFixed[s][c][k];
        f.lumaClip[((size_t)s * 25 + c) * 13 + k] = (int16_t)clipVal[0];   // m_clipDefault
      }
  for (int i = 0; i < nAps; i++) {
    const int id = sh.alfApsLuma[i];
    VVCP_CHECK(id < 0 || id > 7 || !p.alfValid[id] || !p.alfAps[id].alf.newLuma, "ALF luma APS missing");
    const AlfApsParam &a = p.alfAps[id].alf;
    for (int c = 0; c < 25; c++) {
      const int fi = a.deltaIdx[c];
      VVCP_CHECK(fi < 0 || fi >= a.numLumaFilters, "bad ALF filter index");
      int16_t *co = &f.lumaCoef[((size_t)(16 + i) * 25 + c) * 13], *cl = &f.lumaClip[((size_t)(16 + i) * 25 + c) * 13];
      for (int k = 0; k < 12; k++) {
        co[k] = a.lumaCoeff[fi * 13 + k];
        cl[k] = (int16_t)clipVal[a.nonLinear[0] ? a.lumaClip[fi * 13 + k] : 0];
      }
      co[12] = (int16_t)factor;
      cl[12] = (int16_t)clipVal[0];
    }
  }
  std::memset(f.chromaCoef, 0, sizeof(f.chromaCoef));
  std::memset(f.chromaClip, 0, sizeof(f.chromaClip));
  if (sh.alf[1] || sh.alf[2]) {
    const int id = sh.alfApsChroma;
    VVCP_CHECK(id < 0 || id > 7 || !p.alfValid[id] || !p.alfAps[id].alf.newChroma, "ALF chroma APS missing");
    const AlfApsParam &a = p.alfAps[id].alf;
    for (int alt = 0; alt < a.numAltChroma; alt++) {
      for (int k = 0; k < 6; k++) {
        f.chromaCoef[alt][k] = a.chromaCoeff[alt][k];
        f.chromaClip[alt][k] = (int16_t)clipVal[a.nonLinear[1] ? a.chromaClip[alt][k] : 0];
      }
      f.chromaCoef[alt][6] = (int16_t)factor;
      f.chromaClip[alt][6] = (int16_t)clipVal[0];
    }
  }
  std::memset(f.ccCoef, 0, sizeof(f.ccCoef));
  for (int c = 0; c < 2; c++) {
    if (!sh.ccAlf[c]) continue;
    const int id = sh.ccAlfApsId[c];
    VVCP_CHECK(id < 0 || id > 7 || !p.alfValid[id] || !p.alfAps[id].alf.ccNew[c], "CC-ALF APS missing");
    const AlfApsParam &a = p.alfAps[id].alf;
    for (int fi = 0; fi < a.ccCount[c]; fi++)
      for (int k = 0; k < 7; k++) f.ccCoef[c][fi][k] = a.ccCoeff[c][fi][k];
  }
}

}  // namespace vvcp
