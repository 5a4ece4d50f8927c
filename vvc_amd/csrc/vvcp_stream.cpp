// vvcp_stream.cpp — see vvcp_stream.h. Picture boundaries, POC and reference lists follow
// DecLib::decode / xDecodeSlice (DecLib.cpp:1339-1645); the C-ABI of include/vvcp.h is at the end.
#include "vvcp_stream.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <tuple>

#include "vvcp.h"
#include "vvcp_params.h"

namespace vvcp {

namespace {
// DecLib.cpp:1535-1642 (checkLDC, SMVD reference pair) and Slice::constructRefPicList (Slice.cpp:414)
void derive_refs(SliceHeader &s) {
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < VVCR_MAX_REF; i++) { s.refPoc[l][i] = 0; s.refLT[l][i] = false; }
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < s.numRef[l]; i++) {
      VVCP_CHECK(i >= s.rpl[l].num, "active reference beyond the list");
      VVCP_CHECK(s.rpl[l].isLT[i], "long-term references are not supported");
      s.refPoc[l][i] = s.poc - s.rpl[l].ident[i];
      s.refLT[l][i] = false;
    }
  s.checkLDC = false;
  s.biDirPred = false;
  s.symRefIdx[0] = s.symRefIdx[1] = -1;
  if (s.isIntra()) return;
  bool low = true;
  for (int i = 0; i < s.numRef[0] && low; i++)
    if (s.refPoc[0][i] > s.poc) low = false;
  if (s.isInterB())
    for (int i = 0; i < s.numRef[1] && low; i++)
      if (s.refPoc[1][i] > s.poc) low = false;
  s.checkLDC = low;
}
void derive_smvd(SliceHeader &s, const SPS &sps, const PicHeader &ph) {
  if (!(sps.smvd && !s.checkLDC && !ph.mvdL1Zero)) return;
  const int cur = s.poc;
  int fwd = cur, bwd = cur, r0 = -1, r1 = -1;
  for (int r = 0; r < s.numRef[0]; r++) {
    const int poc = s.refPoc[0][r];
    if (poc < cur && (poc > fwd || r0 == -1) && !s.refLT[0][r]) { fwd = poc; r0 = r; }
  }
  for (int r = 0; r < s.numRef[1]; r++) {
    const int poc = s.refPoc[1][r];
    if (poc > cur && (poc < bwd || r1 == -1) && !s.refLT[1][r]) { bwd = poc; r1 = r; }
  }
  if (!(fwd < cur && bwd > cur)) {
    fwd = bwd = cur;
    r0 = r1 = -1;
    for (int r = 0; r < s.numRef[0]; r++) {
      const int poc = s.refPoc[0][r];
      if (poc > cur && (poc < bwd || r0 == -1) && !s.refLT[0][r]) { bwd = poc; r0 = r; }
    }
    for (int r = 0; r < s.numRef[1]; r++) {
      const int poc = s.refPoc[1][r];
      if (poc < cur && (poc > fwd || r1 == -1) && !s.refLT[1][r]) { fwd = poc; r1 = r; }
    }
  }
  if (fwd < cur && bwd > cur) { s.biDirPred = true; s.symRefIdx[0] = r0; s.symRefIdx[1] = r1; }
}
}  // namespace

// sei_rbsp (SEIReader::parseSEImessage, SEIread.cpp:117): the decoded picture hash message (type 132)
static void parse_sei_hash(const std::vector<uint8_t> &r, PictureUnit &p) {
  size_t pos = 0;
  while (pos < r.size() && !(pos + 1 == r.size() && r[pos] == 0x80)) {
    uint32_t type = 0, size = 0;
    while (pos < r.size() && r[pos] == 0xff) { type += 255; pos++; }
    if (pos >= r.size()) return;
    type += r[pos++];
    while (pos < r.size() && r[pos] == 0xff) { size += 255; pos++; }
    if (pos >= r.size()) return;
    size += r[pos++];
    if (pos + size > r.size()) return;
    if (type == 132 && size >= 1) {
      const int t = r[pos];
      const int per = t == 0 ? 16 : (t == 1 ? 2 : (t == 2 ? 4 : 0));
      if (per && size >= 1 + 3 * (uint32_t)per) {
        p.hashType = t;
        for (int c = 0; c < 3; c++) std::memcpy(p.hash[c], &r[pos + 1 + c * per], per);
      }
    }
    pos += size;
  }
}

void Stream::open(const uint8_t *d, size_t n) {
  data.assign(d, d + n);
  nals = split_annexb(data.data(), data.size());
  ParamSets ps;
  PicHeader ph;
  int prevTid0Poc = 0;
  PictureUnit *cur = nullptr;
  for (size_t k = 0; k < nals.size(); k++) {
    Nal &nal = nals[k];
    if (is_vcl(nal.type)) {   // trailing cabac_zero_words (NALread.cpp:89)
      while (!nal.rbsp.empty() && nal.rbsp.back() == 0) nal.rbsp.pop_back();
    }
    Bits b(nal.rbsp.data(), nal.rbsp.size());
    switch (nal.type) {
      case NAL_SPS:
      case NAL_PPS: {
        if (nal.type == NAL_SPS) { SPS s; parse_sps(b, s); ps.spsMap[s.id] = s; }
        else { PPS p; parse_pps(b, p); ps.ppsMap[p.id] = p; }
        for (auto &kv : ps.ppsMap) {   // tile layout needs the CTU size of the referenced SPS
          const SPS *sps = ps.sps(kv.second.spsId);
          if (sps) finalize_pps(kv.second, *sps);
        }
        break;
      }
      case NAL_PREFIX_APS:
      case NAL_SUFFIX_APS: {
        APS a;
        parse_aps(b, a);
        a.tid = nal.tid;
        if (a.type == 0) { VVCP_CHECK(a.id > 7, "bad ALF APS id"); ps.alfAps[a.id] = a; ps.alfValid[a.id] = true; }
        else { VVCP_CHECK(a.id > 3, "bad LMCS APS id"); ps.lmcsAps[a.id] = a; ps.lmcsValid[a.id] = true; }
        break;
      }
      case NAL_PH:
        parse_ph(b, ph, ps);
        cur = nullptr;   // next slice starts a new picture
        break;
      case NAL_SUFFIX_SEI:
        if (cur) parse_sei_hash(nal.rbsp, *cur);   // the hash of the picture whose slices it follows
        break;
      default:
        if (nal.type <= NAL_GDR && is_vcl(nal.type)) {
          SliceHeader sh;
          sh.nalType = nal.type;
          sh.tid = nal.tid;
          const bool phInSh = nal.rbsp.size() > 0 && (nal.rbsp[0] & 0x80);
          if (phInSh) cur = nullptr;
          parse_sh(b, sh, ph, ps, prevTid0Poc);
          const PPS *pps = ps.pps(ph.ppsId);
          const SPS *sps = ps.sps(pps->spsId);
          if (!cur) {
            pics.emplace_back(new PictureUnit());
            cur = pics.back().get();
            cur->poc = sh.poc;
            cur->nalType = nal.type;
            cur->tid = nal.tid;
            cur->sps = *sps;
            cur->pps = *pps;
            cur->ph = ph;
            for (int i = 0; i < 8; i++) { cur->alfAps[i] = ps.alfAps[i]; cur->alfValid[i] = ps.alfValid[i]; }
            for (int i = 0; i < 4; i++) { cur->lmcsAps[i] = ps.lmcsAps[i]; cur->lmcsValid[i] = ps.lmcsValid[i]; }
          }
          VVCP_CHECK(sh.poc != cur->poc, "slices of one picture with different POC");
          derive_refs(sh);
          derive_smvd(sh, cur->sps, cur->ph);
          sh.indepSliceIdx = (int)cur->slices.size();
          cur->slices.push_back(sh);
          cur->sliceNal.push_back((int)k);
          if (nal.tid == 0 && nal.type != NAL_RASL && nal.type != NAL_RADL) prevTid0Poc = sh.poc;   // DecLib.h:209
        }
        break;
    }
  }
}

// Threads of a picture's tile-parallel CABAC pass (parse_picture_data): VVCP_TILE_THREADS, default 8; 1 parses
// the tiles in order on the calling thread
static int tile_threads() {
  static const int n = [] {
    const char *e = std::getenv("VVCP_TILE_THREADS");
    const int v = e ? std::atoi(e) : 8;
    return std::max(1, std::min(v, 64));
  }();
  return n;
}

void Stream::parse_picture(int idx) {
  PictureUnit &p = *pics.at(idx);
  if (p.parsed) {
    VVCP_CHECK(p.failed, "picture failed to parse");
    return;
  }
  bool intra = !p.slices.empty();
  for (const auto &sh : p.slices) intra = intra && sh.isIntra();
  p.syn.reset(p.pps.width, p.pps.height, p.sps.ctuLog2, intra);
  ParamSets ps;
  for (int i = 0; i < 8; i++) { ps.alfAps[i] = p.alfAps[i]; ps.alfValid[i] = p.alfValid[i]; }
  for (int i = 0; i < 4; i++) { ps.lmcsAps[i] = p.lmcsAps[i]; ps.lmcsValid[i] = p.lmcsValid[i]; }
  try {
    std::vector<SliceData> sd;
    for (size_t s = 0; s < p.slices.size(); s++) {
      const Nal &nal = nals[p.sliceNal[s]];
      sd.push_back({SliceCtx{&p.sps, &p.pps, &p.ph, &p.slices[s], &ps, (int)s}, nal.rbsp.data(), nal.rbsp.size(), &nal.epb});
    }
    const int lg = p.sps.ctuLog2;
    const int ry0 = std::max(0, parseY0) >> lg, ry1 = parseY1 >= (1 << 30) ? (1 << 30) : (std::max(0, parseY1) + (1 << lg) - 1) >> lg;
    std::tie(p.parseR0, p.parseR1) = parse_picture_data(p.syn, sd, tile_threads(), ry0, ry1);
  } catch (...) {
    p.parsed = true;   // the rows parsed so far stay readable (diagnostics)
    p.failed = true;
    throw;
  }
  finish_picture_syntax(p.syn, p.sps.bitDepth);
  p.parsed = true;
}

void Stream::derive_motion(int idx) {
  PictureUnit &p = *pics.at(idx);
  VVCP_CHECK(!p.parsed || p.failed, "picture not parsed");
  if (p.derived) return;
  std::vector<const MotionPicture *> dpb;
  for (int i = std::max(0, idx - 64); i < idx; i++)
    if (pics[i]->refined) dpb.push_back(pics[i]->refined.get());
  vvcp::derive_motion(p, dpb, p.field, p.motion, p.geo);
  p.derived = true;
}

void Stream::refine_motion(int idx, const int32_t *deltas, int64_t n) {
  PictureUnit &p = *pics.at(idx);
  VVCP_CHECK(!p.derived, "picture motion not derived");
  std::unique_ptr<MotionPicture> m(new MotionPicture());
  vvcp::refine_motion(p, std::move(p.field), deltas, n, *m);
  p.refined = std::move(m);
  // pictures far behind in decoding order are no longer collocated candidates
  if (idx >= 64 && pics[idx - 64]->refined) pics[idx - 64]->refined.reset();
}

}  // namespace vvcp

// ================================================================================================
// C-ABI (include/vvcp.h)
// ================================================================================================
static thread_local std::string g_vvcp_err;
void vvcp::set_api_error(const std::string &msg) { g_vvcp_err = msg; }

#define VVCP_API_BEGIN try {
#define VVCP_API_END                                              \
  }                                                               \
  catch (const std::exception &e) {                               \
    g_vvcp_err = e.what();                                        \
    return VVCR_E_UNSUPPORTED;                                    \
  }

extern "C" {

int vvcp_open(const uint8_t *data, size_t n, vvcp_stream **out) {
  if (!data || !out) return VVCR_E_ARG;
  *out = nullptr;
  VVCP_API_BEGIN
  std::unique_ptr<vvcp_stream> h(new vvcp_stream());
  h->s.open(data, n);
  *out = h.release();
  return VVCR_OK;
  VVCP_API_END
}

int vvcp_close(vvcp_stream *h) {
  delete h;
  return VVCR_OK;
}

const char *vvcp_last_error(void) { return g_vvcp_err.c_str(); }

int vvcp_num_pictures(const vvcp_stream *h) { return h ? (int)h->s.pics.size() : VVCR_E_ARG; }

int vvcp_picture_info(const vvcp_stream *h, int32_t idx, int32_t *info, int32_t n) {
  if (!h || !info || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  const vvcp::PictureUnit &p = *h->s.pics[idx];
  const int sw = p.sps.chromaFormat == 1 || p.sps.chromaFormat == 2 ? 2 : 1, shh = p.sps.chromaFormat == 1 ? 2 : 1;
  const int32_t v[] = {p.poc, p.slices.empty() ? 2 : p.slices[0].sliceType, p.pps.width, p.pps.height, p.sps.ctuLog2,
                       p.sps.bitDepth, (int32_t)p.slices.size(), p.tid, p.nalType, p.slices.empty() ? 0 : p.slices[0].qp,
                       p.pps.confLeft * sw, p.pps.confRight * sw, p.pps.confTop * shh, p.pps.confBottom * shh,
                       p.ph.picOutput ? 1 : 0, p.ph.nonRef ? 1 : 0};
  const int m = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < m; i++) info[i] = v[i];
  return m;
}

int vvcp_picture_hash(const vvcp_stream *h, int32_t idx, uint8_t *out, int32_t n) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  const vvcp::PictureUnit &p = *h->s.pics[idx];
  if (p.hashType < 0) return -1;
  const int per = p.hashType == 0 ? 16 : (p.hashType == 1 ? 2 : 4);
  for (int c = 0; c < 3; c++)
    for (int k = 0; k < per && c * per + k < n; k++) out[c * per + k] = p.hash[c][k];
  return p.hashType;
}

int vvcp_parse_picture(vvcp_stream *h, int32_t idx) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  VVCP_API_BEGIN
  h->s.parse_picture(idx);
  return VVCR_OK;
  VVCP_API_END
}

int vvcp_set_parse_rows(vvcp_stream *h, int32_t y0, int32_t y1) {
  if (!h) return VVCR_E_ARG;
  if (y1 <= y0) { h->s.parseY0 = 0; h->s.parseY1 = 1 << 30; }
  else { h->s.parseY0 = y0; h->s.parseY1 = y1; }
  return VVCR_OK;
}

int vvcp_dmvr_split(const vvcp_stream *h, int32_t idx, int32_t y0, int32_t y1, int64_t *out) {
  if (!h || !out || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  const vvcp::PictureUnit &p = *h->s.pics[idx];
  if (!p.derived) return VVCR_E_STATE;
  out[0] = out[1] = out[2] = 0;
  if (p.rowsMoved) return VVCR_OK;   // planned with no DMVR refinement to wait for: none of its PUs refines
  for (const vvcr_pu &u : p.syn.pu) {
    if (!u.dmvr) continue;
    const int dy = std::min(u.h, 16), dx = std::min(u.w, 16);
    out[u.y < y0 ? 0 : (u.y < y1 ? 1 : 2)] += (int64_t)(u.h / dy) * (u.w / dx);
  }
  return VVCR_OK;
}

int vvcp_derive_motion(vvcp_stream *h, int32_t idx) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  VVCP_API_BEGIN
  h->s.derive_motion(idx);
  return VVCR_OK;
  VVCP_API_END
}

int vvcp_refine_motion(vvcp_stream *h, int32_t idx, const int32_t *deltas, int64_t n) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size() || n < 0) return VVCR_E_ARG;
  VVCP_API_BEGIN
  h->s.refine_motion(idx, deltas, n);
  return VVCR_OK;
  VVCP_API_END
}

int vvcp_picture_params(const vvcp_stream *h, int32_t idx, vvcr_pic_params *pp) {
  if (!h || !pp || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  VVCP_API_BEGIN
  vvcp::build_pic_params(*h->s.pics[idx], *pp);
  return VVCR_OK;
  VVCP_API_END
}

int vvcp_alf_filters(const vvcp_stream *h, int32_t idx, int16_t *luma_coef, int16_t *luma_clip, int32_t max_sets,
                     int16_t *chroma_coef, int16_t *chroma_clip, int16_t *cc_coef) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  VVCP_API_BEGIN
  vvcp::AlfFilters f;
  vvcp::build_alf(*h->s.pics[idx], f);
  const size_t per = 25 * 13;
  const int n = std::min(max_sets, f.numLumaSets);
  if (luma_coef && n > 0) std::memcpy(luma_coef, f.lumaCoef.data(), n * per * sizeof(int16_t));
  if (luma_clip && n > 0) std::memcpy(luma_clip, f.lumaClip.data(), n * per * sizeof(int16_t));
  if (chroma_coef) std::memcpy(chroma_coef, f.chromaCoef, sizeof(f.chromaCoef));
  if (chroma_clip) std::memcpy(chroma_clip, f.chromaClip, sizeof(f.chromaClip));
  if (cc_coef) std::memcpy(cc_coef, f.ccCoef, sizeof(f.ccCoef));
  return f.numLumaSets;
  VVCP_API_END
}

int64_t vvcp_picture_rows(const vvcp_stream *h, int32_t idx, int32_t what, void *dst, int64_t cap) {
  if (!h || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  const vvcp::PictureUnit &p = *h->s.pics[idx];
  if (!p.parsed) return VVCR_E_STATE;
  const vvcp::PictureSyntax &s = p.syn;
  const void *src = nullptr;
  int64_t count = 0, esz = 0;
  std::vector<vvcr_tu> dtu;     // TU rows and coefficient pool in vvcr_picture_submit's dense form
  std::vector<int32_t> dcoef;
  if (what == VVCP_ROWS_TU || what == VVCP_ROWS_COEF) {
    if (p.handedOver) return VVCR_E_STATE;
    s.dense_rows(dtu, dcoef);
  }
  if ((what == VVCP_ROWS_CU || what == VVCP_ROWS_PU) && p.rowsMoved) return VVCR_E_STATE;
  switch (what) {
    case VVCP_ROWS_CU: src = s.cu.data(); count = (int64_t)s.cu.size(); esz = sizeof(vvcr_cu); break;
    case VVCP_ROWS_PU: src = s.pu.data(); count = (int64_t)s.pu.size(); esz = sizeof(vvcr_pu); break;
    case VVCP_ROWS_TU: src = dtu.data(); count = (int64_t)dtu.size(); esz = sizeof(vvcr_tu); break;
    case VVCP_ROWS_COEF: src = dcoef.data(); count = (int64_t)dcoef.size(); esz = 4; break;
    case VVCP_ROWS_SAO: src = s.sao.data(); count = (int64_t)s.sao.size(); esz = sizeof(vvcr_sao); break;
    case VVCP_ROWS_ALF_EN0: case VVCP_ROWS_ALF_EN0 + 1: case VVCP_ROWS_ALF_EN0 + 2:
      src = s.alfEn[what - VVCP_ROWS_ALF_EN0].data(); count = (int64_t)s.alfEn[0].size(); esz = 1; break;
    case VVCP_ROWS_ALF_ALT0: case VVCP_ROWS_ALF_ALT0 + 1: case VVCP_ROWS_ALF_ALT0 + 2:
      src = s.alfAlt[what - VVCP_ROWS_ALF_ALT0].data(); count = (int64_t)s.alfAlt[0].size(); esz = 1; break;
    case VVCP_ROWS_ALF_FSET: src = s.alfFset.data(); count = (int64_t)s.alfFset.size(); esz = 2; break;
    case VVCP_ROWS_CCALF0: case VVCP_ROWS_CCALF0 + 1:
      src = s.ccCtl[what - VVCP_ROWS_CCALF0].data(); count = (int64_t)s.ccCtl[0].size(); esz = 1; break;
    case VVCP_ROWS_MOTION:
      if (!p.derived) return VVCR_E_STATE;
      // the 24-byte internal records, widened to vvcr_motion rows; an intra picture has none: all-zero rows
      count = p.motion.empty() ? (int64_t)s.w4 * s.h4 : (int64_t)p.motion.size();
      if (dst && cap > 0)
        for (int64_t i = 0; i < std::min(cap, count); i++) ((vvcr_motion *)dst)[i] = from_rec(p.motion.empty() ? MotionRec{} : p.motion[i]);
      return count;
    case VVCP_ROWS_GEO:
      if (!p.derived) return VVCR_E_STATE;
      src = p.geo.data(); count = (int64_t)p.geo.size(); esz = sizeof(vvcr_geo); break;
    default: return VVCR_E_ARG;
  }
  if (dst && cap > 0) std::memcpy(dst, src, (size_t)(std::min(cap, count) * esz));
  return count;
}

}  // extern "C"
