// vvcr_api.cpp — C-ABI implementation of libvvcr: device DPB, descriptor staging, per-picture work-list
// construction on the host (C++), kernel launches on one ordered HIP stream.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "vvcr_internal.h"
#include "vvcr_host.h"
#include "vvcr_dbk.h"
#include "vvcr_intra.h"

namespace {

thread_local std::string g_create_error;

template <class T>
struct DevVec {
  T *p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) hipFree(p);
    size_t c = std::max<size_t>(n, cap * 3 / 2 + 64);
    VVCR_CHECK_HIP(hipMalloc(&p, c * sizeof(T)));
    cap = c;
  }
  void upload(const std::vector<T> &v, hipStream_t s) {
    ensure(v.size() + 1);
    if (!v.empty()) VVCR_CHECK_HIP(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  }
  ~DevVec() { if (p) hipFree(p); }
};

DPlane alloc_plane(int w, int h) {
  DPlane d;
  d.w = w; d.h = h;
  d.stride = (w + 63) & ~63;
  VVCR_CHECK_HIP(hipMalloc(&d.p, (size_t)d.stride * h * sizeof(int16_t)));
  VVCR_CHECK_HIP(hipMemset(d.p, 0, (size_t)d.stride * h * sizeof(int16_t)));
  return d;
}

}  // namespace

struct vvcr_ctx {
  vvcr_seq_params sp{};
  std::string err;
  hipStream_t stream = nullptr;
  std::vector<std::array<DPlane, 3>> dpb;
  DPlane pred[3], resi[3], tmp[3];
  vvcr_pic_params pp{};
  bool in_picture = false;
  PictureDescriptors desc;          // host copy of the submitted descriptors (vvcr_host.h)
  WorkLists wl;                     // host-built work lists
  DevVec<McJob> d_mc_basic, d_mc_bidir;
  DevVec<AffPu> d_aff_pu;
  DevVec<AffJob> d_aff_jobs;
  DevVec<int32_t> d_dmvr;           // DMVR deltas of the last picture, [n][2]
  int n_dmvr = 0;
  DevVec<TbJob> d_tb;
  DevVec<int32_t> d_coef;
  DevVec<uint16_t> d_scans;
  ScanTables scans;
  // loop-filter parameters of the current picture
  DevVec<int32_t> d_sao;
  DevVec<int16_t> d_alf_luma_coef, d_alf_luma_clip, d_alf_chroma, d_alf_cc;
  DevVec<uint8_t> d_alf_ctb;      // ctb_en[3n] | ctb_alt[3n] | cc_ctl[2n]
  DevVec<int16_t> d_alf_set;
  IntraPlan intra;
  DevVec<int32_t> d_order;          // luma | chroma order maps
  DevVec<ReconTile> d_tiles;
  DevVec<IntraJob> d_ijobs;
  DbkLists dbk;
  std::vector<DbkSeg> dbk_all;
  DevVec<DbkSeg> d_dbk;
  bool have_sao = false, have_alf = false;
  hipEvent_t ev[2] = {};            // whole end_picture call
  hipEvent_t sev[7][2] = {};        // per stage begin / end
  bool stage_ran[7] = {};
};

#define API_BEGIN try {
#define API_END                                                  \
  }                                                              \
  catch (const VvcrError &e) { ctx->err = e.msg; return e.code; } \
  catch (const std::exception &e) { ctx->err = e.what(); return VVCR_E_STATE; }

extern "C" {

int vvcr_create(const vvcr_seq_params *sp, vvcr_ctx **out) {
  if (!sp || !out) return VVCR_E_ARG;
  *out = nullptr;
  if (sp->chroma_format != 1 || sp->bit_depth < 8 || sp->bit_depth > 10 || sp->width <= 0 || sp->height <= 0 ||
      sp->dpb_slots <= 0 || sp->dpb_slots > 32) {
    g_create_error = "unsupported sequence parameters (4:2:0, 8..10 bit, <= 32 DPB slots)";
    return VVCR_E_UNSUPPORTED;
  }
  auto ctx = std::make_unique<vvcr_ctx>();
  ctx->sp = *sp;
  try {
    VVCR_CHECK_HIP(hipSetDevice(sp->device));
    VVCR_CHECK_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    const int W = sp->width, H = sp->height;
    ctx->dpb.resize(sp->dpb_slots);
    for (auto &s : ctx->dpb) {
      s[0] = alloc_plane(W, H);
      s[1] = alloc_plane(W / 2, H / 2);
      s[2] = alloc_plane(W / 2, H / 2);
    }
    for (int c = 0; c < 3; c++) {
      int w = c ? W / 2 : W, h = c ? H / 2 : H;
      ctx->pred[c] = alloc_plane(w, h);
      ctx->resi[c] = alloc_plane(w, h);
      ctx->tmp[c] = alloc_plane(w, h);
    }
    for (auto &e : ctx->ev) VVCR_CHECK_HIP(hipEventCreate(&e));
    for (auto &se : ctx->sev)
      for (auto &e : se) VVCR_CHECK_HIP(hipEventCreate(&e));
    build_scan_tables(ctx->scans);
    ctx->d_scans.upload(ctx->scans.data, ctx->stream);
  } catch (const VvcrError &e) {
    g_create_error = e.msg;
    return e.code;
  }
  *out = ctx.release();
  return VVCR_OK;
}

int vvcr_destroy(vvcr_ctx *ctx) {
  if (!ctx) return VVCR_E_ARG;
  hipStreamSynchronize(ctx->stream);
  for (auto &s : ctx->dpb)
    for (auto &p : s) hipFree(p.p);
  for (int c = 0; c < 3; c++) { hipFree(ctx->pred[c].p); hipFree(ctx->resi[c].p); hipFree(ctx->tmp[c].p); }
  for (auto &e : ctx->ev) if (e) hipEventDestroy(e);
  for (auto &se : ctx->sev)
    for (auto &e : se) if (e) hipEventDestroy(e);
  hipStreamDestroy(ctx->stream);
  delete ctx;
  return VVCR_OK;
}

const char *vvcr_last_error(vvcr_ctx *ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

void *vvcr_stream(vvcr_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int vvcr_begin_picture(vvcr_ctx *ctx, const vvcr_pic_params *pp) {
  if (!ctx || !pp) return VVCR_E_ARG;
  API_BEGIN
  if (pp->slot < 0 || pp->slot >= (int)ctx->dpb.size()) throw VvcrError(VVCR_E_ARG, "picture slot out of range");
  for (int l = 0; l < 2; l++) {
    if (pp->num_ref[l] < 0 || pp->num_ref[l] > VVCR_MAX_REF) throw VvcrError(VVCR_E_ARG, "bad num_ref");
    for (int i = 0; i < pp->num_ref[l]; i++)
      if (pp->ref_slot[l][i] < 0 || pp->ref_slot[l][i] >= (int)ctx->dpb.size()) throw VvcrError(VVCR_E_ARG, "ref slot out of range");
  }
  ctx->pp = *pp;
  ctx->desc.clear();
  ctx->have_sao = ctx->have_alf = false;   // loop-filter parameters are per picture
  ctx->in_picture = true;
  return VVCR_OK;
  API_END
}

int vvcr_submit(vvcr_ctx *ctx, const vvcr_cu *cu, int32_t ncu, const vvcr_pu *pu, int32_t npu, const vvcr_tu *tu,
                int32_t ntu, const int32_t *coef, int64_t ncoef, const vvcr_motion *motion, const vvcr_geo *geo,
                int32_t ngeo, const int32_t *dmvr_delta_unused, int32_t nd) {
  (void)dmvr_delta_unused; (void)nd;
  if (!ctx || ncu < 0 || npu < 0 || ntu < 0 || ncoef < 0 || ngeo < 0) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_submit outside begin/end picture");
  auto &d = ctx->desc;
  d.cu.assign(cu, cu + ncu);
  d.pu.assign(pu, pu + npu);
  d.tu.assign(tu, tu + ntu);
  d.coef.assign(coef, coef + ncoef);
  const size_t nm = (size_t)(ctx->sp.width / 4) * (ctx->sp.height / 4);
  if (motion) d.motion.assign(motion, motion + nm); else d.motion.clear();
  d.geo.assign(geo, geo + ngeo);
  validate_descriptors(ctx->sp, ctx->pp, d);
  return VVCR_OK;
  API_END
}

static int n_ctb(const vvcr_seq_params &sp) {
  const int ctu = 1 << sp.ctu_log2;
  return ((sp.width + ctu - 1) / ctu) * ((sp.height + ctu - 1) / ctu);
}

int vvcr_set_loop_filter_params(vvcr_ctx *ctx, const vvcr_sao *sao, const vvcr_alf *alf) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_set_loop_filter_params outside begin/end picture");
  const int n = n_ctb(ctx->sp);
  hipStream_t s = ctx->stream;
  ctx->have_sao = sao != nullptr;
  if (sao) {
    std::vector<int32_t> v((const int32_t *)sao, (const int32_t *)sao + (size_t)n * 3 * 35);
    ctx->d_sao.upload(v, s);
  }
  ctx->have_alf = alf != nullptr;
  if (alf) {
    if (alf->num_luma_sets < 16 || alf->num_luma_sets > 24) throw VvcrError(VVCR_E_ARG, "bad ALF luma set count");
    const size_t L = (size_t)alf->num_luma_sets * 25 * 13;
    ctx->d_alf_luma_coef.upload(std::vector<int16_t>(alf->luma_coef, alf->luma_coef + L), s);
    ctx->d_alf_luma_clip.upload(std::vector<int16_t>(alf->luma_clip, alf->luma_clip + L), s);
    std::vector<int16_t> ch(alf->chroma_coef, alf->chroma_coef + 56);
    ch.insert(ch.end(), alf->chroma_clip, alf->chroma_clip + 56);
    ctx->d_alf_chroma.upload(ch, s);
    ctx->d_alf_cc.upload(std::vector<int16_t>(alf->cc_coef, alf->cc_coef + 64), s);
    std::vector<uint8_t> ctb(alf->ctb_en, alf->ctb_en + 3 * n);
    ctb.insert(ctb.end(), alf->ctb_alt, alf->ctb_alt + 3 * n);
    ctb.insert(ctb.end(), alf->cc_ctl, alf->cc_ctl + 2 * n);
    for (int i = 0; i < 3 * n; i++) if (ctb[3 * n + i] > 7) throw VvcrError(VVCR_E_ARG, "bad ALF chroma alternative");
    for (int i = 0; i < 2 * n; i++) if (ctb[6 * n + i] > 4) throw VvcrError(VVCR_E_ARG, "bad CC-ALF filter index");
    std::vector<int16_t> set(alf->ctb_filter_set, alf->ctb_filter_set + n);
    for (int v : set) if (v < 0 || v >= alf->num_luma_sets) throw VvcrError(VVCR_E_ARG, "bad ALF filter set index");
    ctx->d_alf_ctb.upload(ctb, s);
    ctx->d_alf_set.upload(set, s);
  }
  return VVCR_OK;
  API_END
}

static McParams make_mc_params(vvcr_ctx *ctx) {
  McParams P{};
  for (size_t s = 0; s < ctx->dpb.size() && s < 32; s++)
    for (int c = 0; c < 3; c++) P.ref[s][c] = ctx->dpb[s][c];
  for (int c = 0; c < 3; c++) P.out[c] = ctx->pred[c];
  P.pic_w = ctx->sp.width;
  P.pic_h = ctx->sp.height;
  P.bd = ctx->sp.bit_depth;
  P.ctu = 1 << ctx->sp.ctu_log2;
  return P;
}

namespace {
enum { ST_RESID, ST_INTER, ST_INTRA, ST_LMCS, ST_DBK, ST_SAO, ST_ALF };
struct StageTimer {
  vvcr_ctx *c;
  int k;
  StageTimer(vvcr_ctx *cc, int kk) : c(cc), k(kk) {
    c->stage_ran[k] = true;
    VVCR_CHECK_HIP(hipEventRecord(c->sev[k][0], c->stream));
  }
  ~StageTimer() { (void)hipEventRecord(c->sev[k][1], c->stream); }
};
}  // namespace

int vvcr_end_picture_stages(vvcr_ctx *ctx, uint32_t mask) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_end_picture without begin");
  build_work_lists(ctx->sp, ctx->pp, ctx->desc, ctx->wl);
  if (mask & VVCR_STAGE_DBK) plan_deblocking(ctx->sp, ctx->pp, ctx->desc, ctx->dbk);
  if (mask & VVCR_STAGE_INTRA) plan_intra(ctx->sp, ctx->pp, ctx->desc, ctx->intra);
  for (bool &r : ctx->stage_ran) r = false;
  hipStream_t s = ctx->stream;
  VVCR_CHECK_HIP(hipEventRecord(ctx->ev[0], s));
  if (mask & VVCR_STAGE_RESID) {
    StageTimer t(ctx, ST_RESID);
    for (int c = 0; c < 3; c++)
      VVCR_CHECK_HIP(hipMemsetAsync(ctx->resi[c].p, 0, (size_t)ctx->resi[c].stride * ctx->resi[c].h * 2, s));
    ctx->d_coef.upload(ctx->desc.coef, s);
    ctx->d_tb.upload(ctx->wl.tb, s);
    TbParams tp{};
    for (int c = 0; c < 3; c++) tp.out[c] = ctx->resi[c];
    tp.bd = ctx->sp.bit_depth;
    memcpy(tp.scan_off, ctx->scans.off, sizeof(tp.scan_off));
    memcpy(tp.lfnst_scan_off, ctx->scans.lfnst_off, sizeof(tp.lfnst_scan_off));
    launch_resid(tp, ctx->d_tb.p, (int)ctx->wl.tb.size(), ctx->d_coef.p, ctx->d_scans.p, s);
    VVCR_CHECK_HIP(hipGetLastError());
  }
  if (mask & VVCR_STAGE_INTER) {
    StageTimer t(ctx, ST_INTER);
    if (ctx->wl.n_unsupported_inter)
      throw VvcrError(VVCR_E_UNSUPPORTED, std::to_string(ctx->wl.n_unsupported_inter) + " inter CUs use tools not supported yet");
    const McParams mp = make_mc_params(ctx);
    ctx->d_mc_basic.upload(ctx->wl.mc_basic, s);
    launch_mc_basic(mp, ctx->d_mc_basic.p, (int)ctx->wl.mc_basic.size(), s);
    VVCR_CHECK_HIP(hipGetLastError());
    ctx->n_dmvr = ctx->wl.n_dmvr;
    ctx->d_dmvr.ensure(2 * (size_t)ctx->n_dmvr + 2);
    ctx->d_mc_bidir.upload(ctx->wl.mc_bidir, s);
    launch_mc_bidir(mp, ctx->d_mc_bidir.p, (int)ctx->wl.mc_bidir.size(), ctx->d_dmvr.p, s);
    VVCR_CHECK_HIP(hipGetLastError());
    ctx->d_aff_pu.upload(ctx->wl.aff_pu, s);
    ctx->d_aff_jobs.upload(ctx->wl.aff_jobs, s);
    launch_mc_affine(mp, ctx->d_aff_jobs.p, (int)ctx->wl.aff_jobs.size(), ctx->d_aff_pu.p, s);
    VVCR_CHECK_HIP(hipGetLastError());
  }
  // ---- reconstruction: inter CUs, then intra / CIIP steps level by level (vvcr_intra.h)
  if (mask & VVCR_STAGE_INTRA) {
    StageTimer t(ctx, ST_INTRA);
    IntraPlan &ip = ctx->intra;
    const size_t nu = ip.order[0].size();
    std::vector<int32_t> ord(ip.order[0]);
    ord.insert(ord.end(), ip.order[1].begin(), ip.order[1].end());
    ctx->d_order.upload(ord, s);
    ctx->d_tiles.upload(ip.inter_tiles, s);
    ctx->d_ijobs.upload(ip.jobs, s);
    IntraParams P{};
    for (int c = 0; c < 3; c++) { P.reco[c] = ctx->dpb[ctx->pp.slot][c]; P.pred[c] = ctx->pred[c]; P.resi[c] = ctx->resi[c]; }
    P.order[0] = ctx->d_order.p;
    P.order[1] = ctx->d_order.p + nu;
    P.W4 = ctx->sp.width / 4;
    P.bd = ctx->sp.bit_depth;
    P.ctu = 1 << ctx->sp.ctu_log2;
    launch_recon_inter(P, ctx->d_tiles.p, (int)ip.inter_tiles.size(), s);
    VVCR_CHECK_HIP(hipGetLastError());
    for (size_t L = 1; L + 1 < ip.level_start.size(); L++) {
      const int a = ip.level_start[L], b = ip.level_start[L + 1];
      launch_intra_level(P, ctx->d_ijobs.p + a, b - a, s);
    }
    VVCR_CHECK_HIP(hipGetLastError());
  }
  // ---- deblocking, in place on the picture slot: all vertical edges, then all horizontal edges
  if ((mask & VVCR_STAGE_DBK) && ctx->dbk.total()) {
    StageTimer t(ctx, ST_DBK);
    auto &all = ctx->dbk_all;
    all.clear();
    int counts[4];
    const std::vector<DbkSeg> *parts[4] = {&ctx->dbk.luma[0], &ctx->dbk.chroma[0], &ctx->dbk.luma[1], &ctx->dbk.chroma[1]};
    for (int k = 0; k < 4; k++) {
      counts[k] = (int)parts[k]->size();
      all.insert(all.end(), parts[k]->begin(), parts[k]->end());
    }
    ctx->d_dbk.upload(all, s);
    DbkParams dp{};
    for (int c = 0; c < 3; c++) dp.pl[c] = ctx->dpb[ctx->pp.slot][c];
    dp.bd = ctx->sp.bit_depth;
    dp.beta_offset_div2 = ctx->pp.dbk_beta_offset_div2;
    dp.tc_offset_div2 = ctx->pp.dbk_tc_offset_div2;
    launch_dbk(dp, ctx->d_dbk.p, counts, s);
  }
  // ---- SAO (DBK picture in the slot -> tmp) and ALF (-> slot)
  {
    const vvcr_pic_params &pp = ctx->pp;
    auto &A = ctx->dpb[pp.slot];
    const int ctu = 1 << ctx->sp.ctu_log2;
    const int wc = (ctx->sp.width + ctu - 1) / ctu, n = n_ctb(ctx->sp);
    bool inTmp = false;
    const bool alfOn = pp.alf_en[0] || pp.alf_en[1] || pp.alf_en[2];
    if ((mask & VVCR_STAGE_SAO) && (pp.sao_luma || pp.sao_chroma) && !ctx->have_sao)
      throw VvcrError(VVCR_E_STATE, "SAO is enabled for the picture but no SAO parameters were set");
    if ((mask & VVCR_STAGE_ALF) && alfOn && !ctx->have_alf)
      throw VvcrError(VVCR_E_STATE, "ALF is enabled for the picture but no ALF parameters were set");
    if ((mask & VVCR_STAGE_SAO) && ctx->have_sao && (pp.sao_luma || pp.sao_chroma)) {
      StageTimer t(ctx, ST_SAO);
      SaoParams sp{};
      for (int c = 0; c < 3; c++) { sp.src[c] = A[c]; sp.dst[c] = ctx->tmp[c]; }
      sp.sao = ctx->d_sao.p; sp.bd = ctx->sp.bit_depth; sp.ctu = ctu; sp.wc = wc;
      launch_sao(sp, s);
      VVCR_CHECK_HIP(hipGetLastError());
      inTmp = true;
    }
    if ((mask & VVCR_STAGE_ALF) && ctx->have_alf && alfOn) {
      StageTimer t(ctx, ST_ALF);
      AlfParams ap{};
      for (int c = 0; c < 3; c++) { ap.src[c] = inTmp ? ctx->tmp[c] : A[c]; ap.dst[c] = inTmp ? A[c] : ctx->tmp[c]; }
      ap.bd = ctx->sp.bit_depth; ap.ctu_log2 = ctx->sp.ctu_log2; ap.wc = wc; ap.nctb = n;
      ap.vb_luma = pp.alf_vb_luma; ap.vb_chroma = pp.alf_vb_chroma;
      for (int c = 0; c < 3; c++) ap.en[c] = pp.alf_en[c];
      ap.en[3] = pp.ccalf_en[0]; ap.en[4] = pp.ccalf_en[1];
      ap.luma_coef = ctx->d_alf_luma_coef.p; ap.luma_clip = ctx->d_alf_luma_clip.p;
      ap.chroma_coef = ctx->d_alf_chroma.p; ap.chroma_clip = ctx->d_alf_chroma.p + 56; ap.cc_coef = ctx->d_alf_cc.p;
      ap.ctb_en = ctx->d_alf_ctb.p; ap.ctb_alt = ctx->d_alf_ctb.p + 3 * n; ap.cc_ctl = ctx->d_alf_ctb.p + 6 * n;
      ap.ctb_set = ctx->d_alf_set.p;
      launch_alf(ap, s);
      VVCR_CHECK_HIP(hipGetLastError());
      inTmp = !inTmp;
    }
    if (inTmp)
      for (int c = 0; c < 3; c++)
        VVCR_CHECK_HIP(hipMemcpy2DAsync(A[c].p, A[c].stride * 2, ctx->tmp[c].p, ctx->tmp[c].stride * 2, A[c].w * 2, A[c].h,
                                        hipMemcpyDeviceToDevice, s));
  }
  VVCR_CHECK_HIP(hipEventRecord(ctx->ev[1], s));
  ctx->in_picture = false;
  return VVCR_OK;
  API_END
}

int vvcr_end_picture(vvcr_ctx *ctx) { return vvcr_end_picture_stages(ctx, VVCR_STAGE_ALL); }

int vvcr_sync(vvcr_ctx *ctx) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return VVCR_OK;
  API_END
}

int vvcr_last_stage_times(vvcr_ctx *ctx, float *ms, int32_t n) {
  if (!ctx || !ms) return VVCR_E_ARG;
  API_BEGIN
  VVCR_CHECK_HIP(hipEventSynchronize(ctx->ev[1]));
  float t = 0;
  VVCR_CHECK_HIP(hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]));
  if (n > 0) ms[0] = t;
  for (int k = 0; k < 7 && k + 1 < n; k++) {
    float v = 0;
    if (ctx->stage_ran[k]) VVCR_CHECK_HIP(hipEventElapsedTime(&v, ctx->sev[k][0], ctx->sev[k][1]));
    ms[k + 1] = v;
  }
  return VVCR_OK;
  API_END
}

static DPlane *select_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp) {
  if (comp < 0 || comp > 2) throw VvcrError(VVCR_E_ARG, "bad component");
  switch (buf) {
    case VVCR_BUF_RECO:
      if (slot < 0 || slot >= (int)ctx->dpb.size()) throw VvcrError(VVCR_E_ARG, "bad slot");
      return &ctx->dpb[slot][comp];
    case VVCR_BUF_PRED: return &ctx->pred[comp];
    case VVCR_BUF_RESI: return &ctx->resi[comp];
    default: throw VvcrError(VVCR_E_ARG, "bad buffer id");
  }
}

int vvcr_read_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, int16_t *dst, int32_t dst_stride) {
  if (!ctx || !dst) return VVCR_E_ARG;
  API_BEGIN
  DPlane *p = select_plane(ctx, buf, slot, comp);
  VVCR_CHECK_HIP(hipMemcpy2DAsync(dst, dst_stride * 2, p->p, p->stride * 2, p->w * 2, p->h, hipMemcpyDeviceToHost, ctx->stream));
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return VVCR_OK;
  API_END
}

int vvcr_write_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, const int16_t *src, int32_t src_stride) {
  if (!ctx || !src) return VVCR_E_ARG;
  API_BEGIN
  DPlane *p = select_plane(ctx, buf, slot, comp);
  VVCR_CHECK_HIP(hipMemcpy2DAsync(p->p, p->stride * 2, src, src_stride * 2, p->w * 2, p->h, hipMemcpyHostToDevice, ctx->stream));
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return VVCR_OK;
  API_END
}

int vvcr_read_picture(vvcr_ctx *ctx, int32_t slot, uint16_t *planes[3], const int32_t strides[3]) {
  if (!ctx || !planes || !strides) return VVCR_E_ARG;
  for (int c = 0; c < 3; c++) {
    int r = vvcr_read_plane(ctx, VVCR_BUF_RECO, slot, c, (int16_t *)planes[c], strides[c]);
    if (r) return r;
  }
  return VVCR_OK;
}

int vvcr_get_dmvr_deltas(vvcr_ctx *ctx, int32_t *out, int64_t n) {
  if (!ctx || (!out && n)) return VVCR_E_ARG;
  API_BEGIN
  if (n < 0) throw VvcrError(VVCR_E_ARG, "negative count");
  const int64_t m = std::min<int64_t>(n, ctx->n_dmvr);
  if (m > 0) {
    VVCR_CHECK_HIP(hipMemcpyAsync(out, ctx->d_dmvr.p, (size_t)m * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  }
  return (int)ctx->n_dmvr;
  API_END
}

}  // extern "C"
