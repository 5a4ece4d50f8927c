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
  DevVec<McJob> d_mc_basic;
  DevVec<TbJob> d_tb;
  DevVec<int32_t> d_coef;
  DevVec<uint16_t> d_scans;
  ScanTables scans;
  hipEvent_t ev[8] = {};
  float stage_ms[8] = {};
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

int vvcr_set_loop_filter_params(vvcr_ctx *ctx, const vvcr_sao *sao, const vvcr_alf *alf) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  (void)sao; (void)alf;
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
  return P;
}

int vvcr_end_picture_stages(vvcr_ctx *ctx, uint32_t mask) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_end_picture without begin");
  build_work_lists(ctx->sp, ctx->pp, ctx->desc, ctx->wl);
  hipStream_t s = ctx->stream;
  VVCR_CHECK_HIP(hipEventRecord(ctx->ev[0], s));
  if (mask & VVCR_STAGE_RESID) {
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
    ctx->d_mc_basic.upload(ctx->wl.mc_basic, s);
    launch_mc_basic(make_mc_params(ctx), ctx->d_mc_basic.p, (int)ctx->wl.mc_basic.size(), s);
    VVCR_CHECK_HIP(hipGetLastError());
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
  ctx->err = "DMVR delta readback not implemented yet";
  return VVCR_E_UNSUPPORTED;
}

}  // extern "C"
