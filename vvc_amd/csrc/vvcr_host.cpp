// vvcr_host.cpp — host producer logic: turns the picture's CU/PU/TU descriptors into GPU work lists.
// The decisions mirror the reference's dispatch in InterPrediction::motionCompensation
// (InterPrediction.cpp:1517-1660) so that every PU reaches the kernel that reproduces its prediction.
#include "vvcr_host.h"
#include "vvcr_tables.h"
#include <string>
#include <cstring>
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int MODE_INTER = 0;
constexpr int IMV_HPEL = 3;      // TypeDef.h:924
constexpr int MRG_TYPE_DEFAULT_N = 0, MRG_TYPE_SUBPU_ATMVP = 1;
constexpr int B_SLICE = 0;       // SliceType (TypeDef.h): B_SLICE=0, P_SLICE=1, I_SLICE=2

void fail(const std::string &m) { throw VvcrError(VVCR_E_ARG, m); }
int ilog2i(int v) { int r = 0; while ((1 << (r + 1)) <= v) r++; return r; }

// InterPrediction::xCheckIdenticalMotion (InterPrediction.cpp:248): bi-prediction from the same
// picture with the same MV is predicted as uni-prediction from list 0.
bool identical_motion(const vvcr_pic_params &pp, int interDir, int r0, int r1, int mv0x, int mv0y, int mv1x, int mv1y) {
  if (pp.slice_type != B_SLICE || pp.wp_b) return false;
  if (interDir != 3 || r0 < 0 || r1 < 0) return false;
  return pp.ref_poc[0][r0] == pp.ref_poc[1][r1] && mv0x == mv1x && mv0y == mv1y;
}

void push_tiles(bigbuf::vec<McJob> &out, int x0, int y0, int w, int h, McJob proto) {
  for (int y = 0; y < h; y += 16)
    for (int x = 0; x < w; x += 16) {
      McJob j = proto;
      j.x = (int16_t)(x0 + x);
      j.y = (int16_t)(y0 + y);
      j.w = (uint8_t)std::min(16, w - x);
      j.h = (uint8_t)std::min(16, h - y);
      out.push_back(j);
    }
}


// One plain MC unit (a PU, or an SbTMVP sub-block): 32x32 tiles for k_mc_tile when the PU is at least
// 32x32 (all VVC block sizes are powers of two, so the tiles cover it exactly), else <= 16x16 jobs.
void push_mc(WorkLists &wl, int x0, int y0, int w, int h, const McJob &proto, bool count = true) {
  if (count) wl.mc_alg += mc_alg_bytes(proto.flags, w, h);
  if (w >= 32 && h >= 32 && (x0 & 7) == 0) {
    for (int y = 0; y < h; y += 32)
      for (int x = 0; x < w; x += 32) {
        McJob j = proto;
        j.x = (int16_t)(x0 + x);
        j.y = (int16_t)(y0 + y);
        j.w = j.h = 32;
        wl.mc_tile.push_back(j);
      }
    return;
  }
  push_tiles(wl.mc_basic, x0, y0, w, h, proto);
}

static bool mc_bi(const McJob &j) { return (j.flags & (MC_L0 | MC_L1)) == (MC_L0 | MC_L1); }

// Jobs in descending (w, h), bi-predicted first within a size, stable: a counting sort over the 2 x 8 x 8
// power-of-two size buckets (a comparison sort of a picture's SbTMVP sub-blocks took milliseconds).
void sort_by_size_bi(bigbuf::vec<McJob> &v) {
  auto lg = [](int x) { return x > 0 && (x & (x - 1)) == 0 && x <= 128 ? __builtin_ctz(x) : -1; };
  int cnt[128] = {};
  for (const McJob &j : v) {
    const int a = lg(j.w), b = lg(j.h);
    if (a < 0 || b < 0) {   // (never for VVC block sizes) the comparison sort
      std::stable_sort(v.begin(), v.end(), [](const McJob &x, const McJob &y) {
        const int kx = x.w << 8 | x.h, ky = y.w << 8 | y.h;
        if (kx != ky) return kx > ky;
        return mc_bi(x) > mc_bi(y);
      });
      return;
    }
    cnt[127 - ((a * 8 + b) * 2 + (mc_bi(j) ? 1 : 0))]++;   // bucket order = the sort order
  }
  int pos[128], run = 0;
  for (int k = 0; k < 128; k++) { pos[k] = run; run += cnt[k]; }
  static thread_local bigbuf::raw<McJob> out;   // (a value-initialised vector would zero it first)
  if (out.size() < v.size()) out.alloc(v.size() + v.size() / 4, false);
  for (const McJob &j : v) out[pos[127 - ((lg(j.w) * 8 + lg(j.h)) * 2 + (mc_bi(j) ? 1 : 0))]++] = j;
  if (!v.empty()) std::memcpy((void *)v.data(), out.data(), v.size() * sizeof(McJob));
}

// A k_mc class table over job arrays laid out one after another from job index base (each flagged: its
// windows may leave the picture): one class per run of equal (w, h), its cell ranges padded to whole waves.
void build_mc_classes(McClassTable &ct, std::initializer_list<std::pair<const bigbuf::vec<McJob> *, bool>> lists, int base) {
  ct = McClassTable();
  int lc = 0, cc = 0;
  for (const auto &lv : lists) {
    const bigbuf::vec<McJob> &v = *lv.first;
    for (size_t i = 0; i < v.size();) {
      size_t e = i + 1;
      while (e < v.size() && v[e].w == v[i].w && v[e].h == v[i].h) e++;
      if (ct.n == MC_MAXCLS) fail("more plain-MC block classes than k_mc classes");
      const int k = ct.n++, w = v[i].w, h = v[i].h, n = (int)(e - i);
      ct.job0[k] = base + (int)i;
      ct.w[k] = w;
      ct.h[k] = h;
      ct.edge[k] = lv.second ? 1 : 0;
      ct.lcell0[k] = lc;
      ct.ccell0[k] = cc;
      lc += (n * mc_luma_cells(w, h)) + 63 & ~63;
      cc += (n * mc_chroma_cells(w, h)) + 63 & ~63;
      i = e;
    }
    base += (int)v.size();
  }
  ct.job0[ct.n] = base;
  ct.lcell0[ct.n] = lc;
  ct.ccell0[ct.n] = cc;
}

// Whether any reference window of a plain MC job, as k_mc's cells read it (aligned dword runs of 12 luma /
// 8 chroma samples from the even column at or before the first tap, 15 / 7 or 11 rows), may leave the
// picture (conservative): such jobs form classes of their own whose waves take the clamped path (rows
// and columns clamped: the edge-replicated margin, Picture.cpp:737); the others assume their windows
// inside, with no per-lane test and no edge code in their path.
bool mc_job_edge(const McJob &j, int W, int H) {
  for (int l = 0; l < 2; l++) {
    if (!(j.flags & (l ? MC_L1 : MC_L0))) continue;
    const int mvx = j.mv[l][0], mvy = j.mv[l][1];
    // luma: columns [x + (mvx >> 4) - 4, x + w + (mvx >> 4) + 8), rows [y + (mvy >> 4) - 3, y + h + (mvy >> 4) + 4]
    // (a block shorter than a cell still filters the cell's rows: heights rounded up to the cell)
    if (j.x + (mvx >> 4) - 4 < 0 || j.x + j.w + (mvx >> 4) + 8 > W) return true;
    if (j.y + (mvy >> 4) - 3 < 0 || j.y + std::max<int>(j.h, 8) + (mvy >> 4) + 6 > H) return true;
    // chroma (4:2:0)
    const int cx = j.x >> 1, cy = j.y >> 1, cw = std::max(2, j.w >> 1), ch = std::max(4, j.h >> 1);
    if (cx + (mvx >> 5) - 2 < 0 || cx + cw + (mvx >> 5) + 8 > (W >> 1)) return true;
    if (cy + (mvy >> 5) - 1 < 0 || cy + ch + (mvy >> 5) + 5 > (H >> 1)) return true;
  }
  return false;
}

McJob make_job(const vvcr_pic_params &pp, int interDir, int r0, int r1, int mv0x, int mv0y, int mv1x, int mv1y,
               int bcw, bool altHpel) {
  McJob j{};
  j.flags = MC_LUMA | MC_CHROMA;
  if (identical_motion(pp, interDir, r0, r1, mv0x, mv0y, mv1x, mv1y)) interDir = 1;
  if (interDir & 1) { j.flags |= MC_L0; j.slot[0] = (uint8_t)pp.ref_slot[0][r0]; j.mv[0][0] = (int16_t)mv0x; j.mv[0][1] = (int16_t)mv0y; }
  if (interDir & 2) { j.flags |= MC_L1; j.slot[1] = (uint8_t)pp.ref_slot[1][r1]; j.mv[1][0] = (int16_t)mv1x; j.mv[1][1] = (int16_t)mv1y; }
  if (altHpel) j.flags |= MC_ALT_HPEL;
  j.bcw = (int8_t)bcw;
  return j;
}

// Explicit weighted prediction replaces the default combine (InterPrediction::xPredInterBi,
// InterPrediction.cpp:633-678): P slices with the PPS weighted_pred flag (uni), B slices with
// weighted_bipred (uni, and bi unless DMVR / BDOF / a non-default BcwIdx of the CU take over; GEO never).
bool wp_applies(const vvcr_pic_params &pp, bool bi, int cu_bcw) {
  if (pp.slice_type == 1) return pp.wp_p != 0;
  if (pp.slice_type == B_SLICE && pp.wp_b) return !bi || cu_bcw == 2;
  return false;
}

void set_wp(const vvcr_pic_params &pp, McJob &j, int r0, int r1, int cu_bcw) {
  const bool bi = (j.flags & (MC_L0 | MC_L1)) == (MC_L0 | MC_L1);
  if (!wp_applies(pp, bi, cu_bcw)) return;
  j.flags |= MC_WP;
  j.ridx = (uint8_t)(((j.flags & MC_L0) ? r0 : 0) | ((j.flags & MC_L1) ? r1 : 0) << 4);
}

}  // namespace

// Algorithmic bytes of one plain MC unit: every reference window once per list (8-tap luma
// (w+7)(h+7), 4-tap chroma 2 (w/2+3)(h/2+3)) and the 4:2:0 prediction written once, 2 B per sample.
double mc_alg_bytes(uint16_t flags, int w, int h) {
  const int lists = ((flags & MC_L0) ? 1 : 0) + ((flags & MC_L1) ? 1 : 0);
  const double in = (double)(w + 7) * (h + 7) + 2.0 * (w / 2 + 3) * (h / 2 + 3);
  // + the residual read by a fused reconstruction (MC_RESI << comp); the output is written once either way
  return 2.0 * (lists * in + 1.5 * w * h) + resi_bytes(flags, w, h);
}

// Residual bytes a fused reconstruction reads for a w x h luma area with recon flags f (4:2:0).
double resi_bytes(int f, int w, int h) {
  return 2.0 * (((f & MC_RESI) ? w * h : 0) + ((f & MC_RESI_CB) ? w * h / 4 : 0) + ((f & MC_RESI_CR) ? w * h / 4 : 0));
}

// Which components of a CU have a coded residual (the coded-block rule of build_tb_jobs: a joint Cb-Cr TB
// writes both chroma components): MC_RESI << comp per component.
uint16_t cu_resi_flags(const PictureDescriptors &d, const vvcr_cu &c) {
  if (!c.rootcbf) return 0;
  uint16_t f = 0;
  for (int k = 0; k < c.ntu; k++) {
    const int ti = c.firsttu + k;
    if (ti < 0 || ti >= (int)d.tu.size()) break;
    const vvcr_tu &t = d.tu[ti];
    for (int comp = 0; comp < 3; comp++) {
      const int32_t *b = t.b[comp];
      if (b[2] <= 0) continue;
      bool written;
      if (comp > 0 && t.jccr) written = t.b[(t.jccr >> 1) ? 1 : 2][6] >= 0;
      else written = b[4] != 0 && b[6] >= 0;
      if (written) f |= (uint16_t)(MC_RESI << comp);
    }
  }
  return f;
}

void validate_descriptors(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d) {
  const int ncu = (int)d.cu.size(), npu = (int)d.pu.size(), ntu = (int)d.tu.size();
  for (int i = 0; i < ncu; i++) {
    const vvcr_cu &c = d.cu[i];
    // CUs lie inside the picture: VVC splits implicitly at the picture boundary (CU::divideSplit /
    // the implicit QT/BT of UnitPartitioner), and the sizes are multiples of 8 (vvcr_create)
    if (c.yvalid && (c.x < 0 || c.y < 0 || c.w <= 0 || c.h <= 0 || c.w > 128 || c.h > 128 || c.x + c.w > sp.width ||
                     c.y + c.h > sp.height))
      fail("CU " + std::to_string(i) + " has a bad luma area");
    if (c.cvalid && (c.cx < 0 || c.cy < 0 || c.cw <= 0 || c.ch <= 0 || c.cw > 64 || c.ch > 64 || c.cx + c.cw > sp.width / 2 ||
                     c.cy + c.ch > sp.height / 2))
      fail("CU " + std::to_string(i) + " has a bad chroma area");
    if (!c.yvalid && !c.cvalid) fail("CU " + std::to_string(i) + " has no component");
    if (c.npu > 0 && (c.firstpu < 0 || c.firstpu + c.npu > npu)) fail("CU " + std::to_string(i) + " PU range");
    if (c.ntu > 0 && (c.firsttu < 0 || c.firsttu + c.ntu > ntu)) fail("CU " + std::to_string(i) + " TU range");
  }
  for (int i = 0; i < npu; i++) {
    const vvcr_pu &p = d.pu[i];
    if (p.cu < 0 || p.cu >= ncu) fail("PU " + std::to_string(i) + " CU index");
    const vvcr_cu &c = d.cu[p.cu];
    if (p.w > 0 && (p.x < 0 || p.y < 0 || p.x + p.w > sp.width || p.y + p.h > sp.height || p.w > 128 || p.h > 128))
      fail("PU " + std::to_string(i) + " area");
    if (c.predmode == MODE_INTER) {
      if ((p.interdir & 1) && (p.ref0 < 0 || p.ref0 >= pp.num_ref[0])) fail("PU " + std::to_string(i) + " ref0");
      if ((p.interdir & 2) && (p.ref1 < 0 || p.ref1 >= pp.num_ref[1])) fail("PU " + std::to_string(i) + " ref1");
    }
  }
  const bool packed = !d.coef_box.empty();
  if (packed && d.coef_box.size() < 3 * (size_t)ntu) fail("packed coefficient boxes");
  for (int i = 0; i < ntu; i++) {
    const vvcr_tu &t = d.tu[i];
    if (t.cu < 0 || t.cu >= ncu) fail("TU " + std::to_string(i) + " CU index");
    for (int c = 0; c < 3; c++) {
      const int32_t *b = t.b[c];
      if (b[2] <= 0) continue;
      const int pw = c ? sp.width / 2 : sp.width, ph = c ? sp.height / 2 : sp.height;
      const int maxs = b[6] >= 0 ? 64 : 128;   // coded TBs are <= 64 (maxTbSize); residual-free TUs span the CU
      // every block lies inside its plane: the kernels store residual / reconstruction rows unclipped
      if (b[0] < 0 || b[1] < 0 || b[0] + b[2] > pw || b[1] + b[3] > ph || b[2] > maxs || b[3] > maxs) fail("TU " + std::to_string(i) + " area");
      if (!packed && b[6] >= 0 && (int64_t)b[6] + (int64_t)b[2] * b[3] > (int64_t)d.coef.size()) fail("TU " + std::to_string(i) + " coefficient range");
      if (packed && b[6] >= 0) {
        const int rows = d.coef_box[3 * (size_t)i + c] & 255, cols = d.coef_box[3 * (size_t)i + c] >> 8;
        if (rows > b[3] || cols > b[2] || (int64_t)b[6] + (int64_t)rows * cols > (int64_t)d.coef.size()) fail("TU " + std::to_string(i) + " coefficient range");
      }
    }
  }
  if (!d.motion.empty() && d.motion.size() != (size_t)(sp.width / 4) * (sp.height / 4)) fail("motion field size");
  // picture partitioning: tiles with loop filtering across their edges, one or more slices with loop
  // filtering across theirs (the deblocking / SAO / ALF planners do not stop at tile or slice edges)
  const int ctu = 1 << sp.ctu_log2, wc = (sp.width + ctu - 1) / ctu, hc = (sp.height + ctu - 1) / ctu;
  for (int k = 0; k < 2; k++) {
    const int n = k ? pp.num_tile_rows : pp.num_tile_cols, lim = k ? hc : wc;
    const int32_t *bd = k ? pp.tile_row_bd : pp.tile_col_bd;
    if (n < 0 || n > VVCR_MAX_TILE_LINES) fail("tile count");
    if (n > 0 && (bd[0] != 0 || bd[n] != lim)) fail("tile boundaries do not span the picture");
    for (int t = 0; t < n; t++) if (bd[t + 1] <= bd[t]) fail("tile boundaries not increasing");
  }
  // (tiles / slices without loop filtering across their boundaries: lf_ctb_neighbours; the shard path needs
  // the filters across its tile rows)
  if (pp.shard_y1 > 0 && !pp.lf_across_tiles && (pp.num_tile_cols > 1 || pp.num_tile_rows > 1))
    throw VvcrError(VVCR_E_UNSUPPORTED, "spatial shards of a picture without loop filtering across tiles");
  // (entropy_sync, WPP: a property of the CABAC pass only; the reconstruction is the same)
  if (pp.shard_y1 > 0) {
    // a shard is a run of whole tile rows: intra prediction and CABAC stop at its edges, so its
    // reconstruction needs nothing from the other shards (the loop filters do: VVCR_LF_HALO)
    auto on_tile_row = [&](int y) {
      if (y == 0 || y == sp.height) return true;
      if (y % ctu) return false;
      for (int t = 0; t <= pp.num_tile_rows; t++) if (pp.tile_row_bd[t] * ctu == y) return true;
      return false;
    };
    if (pp.shard_y0 < 0 || pp.shard_y0 >= pp.shard_y1 || pp.shard_y1 > sp.height || !on_tile_row(pp.shard_y0) ||
        !on_tile_row(pp.shard_y1))
      fail("shard rows must be a run of whole tile rows");
  }
}

void build_tb_jobs(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, bigbuf::vec<TbJob> &out,
                   bigbuf::vec<int32_t> &packed);
void build_zero_jobs(const vvcr_pic_params &pp, const PictureDescriptors &d, bigbuf::vec<TbJob> &out);

namespace {

// initGeoTemplate (Rom.cpp:760-777): split mode -> (angle, distance)
struct GeoModes {
  int16_t angle[64], dist[64];
  GeoModes() {
    static const int8_t a2m[32] = {0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1, 0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1};
    int m = 0;
    for (int a = 0; a < 32; a++)
      for (int d = 0; d < 4; d++) {
        if ((d == 0 && a >= 16) || ((d == 2 || d == 0) && (a2m[a] == 0 || a2m[a] == 5)) || a2m[a] == -1) continue;
        if (m < 64) { angle[m] = (int16_t)a; dist[m] = (int16_t)d; }
        m++;
      }
  }
};
const GeoModes &geo_modes() {
  static const GeoModes g;
  return g;
}

// InterPrediction::isSubblockVectorSpreadOverLimit (InterPrediction.cpp:850)
bool spread_over_limit(int a, int b, int c, int d, int predType) {
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

// affine model of one list (xPredAffineBlk :917-960)
AffList affine_list(const vvcr_pic_params &pp, const vvcr_cu &c, const vvcr_pu &p, int l) {
  AffList A{};
  const int ref = l ? p.ref1 : p.ref0;
  A.present = 1;
  A.slot = pp.ref_slot[l][ref];
  A.ridx = ref;
  const int *mv = &p.aff[l * 6];   // LT, RT, LB
  const int iBit = 7;
  const int lw = ilog2i(p.w), lh = ilog2i(p.h);
  A.dhx = (mv[2] - mv[0]) << (iBit - lw);
  A.dhy = (mv[3] - mv[1]) << (iBit - lw);
  if (c.affinetype == 1) {   // AFFINEMODEL_6PARAM
    A.dvx = (mv[4] - mv[0]) << (iBit - lh);
    A.dvy = (mv[5] - mv[1]) << (iBit - lh);
  } else {
    A.dvx = -A.dhy;
    A.dvy = A.dhx;
  }
  A.mvx = mv[0] * (1 << iBit);
  A.mvy = mv[1] * (1 << iBit);
  A.spread = spread_over_limit(A.dhx, A.dhy, A.dvx, A.dvy, p.interdir);
  const bool same = c.affinetype == 1 ? (mv[0] == mv[2] && mv[1] == mv[3] && mv[0] == mv[4] && mv[1] == mv[5])
                                      : (mv[0] == mv[2] && mv[1] == mv[3]);
  A.prof = pp.prof_enabled && !same && !A.spread;
  return A;
}

}  // namespace

void build_work_lists(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, WorkLists &wl,
                      bool fuse) {
  static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;   // diagnostics: phase times to stderr
  auto tp = std::chrono::steady_clock::now();
  auto mark = [&](const char *n) {
    if (!prof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "    wl %-8s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t - tp).count());
    tp = t;
  };
  wl.clear();
  build_tb_jobs(sp, pp, d, wl.tb, wl.coef);
  mark("tb");
  if (fuse) {   // the reconstruction stages run together: the residual reads are known, zero only those
    build_zero_jobs(pp, d, wl.tb);
    wl.zero_filled = true;
  }
  mark("zero");
  // small blocks first (64-lane workgroups), then the large ones (256 lanes)
  wl.tb_small = (int)(std::stable_partition(wl.tb.begin(), wl.tb.end(), [](const TbJob &j) { return j.w * j.h <= 256; }) - wl.tb.begin());
  const int W4 = sp.width / 4;
  bigbuf::vec<int> geo_of(d.cu.size(), -1);
  for (size_t g = 0; g < d.geo.size(); g++)
    if (d.geo[g].cu >= 0 && d.geo[g].cu < (int)d.cu.size()) geo_of[d.geo[g].cu] = (int)g;
  int ry0 = 1 << 30, ry1 = -(1 << 30);   // reference rows read (luma), with filter / DMVR / BDOF margins
  auto reach = [&](int y, int h, int mvy) {
    ry0 = std::min(ry0, y + (mvy >> 4) - 8);
    ry1 = std::max(ry1, y + h + (mvy >> 4) + 9);
  };
  for (size_t ci = 0; ci < d.cu.size(); ci++) {
    const vvcr_cu &c = d.cu[ci];
    if (c.predmode != MODE_INTER || !c.yvalid || !in_shard(pp, c)) continue;
    const uint16_t recon = (fuse && fused_inter_cu(pp, d, c)) ? (uint16_t)(MC_RECON | cu_resi_flags(d, c)) : 0;
    if (c.geo) {
      // motionCompensationGeo (InterPrediction.cpp:1749): two uni candidates at 14 bits, blended
      const vvcr_pu &p = d.pu[c.firstpu];
      if (geo_of[ci] < 0 || p.geodir < 0 || p.geodir >= 64) { wl.n_unsupported_inter++; continue; }
      const vvcr_geo &g = d.geo[geo_of[ci]];
      McJob j{};
      j.flags = MC_L0 | MC_L1 | MC_LUMA | MC_CHROMA | MC_GEO | recon;
      for (int k = 0; k < 2; k++) {
        const int l = g.cand[k][1], r = g.cand[k][2];
        if (l < 0 || l > 1 || r < 0 || r >= pp.num_ref[l]) fail("GEO candidate reference");
        j.slot[k] = (uint8_t)pp.ref_slot[l][r];
        j.mv[k][0] = (int16_t)g.cand[k][3];
        j.mv[k][1] = (int16_t)g.cand[k][4];
      }
      const GeoModes &gm = geo_modes();
      const int angle = gm.angle[p.geodir], dist = gm.dist[p.geodir];
      int offX = (224 - p.w) >> 1, offY = (224 - p.h) >> 1;   // InitGeoTemplate weight offsets (Rom.cpp:807-826)
      if (dist > 0) {
        if (angle % 16 == 8 || (angle % 16 != 0 && p.h >= p.w)) offY += angle < 16 ? ((dist * p.h) >> 3) : -((dist * p.h) >> 3);
        else offX += angle < 16 ? ((dist * p.w) >> 3) : -((dist * p.w) >> 3);
      }
      j.aux = angle | offX << 8 | offY << 16;
      j.pu_x = (int16_t)p.x;
      j.pu_y = (int16_t)p.y;
      j.bcw = 2;
      push_mc(wl, p.x, p.y, p.w, p.h, j);
      continue;
    }
    for (int k = 0; k < c.npu; k++) {
      const vvcr_pu &p = d.pu[c.firstpu + k];
      const bool alt = c.imv == IMV_HPEL;
      const int bcw = p.ciip ? 2 : c.bcw;   // BCW is not applied to CIIP (InterPrediction.cpp:1397)
      if (p.mrgtype == MRG_TYPE_SUBPU_ATMVP) {
        // xSubPuMC (InterPrediction.cpp:283-360): 8x8 sub-blocks with their own motion, no BDOF / DMVR
        // (SbTMVP candidates of the sub-block merge list also carry cu.affine; the merge type decides).
        // The reference predicts each run of sub-blocks with the same motion along the PU's longer side as
        // one block (:307-345), so the algorithmic bytes count per run. The jobs: VVCR_SBT_JOIN 3 (default)
        // a run that is a whole line of the PU is one job, other runs 8x8 jobs (a PU's jobs then stay in
        // one or two k_mc size classes, next to each other in the launch: runs cut into jobs of several
        // sizes scatter over the classes and lose L2 reuse, 14 % more HBM reads and +0.7 / +1.3 us per
        // 4K QP27 / QP32 picture, profiles/r05_sbt_join*); 0 every sub-block a job, 1 a job per run,
        // 2 runs cut into power-of-two lengths.
        static const int join = [] { const char *e = getenv("VVCR_SBT_JOIN"); return e ? atoi(e) : 3; }();
        const bool ver = p.h > p.w;
        const int fe = ver ? p.w : p.h, se = ver ? p.h : p.w;
        auto mot = [&](int a, int b) -> const MotionRec & {   // the sub-block at (first, second) offsets
          const int x = ver ? a : b, y = ver ? b : a;
          return d.motion[(size_t)((p.y + y) >> 2) * W4 + ((p.x + x) >> 2)];
        };
        for (int a = 0; a < fe; a += 8)
          for (int b = 0; b < se;) {
            const MotionRec &m = mot(a, b);
            int run = 8;
            while (b + run < se && std::memcmp(&mot(a, b + run), &m, sizeof(MotionRec)) == 0) run += 8;
            McJob j = make_job(pp, m.inter_dir, m.ref0, m.ref1, m.mv0x, m.mv0y, m.mv1x, m.mv1y, bcw, alt);   // BCW of the CU (xWeightedAverage reads pu.cu->BcwIdx)
            set_wp(pp, j, m.ref0, m.ref1, c.bcw);
            j.flags |= recon;
            const int fw = std::min(8, fe - a);   // the run's extent across the line
            wl.mc_alg += ver ? mc_alg_bytes(j.flags, fw, run) : mc_alg_bytes(j.flags, run, fw);
            for (int o = 0; o < run;) {
              int len = 8;
              if (join == 1 || (join == 3 && b == 0 && run == se)) len = run;
              else if (join == 2) len = 1 << (31 - __builtin_clz(run - o));
              const int x = ver ? a : b + o, y = ver ? b + o : a;
              push_mc(wl, p.x + x, p.y + y, ver ? fw : len, ver ? len : fw, j, false);
              o += len;
            }
            b += run;
          }
        continue;
      }
      if (c.affine) {
        AffPu U{};
        U.x = (int16_t)p.x; U.y = (int16_t)p.y; U.w = (int16_t)p.w; U.h = (int16_t)p.h;
        U.bcw = bcw;
        if (p.interdir & 1) U.l[0] = affine_list(pp, c, p, 0);
        if (p.interdir & 2) U.l[1] = affine_list(pp, c, p, 1);
        U.wp = wp_applies(pp, p.interdir == 3, c.bcw) ? 1 : 0;
        U.recon = (int16_t)recon;
        for (int l = 0; l < 2; l++) {   // the sub-block MVs lie within the model's values at the PU corners
          if (!U.l[l].present) continue;
          const AffList &A = U.l[l];
          for (int cy = 0; cy <= 1; cy++)
            for (int cx = 0; cx <= 1; cx++) reach(p.y + cy * p.h, 0, (A.mvy + A.dhy * cx * p.w + A.dvy * cy * p.h) >> 7);
          reach(p.y, p.h, A.mvy >> 7);
        }
        const int idx = (int)wl.aff_pu.size();
        wl.aff_pu.push_back(U);
        for (int y = 0; y < p.h; y += 16)
          for (int x = 0; x < p.w; x += 16) {
            AffJob j{};
            j.x = (int16_t)(p.x + x); j.y = (int16_t)(p.y + y);
            j.w = (uint8_t)std::min(16, p.w - x); j.h = (uint8_t)std::min(16, p.h - y);
            j.pu = idx;
            wl.aff_jobs.push_back(j);
          }
        continue;
      }
      if (p.dmvr || p.bdof) {
        McJob j = make_job(pp, p.interdir, p.ref0, p.ref1, p.mv0x, p.mv0y, p.mv1x, p.mv1y, bcw, alt);
        if ((j.flags & (MC_L0 | MC_L1)) != (MC_L0 | MC_L1)) fail("DMVR/BDOF PU is not bi-predicted");
        if (p.w % 8 || p.h % 8) fail("DMVR/BDOF PU size is not a multiple of 8");   // k_mc_bidir: 8 or 16 per side
        if (p.bdof) j.flags |= MC_BDOF;
        j.flags |= recon;
        if (p.dmvr) {
          // xProcessDMVR sub-blocks (InterPrediction.cpp:2162-2166), raster order = delta order
          j.flags |= MC_DMVR;
          const int dx = std::min(16, p.w), dy = std::min(16, p.h);
          for (int y = 0; y < p.h; y += dy)
            for (int x = 0; x < p.w; x += dx) {
              McJob t = j;
              t.x = (int16_t)(p.x + x); t.y = (int16_t)(p.y + y);
              t.w = (uint8_t)dx; t.h = (uint8_t)dy;
              t.aux = wl.n_dmvr++;
              wl.mc_bidir.push_back(t);
            }
        } else {
          j.aux = -1;
          push_tiles(wl.mc_bidir, p.x, p.y, p.w, p.h, j);   // xSubPuBio 16x16 split (InterPrediction.cpp:420)
        }
        continue;
      }
      McJob j = make_job(pp, p.interdir, p.ref0, p.ref1, p.mv0x, p.mv0y, p.mv1x, p.mv1y, bcw, alt);
      set_wp(pp, j, p.ref0, p.ref1, c.bcw);   // the CU's BcwIdx, not the CIIP-cleared one (:664 reads pu.cu->BcwIdx)
      j.flags |= recon;
      push_mc(wl, p.x, p.y, p.w, p.h, j);
    }
  }
  mark("cus");
  // bi-predicted work first (about twice the work of a uni job): the long jobs start in the first
  // dispatch rounds instead of forming the launch's tail
  auto bi_first = [](bigbuf::vec<McJob> &v) {
    std::stable_partition(v.begin(), v.end(), [](const McJob &j) { return (j.flags & (MC_L0 | MC_L1)) == (MC_L0 | MC_L1); });
  };
  bi_first(wl.mc_tile);
  // the small blocks by size class (k_mc cell classes), bi-predicted first within a class: a wave's lanes
  // then share one size and mostly one prediction direction
  sort_by_size_bi(wl.mc_basic);
  // jobs whose windows may leave the picture: to the edge list (same order rules), the rest stay
  auto split_edge = [&](bigbuf::vec<McJob> &v) {   // stable, in place (std::stable_partition allocates)
    size_t k = 0;
    for (size_t i = 0; i < v.size(); i++) {
      if (mc_job_edge(v[i], sp.width, sp.height)) wl.mc_edge.push_back(v[i]);
      else v[k++] = v[i];
    }
    v.resize(k);
  };
  split_edge(wl.mc_tile);
  split_edge(wl.mc_basic);
  sort_by_size_bi(wl.mc_edge);
  // the edge classes first: their waves (longer, per-row clamped gathers) start in the first round
  mark("sorts");
  build_mc_classes(wl.mc_ct, {{&wl.mc_edge, true}, {&wl.mc_tile, false}, {&wl.mc_basic, false}}, 0);
  mark("classes");
  {   // bi-predicted affine tiles first, stable (in place: std::stable_partition allocates)
    static thread_local bigbuf::raw<AffJob> uni;
    if (uni.size() < wl.aff_jobs.size()) uni.alloc(wl.aff_jobs.size() + wl.aff_jobs.size() / 4, false);
    size_t k = 0, u = 0;
    for (size_t i = 0; i < wl.aff_jobs.size(); i++) {
      const AffPu &U = wl.aff_pu[wl.aff_jobs[i].pu];
      if (U.l[0].present && U.l[1].present) wl.aff_jobs[k++] = wl.aff_jobs[i];
      else uni[u++] = wl.aff_jobs[i];
    }
    if (u) std::memcpy((void *)(wl.aff_jobs.data() + k), uni.data(), u * sizeof(AffJob));
  }
  mark("affine");
  for (const bigbuf::vec<McJob> *v : {&wl.mc_tile, &wl.mc_basic, &wl.mc_edge, &wl.mc_bidir})
    for (const McJob &j : *v)
      for (int l = 0; l < 2; l++)
        if (j.flags & (l ? MC_L1 : MC_L0)) reach(j.y, j.h, j.mv[l][1]);
  if (ry0 <= ry1) {
    wl.ref_y0 = std::max(0, ry0);
    wl.ref_y1 = std::min(sp.height, ry1);
  }
  mark("reach");
}

// ------------------------------------------------------------------------------------------------
// scans
// ------------------------------------------------------------------------------------------------
namespace {
void diag(int bw, int bh, std::vector<int> &xs, std::vector<int> &ys) {
  xs.resize(bw * bh); ys.resize(bw * bh);
  int line = 0, col = 0;
  for (int i = 0; i < bw * bh; i++) {
    xs[i] = col; ys[i] = line;
    if (col == bw - 1 || line == 0) {
      line += col + 1; col = 0;
      if (line >= bh) { col += line - (bh - 1); line = bh - 1; }
    } else { col++; line--; }
  }
}
int ilog2(int v) { int r = 0; while ((1 << (r + 1)) <= v) r++; return r; }
}  // namespace

void build_scan_tables(ScanTables &st) {
  st.data.clear();
  std::vector<int> gx, gy, cx, cy;
  for (int lw = 0; lw < 7; lw++)
    for (int lh = 0; lh < 7; lh++) {
      const int w = 1 << lw, h = 1 << lh;
      const int gw = 1 << kLog2SbbSize[lw][lh][0], gh = 1 << kLog2SbbSize[lw][lh][1];
      const int wg = std::min(w, 32) / gw, hg = std::min(h, 32) / gh;
      st.off[lw][lh] = (int32_t)st.data.size();
      diag(wg, hg, gx, gy);
      diag(gw, gh, cx, cy);
      for (size_t g = 0; g < gx.size(); g++)
        for (size_t c = 0; c < cx.size(); c++) st.data.push_back((uint16_t)((gy[g] * gh + cy[c]) * w + gx[g] * gw + cx[c]));
    }
  diag(2, 2, gx, gy);
  diag(4, 4, cx, cy);
  for (int lw = 0; lw < 7; lw++) {
    st.lfnst_off[lw] = (int32_t)st.data.size();
    const int w = 1 << lw;
    for (int g = 0; g < 4; g++)
      for (int e = 0; e < 16; e++) st.data.push_back((uint16_t)((gy[g] * 4 + cy[e]) * w + gx[g] * 4 + cx[e]));
  }
}

// ------------------------------------------------------------------------------------------------
// transform blocks: the decisions of TrQuant::invTransformNxN's callers (DecCu.cpp:161-265, 775-850)
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int NUM_LUMA_MODE = 67, NUM_EXT_LUMA_MODE = 28, VDIA_IDX = 66, DIA_IDX = 34;

int wide_angle(int mode, int w, int h) {        // PU::getWideAngIntraMode (UnitTools.cpp:651)
  if (mode < 2) return mode;
  static const int modeShift[] = {0, 6, 10, 12, 14, 15};
  const int d = std::abs(ilog2(w) - ilog2(h));
  int m = mode;
  if (w > h && mode < 2 + modeShift[d]) m += VDIA_IDX - 1;
  else if (h > w && m > VDIA_IDX - modeShift[d]) m -= VDIA_IDX + 1;
  return m;
}
int lfnst_mode_of(int wam) {                    // TrQuant::getLFNSTIntraMode (TrQuant.cpp:283)
  if (wam < 0) return wam + (NUM_EXT_LUMA_MODE >> 1) + NUM_LUMA_MODE;
  if (wam >= NUM_LUMA_MODE) return wam + (NUM_EXT_LUMA_MODE >> 1);
  return wam;
}
bool lfnst_transpose(int m) {                   // TrQuant::getTransposeFlag (TrQuant.cpp:300)
  return (m >= NUM_LUMA_MODE && m >= NUM_LUMA_MODE + (NUM_EXT_LUMA_MODE >> 1)) || (m < NUM_LUMA_MODE && m > DIA_IDX);
}
// TrQuant::getTrTypes (TrQuant.cpp:668)
void tr_types(const vvcr_pic_params &pp, const vvcr_cu &cu, int comp, int w, int h, int mts, int tuLumaW, int tuLumaH, int &trh, int &trv) {
  const bool isIntra = cu.predmode == 1, isInter = cu.predmode == 0, luma = comp == 0;
  const bool explicitMTS = (isIntra ? pp.mts_intra : (pp.mts_inter && isInter)) && luma;
  const bool implicitMTS = isIntra && pp.implicit_mts && luma && cu.lfnst == 0 && cu.mip == 0;
  const bool isISP = isIntra && cu.isp && luma;
  const bool isSBT = isInter && cu.sbtinfo && luma;
  trh = trv = TR_DCT2;
  if (isISP && cu.lfnst) return;
  if (!pp.use_mts) return;
  if (implicitMTS || isISP) {
    if (w >= 4 && w <= 16) trh = TR_DST7;
    if (h >= 4 && h <= 16) trv = TR_DST7;
    return;
  }
  if (isSBT) {
    const int idx = cu.sbtinfo & 0xf, pos = (cu.sbtinfo >> 4) & 3;
    if (idx == 1 || idx == 3) {
      if (tuLumaH > 32) return;
      if (pos == 0) { trh = TR_DCT8; trv = TR_DST7; } else { trh = TR_DST7; trv = TR_DST7; }
    } else {
      if (tuLumaW > 32) return;
      if (pos == 0) { trh = TR_DST7; trv = TR_DCT8; } else { trh = TR_DST7; trv = TR_DST7; }
    }
    return;
  }
  if (explicitMTS && mts > 1) {
    trh = ((mts - 2) & 1) ? TR_DCT8 : TR_DST7;
    trv = ((mts - 2) >> 1) ? TR_DCT8 : TR_DST7;
  }
}
}  // namespace

void build_tb_jobs(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, bigbuf::vec<TbJob> &out,
                   bigbuf::vec<int32_t> &packed) {
  out.clear();
  packed.clear();
  const bool prepacked = !d.coef_box.empty();   // the producer's pool is already packed: uploaded as it is
  const int W4 = sp.width / 4, H4 = sp.height / 4;
  bigbuf::vec<int> lmap;   // luma PU per 4x4, for co-located luma modes (PU::getCoLocatedIntraLumaMode)
  bool haveMap = false;
  static const int kIct[2][4] = {{0, 3, 1, 2}, {0, -3, -1, -2}};
  for (size_t ti = 0; ti < d.tu.size(); ti++) {
    const vvcr_tu &t = d.tu[ti];
    const vvcr_cu &cu = d.cu[t.cu];
    if (!in_shard(pp, cu)) continue;
    const bool sepTree = cu.treetype != 0 || pp.dual_tree;
    for (int comp = 0; comp < 3; comp++) {
      const int32_t *b = t.b[comp];
      if (b[2] <= 0) continue;
      if (comp == 2 && t.jccr) continue;
      int src = comp;
      if (comp == 1 && t.jccr) src = (t.jccr >> 1) ? 1 : 2;
      const int32_t *bs = t.b[src];
      const bool coded = (comp == 1 && t.jccr) ? true : b[4] != 0;
      if (!coded || bs[6] < 0) continue;      // residual planes are cleared per picture
      const int w = bs[2], h = bs[3];
      TbJob j{};
      j.x = (int16_t)bs[0]; j.y = (int16_t)bs[1]; j.w = (uint8_t)w; j.h = (uint8_t)h;
      j.comp = (uint8_t)src;
      const bool ts = bs[5] == 1;
      j.qp = (uint8_t)(ts ? bs[8] : bs[7]);
      j.coef = bs[6];
      int trh, trv;
      tr_types(pp, cu, src, w, h, bs[5], t.b[0][2], t.b[0][3], trh, trv);
      j.trh = (uint8_t)trh; j.trv = (uint8_t)trv;
      if (ts) j.flags |= TB_TS;
      if (pp.dep_quant && !ts) j.flags |= TB_DQ;
      const int bdpcm = src == 0 ? cu.bdpcm : cu.bdpcmc;
      j.flags |= (uint8_t)((bdpcm & 3) << TB_BDPCM_SHIFT);
      int skipW = (trh != TR_DCT2 && w == 32) ? 16 : (w > 32 ? w - 32 : 0);
      int skipH = (trv != TR_DCT2 && h == 32) ? 16 : (h > 32 ? h - 32 : 0);
      if (pp.lfnst_enabled && cu.lfnst) {
        if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
        else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
        if (!ts && (sepTree || src == 0) && cu.lfnst < 3) {
          const vvcr_pu &p = d.pu[cu.firstpu];
          int mode = src == 0 ? p.fidir_l : p.fidir_c;
          if (src > 0 && p.idir_c >= 67 && p.idir_c <= 69) {
            // the luma CU map of the producer when it hands one over (an intra luma CU has one PU), else a
            // PU map built here once per picture
            const bool cmap = d.cu_map[0].size() == (size_t)W4 * H4;
            if (!haveMap && !cmap) {
              lmap.assign((size_t)W4 * H4, -1);
              for (size_t i = 0; i < d.pu.size(); i++) {
                const vvcr_pu &q = d.pu[i];
                if (q.w <= 0 || q.chtype != 0) continue;
                for (int y = q.y >> 2; y < (q.y + q.h) >> 2 && y < H4; y++)
                  for (int x = q.x >> 2; x < (q.x + q.w) >> 2 && x < W4; x++) lmap[(size_t)y * W4 + x] = (int)i;
              }
              haveMap = true;
            }
            const int lx = cu.cx * 2, ly = cu.cy * 2, lww = cu.cw * 2, lhh = cu.ch * 2;
            const int rx = sepTree ? lx + (lww >> 1) : lx, ry = sepTree ? ly + (lhh >> 1) : ly;
            int li;
            if (cmap) {
              const int lc = d.cu_map[0][(size_t)(ry >> 2) * W4 + (rx >> 2)];
              li = lc >= 0 ? d.cu[lc].firstpu : -1;
            } else {
              li = lmap[(size_t)(ry >> 2) * W4 + (rx >> 2)];
            }
            if (li < 0) throw VvcrError(VVCR_E_ARG, "no co-located luma PU for CCLM chroma TU");
            const vvcr_pu &lp = d.pu[li];
            mode = d.cu[lp.cu].mip ? 0 : lp.idir_l;
          }
          if (src == 0 && cu.mip) mode = 0;
          const int m = lfnst_mode_of(wide_angle(mode, w, h));
          if (m < 0 || m >= 95) throw VvcrError(VVCR_E_ARG, "LFNST mode out of range");
          j.lfnst_idx = (uint8_t)cu.lfnst;
          j.lfnst_mode = (uint8_t)m;   // intra mode; the kernel maps it through g_lfnstLut
          j.flags |= TB_LFNST_APPLY;
          if (lfnst_transpose(m)) j.flags |= TB_LFNST_TRANSPOSE;
        }
      }
      j.skip_w = (uint8_t)skipW; j.skip_h = (uint8_t)skipH;
      if (comp == 1 && t.jccr) j.ict = (int8_t)kIct[pp.joint_cbcr_sign ? 1 : 0][t.jccr];
      // bounding box of the non-zero levels: the kernel's passes skip the all-zero rows / columns
      // (dequantisation maps 0 to 0; LFNST widens it to its output area; TS / BDPCM use the whole block)
      if (prepacked) {   // the box as parsed; LFNST widens the processed box past the stored one
        const int SR = d.coef_box[3 * ti + src] & 255, SC = d.coef_box[3 * ti + src] >> 8;
        int R = SR, C = SC;
        if (ts) { R = h; C = w; }
        else if (j.flags & TB_LFNST_APPLY) {
          const int r = (w >= 8 && h >= 8) ? 8 : 4;
          R = std::max(R, std::min(r, h)); C = std::max(C, std::min(r, w));
        }
        j.nz_rows = (uint8_t)R; j.nz_cols = (uint8_t)C;
        j.st_rows = (uint8_t)SR; j.st_cols = (uint8_t)SC;
        j.flags |= TB_PACKED;
      } else {
        int R = 0, C = 0;
        if ((size_t)j.coef + (size_t)w * h > d.coef.size()) throw VvcrError(VVCR_E_ARG, "coefficient offset out of range");
        const int32_t *lv = d.coef.data() + j.coef;
        if (ts) {
          R = h; C = w;
        } else {
          for (int yy = 0; yy < h; yy++) {
            const int32_t *row = lv + yy * w;
            int32_t any = 0;
            for (int xx = 0; xx < w; xx++) any |= row[xx];   // vectorised OR: most rows are all zero
            if (!any) continue;
            R = yy + 1;
            for (int xx = w - 1; xx >= C; xx--)
              if (row[xx]) { C = xx + 1; break; }
          }
          if (j.flags & TB_LFNST_APPLY) {
            const int r = (w >= 8 && h >= 8) ? 8 : 4;
            R = std::max(R, std::min(r, h)); C = std::max(C, std::min(r, w));
          }
        }
        j.nz_rows = (uint8_t)R; j.nz_cols = (uint8_t)C;
        j.st_rows = (uint8_t)R; j.st_cols = (uint8_t)C;
        // only the box travels to the device (most of a large inter TB is zero)
        const size_t off = packed.size();
        packed.resize(off + (size_t)R * C);
        for (int yy = 0; yy < R; yy++) std::memcpy(packed.data() + off + (size_t)yy * C, lv + (size_t)yy * w, (size_t)C * sizeof(int32_t));
        j.coef = (int32_t)off;
        j.flags |= TB_PACKED;
      }
      out.push_back(j);
    }
  }
}

// TB_ZERO jobs: every transform-block area whose residual a consumer reads but no coded block writes (the
// residual planes are not cleared per picture when the reconstruction stages run together). Readers: intra
// CUs (k_intra reads each step's residual rectangle), inter CUs reconstructed by k_recon_inter (LMCS / CIIP:
// the whole CU), and fused inter CUs per component with a coded TB of that component (MC_RESI << comp:
// that component of the whole CU).
void build_zero_jobs(const vvcr_pic_params &pp, const PictureDescriptors &d, bigbuf::vec<TbJob> &out) {
  auto zero = [&](int comp, int x, int y, int w, int h) {
    // split into blocks of at most 64 x 64 (the TbJob sides are 8-bit)
    for (int yy = 0; yy < h; yy += 64)
      for (int xx = 0; xx < w; xx += 64) {
        TbJob j{};
        j.x = (int16_t)(x + xx); j.y = (int16_t)(y + yy);
        j.w = (uint8_t)std::min(64, w - xx); j.h = (uint8_t)std::min(64, h - yy);
        j.comp = (uint8_t)comp;
        j.flags = TB_ZERO;
        out.push_back(j);
      }
  };
  const int ncu = (int)d.cu.size();
  bigbuf::vec<uint8_t> reads(ncu, 0);   // bit comp: the CU's residual of that component is read
  for (int i = 0; i < ncu; i++) {
    const vvcr_cu &c = d.cu[i];
    if (!in_shard(pp, c)) continue;
    if (c.predmode != MODE_INTER) { reads[i] = 7; continue; }
    if (!fused_inter_cu(pp, d, c)) {
      reads[i] = 7;
      if (!c.rootcbf) {   // no transform tree: the whole CU reads zeros
        if (c.yvalid) zero(0, c.x, c.y, c.w, c.h);
        if (c.cvalid) { zero(1, c.cx, c.cy, c.cw, c.ch); zero(2, c.cx, c.cy, c.cw, c.ch); }
        reads[i] = 0;
      }
      continue;
    }
    // a fused CU reads the residual of a component only where one of its TBs is coded (MC_RESI << comp)
    reads[i] = (uint8_t)(cu_resi_flags(d, c) / MC_RESI);
  }
  for (size_t ti = 0; ti < d.tu.size(); ti++) {
    const vvcr_tu &t = d.tu[ti];
    if (t.cu < 0 || t.cu >= ncu || !reads[t.cu]) continue;
    for (int comp = 0; comp < 3; comp++) {
      const int32_t *b = t.b[comp];
      if (b[2] <= 0 || !((reads[t.cu] >> comp) & 1)) continue;
      // the coded-block rule of build_tb_jobs: a JCCR Cb job writes Cr too
      bool written;
      if (comp == 2 && t.jccr) {
        const int src = (t.jccr >> 1) ? 1 : 2;
        written = t.b[src][6] >= 0;
      } else if (comp == 1 && t.jccr) {
        const int src = (t.jccr >> 1) ? 1 : 2;
        written = t.b[src][6] >= 0;
      } else {
        written = b[4] != 0 && b[6] >= 0;
      }
      if (!written) zero(comp, b[0], b[1], b[2], b[3]);
    }
  }
}

void lf_ctb_neighbours(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, std::vector<uint8_t> &nb) {
  nb.clear();
  const int ctu = 1 << sp.ctu_log2, wc = (sp.width + ctu - 1) / ctu, hc = (sp.height + ctu - 1) / ctu;
  const bool tiles = (pp.num_tile_cols > 1 || pp.num_tile_rows > 1) && !pp.lf_across_tiles;
  bool slices = false;
  for (const vvcr_cu &c : d.cu) slices |= c.slice != d.cu[0].slice;
  slices = slices && !pp.lf_across_slices;
  if (!tiles && !slices) return;
  // the slice of every CTB: of the CU at its origin (the first CU of a CTB in decoding order)
  std::vector<int> slice((size_t)wc * hc, -1);
  for (const vvcr_cu &c : d.cu) {
    const int x = c.yvalid ? c.x : 2 * c.cx, y = c.yvalid ? c.y : 2 * c.cy;
    if ((x & (ctu - 1)) == 0 && (y & (ctu - 1)) == 0) slice[(size_t)(y >> sp.ctu_log2) * wc + (x >> sp.ctu_log2)] = c.slice;
  }
  for (int v : slice)
    if (v < 0) throw VvcrError(VVCR_E_ARG, "loop filter boundaries: a CTB without a CU at its origin");
  auto tile_of = [&](int cx, int cy) {
    int tc = 0, tr = 0;
    for (int t = 0; t < pp.num_tile_cols; t++) if (cx >= pp.tile_col_bd[t]) tc = t;
    for (int t = 0; t < pp.num_tile_rows; t++) if (cy >= pp.tile_row_bd[t]) tr = t;
    return tr * 1024 + tc;
  };
  const size_t n = (size_t)wc * hc;
  nb.assign(n, 0);
  std::vector<uint8_t> pad;   // ALF raster-slice corner padding per CTB (bit 0 top-left, bit 1 bottom-right)
  static const int dx[8] = {-1, 1, 0, 0, -1, 1, -1, 1}, dy[8] = {0, 0, -1, 1, -1, -1, 1, 1};
  for (int cy = 0; cy < hc; cy++)
    for (int cx = 0; cx < wc; cx++) {
      const size_t k = (size_t)cy * wc + cx;
      uint8_t m = 0;
      for (int j = 0; j < 8; j++) {
        const int nx = cx + dx[j], ny = cy + dy[j];
        if (nx < 0 || ny < 0 || nx >= wc || ny >= hc) continue;
        const size_t n = (size_t)ny * wc + nx;
        if (slices && slice[n] != slice[k]) continue;
        if (tiles && tile_of(nx, ny) != tile_of(cx, cy)) continue;
        m |= (uint8_t)(1u << j);
      }
      nb[k] = m;
      // ALF's raster-slice corner padding (AdaptiveLoopFilter.cpp:172-198): the top-left (bottom-right) CTB of
      // another slice while the top and left (bottom and right) ones are available: the CTB's copy takes its
      // corner margin from its first column (last column) of the same row (AreaBuf::padBorderPel, Buffer.h:571)
      if (slices) {
        const bool tl = cx > 0 && cy > 0 && (m & LFNB_L) && (m & LFNB_A) && slice[k - wc - 1] != slice[k];
        const bool br = cx + 1 < wc && cy + 1 < hc && (m & LFNB_R) && (m & LFNB_B) && slice[k + wc + 1] != slice[k];
        if (tl || br) {
          if (pad.empty()) pad.assign(n, 0);
          pad[k] = (uint8_t)((tl ? 1 : 0) | (br ? 2 : 0));
        }
      }
    }
  // the pad flags (if any CTB has one) follow the n neighbour masks: entries [n, 2n) (k_alf's AlfParams::pad)
  if (!pad.empty()) nb.insert(nb.end(), pad.begin(), pad.end());
}
