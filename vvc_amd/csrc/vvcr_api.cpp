// vvcr_api.cpp — C-ABI implementation of libvvcr: device DPB, descriptor staging, per-picture work
// planning on the host (C++) and kernel launches on one ordered HIP stream.
//
// A picture goes through two phases: prepare (host planning of every work list + upload of the
// descriptors / lists / loop-filter parameters into device buffers owned by a Prepared record) and
// launch (enqueue the kernels that read only device-resident data). vvcr_end_picture does both;
// vvcr_prepare_picture / vvcr_launch_picture expose them separately so that a caller (or bench.py) can
// keep pictures resident and replay them, and so that host planning of picture N+1 can overlap the GPU
// work of picture N.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <atomic>
#include <pthread.h>
#include <chrono>
#include <string>
#include <vector>

#include "vvcr_internal.h"
#include "vvcr_host.h"
#include "vvcr_dbk.h"
#include "vvcr_intra.h"

namespace {

thread_local std::string g_create_error;
// Error text of the last failing context call, per calling thread (like errno): vvcr_prepare_planned may
// fail on several threads at once, so the message is never a field shared between threads.
thread_local std::string g_ctx_error;
// live contexts: the last vvcr_destroy frees the large-buffer cache's unused page-locked blocks
static std::atomic<int> g_live_ctx{0};

// device / page-locked allocations made while preparing pictures (VVCR_PREP_PROF reports them)
std::atomic<uint64_t> g_prep_allocs{0}, g_prep_alloc_bytes{0};

template <class T>
struct DevVec {
  T *p = nullptr;
  size_t cap = 0;
  bool view = false;   // p points into a Prepared record's upload arena (not owned)
  void set_view(T *q) {
    if (p && !view) VVCR_CHECK_HIP(hipFree(p));
    p = q;
    cap = 0;
    view = true;
  }
  void ensure(size_t n) {
    if (view) { p = nullptr; view = false; }
    if (n <= cap) return;
    if (p) VVCR_CHECK_HIP(hipFree(p));
    // doubling: a prepared record is recycled for pictures of every size, and each regrowth is a hipFree
    // (which waits for the device) and a hipMalloc on the preparing thread
    size_t c = std::max<size_t>(n, cap * 2 + 64);
    VVCR_CHECK_HIP(hipMalloc(&p, c * sizeof(T)));
    g_prep_allocs++;
    g_prep_alloc_bytes += c * sizeof(T);
    cap = c;
  }
  // synchronous upload: the caller guarantees no kernel is reading this buffer (Prepared::wait)
  void upload(const T *src, size_t n) {
    ensure(n + 1);
    if (n) VVCR_CHECK_HIP(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  }
  template <class A> void upload(const std::vector<T, A> &v) { upload(v.data(), v.size()); }
  DevVec() = default;
  DevVec(const DevVec &) = delete;
  DevVec &operator=(const DevVec &) = delete;
  ~DevVec() { if (p && !view) (void)hipFree(p); }
};

// Upload staging of one prepared picture: every host array its kernels read is copied into one pinned
// buffer, then one asynchronous copy moves it to one device arena on the context's upload stream (the
// lanes wait for its event). A picture's upload costs one DMA instead of a dozen synchronous pageable
// copies, and the preparing thread does not wait for it. Large arrays that already sit in page-locked
// memory (bigbuf::is_pinned) are not copied: they get their own DMA into the arena (add_big), and the
// picture that owns them waits for it before it changes or frees them (vvcr_picture::settle).
struct Staging {
  uint8_t *h = nullptr;
  size_t cap = 0, used = 0;
  DevVec<uint8_t> arena;
  struct Item { void **dst; size_t off; };
  std::vector<Item> items;
  struct Ext { void **dst; const void *src; size_t bytes, off; };
  std::vector<Ext> ext;
  size_t ext_used = 0, base = 0;
  ~Staging() { if (h) (void)hipHostFree(h); }
  void begin() { used = 0; items.clear(); ext.clear(); ext_used = 0; }
  template <class T> void add_big(DevVec<T> &d, const T *src, size_t n) {
    static const bool off = getenv("VVCR_NO_DIRECT_UPLOAD") != nullptr;   // diagnostics: stage everything
    const size_t bytes = n * sizeof(T);
    if (off || bytes < bigbuf::kPinMin || !bigbuf::is_pinned(src)) { add(d, src, n); return; }
    const size_t o = (ext_used + 255) & ~(size_t)255;
    ext.push_back({(void **)&d.p, src, bytes, o});
    ext_used = o + bytes + sizeof(T);   // (n + 1) elements, as add() reserves
    d.set_view(nullptr);
  }
  template <class T, class A> void add_big(DevVec<T> &d, const std::vector<T, A> &v) { add_big(d, v.data(), v.size()); }
  void reserve(size_t n) {
    if (n <= cap) return;
    const size_t c = std::max(n, cap * 2 + (1 << 20));
    uint8_t *q = nullptr;
    VVCR_CHECK_HIP(hipHostMalloc((void **)&q, c, hipHostMallocDefault));
    g_prep_allocs++;
    g_prep_alloc_bytes += c;
    if (used) std::memcpy(q, h, used);
    if (h) VVCR_CHECK_HIP(hipHostFree(h));
    h = q;
    cap = c;
  }
  // appends the parts (pointer, count) as one contiguous array for d
  template <class T> void add(DevVec<T> &d, std::initializer_list<std::pair<const T *, size_t>> parts) {
    size_t n = 0;
    for (auto &pt : parts) n += pt.second;
    const size_t off = (used + 255) & ~(size_t)255;
    reserve(off + (n + 1) * sizeof(T));
    size_t o = off;
    for (auto &pt : parts) {
      if (pt.second) std::memcpy(h + o, pt.first, pt.second * sizeof(T));
      o += pt.second * sizeof(T);
    }
    used = off + (n + 1) * sizeof(T);
    items.push_back({(void **)&d.p, off});
    d.set_view(nullptr);
  }
  template <class T, class A> void add(DevVec<T> &d, const std::vector<T, A> &v) { add(d, {{v.data(), v.size()}}); }
  template <class T> void add(DevVec<T> &d, const T *src, size_t n) { add(d, {{src, n}}); }
  // offset of the last add's array in the staging buffer, and its host copy there (valid until the next
  // add): records that hold device pointers of other staged arrays are rewritten after place(), when
  // those pointers are final
  size_t last_off() const { return items.back().off; }
  template <class T> T *host_at(size_t off) { return (T *)(h + off); }
  // the device arena is sized and every staged DevVec points into it; nothing is copied yet
  void place(size_t floor) {
    base = (used + 255) & ~(size_t)255;
    arena.ensure(std::max(base + ext_used + 256, floor));
    for (const Item &it : items) *it.dst = arena.p + it.off;
    for (const Ext &e : ext) *e.dst = arena.p + base + e.off;
  }
  void copy(hipStream_t s, hipEvent_t done) {
    if (used) VVCR_CHECK_HIP(hipMemcpyAsync(arena.p, h, used, hipMemcpyHostToDevice, s));
    for (const Ext &e : ext) VVCR_CHECK_HIP(hipMemcpyAsync(arena.p + base + e.off, e.src, e.bytes, hipMemcpyHostToDevice, s));
    VVCR_CHECK_HIP(hipEventRecord(done, s));
  }
};

DPlane alloc_plane(int w, int h) {
  DPlane d;
  d.w = w; d.h = h;
  d.stride = (w + 63) & ~63;
  // + 64 samples: the MC gathers read whole aligned 4-sample chunks, up to 16 samples past the last
  // window sample (never used, but they must be inside the allocation on the last row)
  const size_t n = (size_t)d.stride * h + 64;
  VVCR_CHECK_HIP(hipMalloc(&d.p, n * sizeof(int16_t)));
  VVCR_CHECK_HIP(hipMemset(d.p, 0, n * sizeof(int16_t)));
  return d;
}

// kernel groups timed with HIP events (vvcr_kernel_stats)
enum { K_RESID, K_MC, K_MC_BIDIR, K_MC_AFFINE, K_RECON, K_INTRA, K_DBK, K_SAO, K_ALF, K_DBKP, NK };
const char *const kKernelNames[NK] = {"resid", "mc", "mc_bidir", "mc_affine", "recon_inter", "intra", "deblock", "sao", "alf",
                                      "deblock_plan"};
// stage of each kernel group (bit index in VVCR_STAGE_*)
const int kKernelStage[NK] = {0, 1, 1, 1, 2, 2, 4, 5, 6, 4};

// Flags of the events host threads wait on (picture done, DMVR deltas read back, upload done): HIP's default
// active wait, or with VVCR_BLOCKING_WAIT hipEventBlockingSync (the waiting thread sleeps until the device
// signals; measured against the default in DESIGN §5)
static unsigned wait_flags() {
  static const unsigned f = getenv("VVCR_BLOCKING_WAIT") ? (unsigned)hipEventBlockingSync : 0u;
  return f;
}

struct Prepared {
  vvcr_pic_params pp{};
  uint32_t mask = 0;
  DevVec<int32_t> coef;
  DevVec<TbJob> tb;
  DevVec<McJob> mc_basic, mc_bidir;
  DevVec<AffPu> aff_pu;
  DevVec<AffJob> aff_jobs;
  DevVec<ReconTile> tiles;
  DevVec<IntraJob> ijobs;
  DevVec<int32_t> idep_start, ideps, istate, ictu_list, ictu_start;
  DevVec<IntraParams> iparams;       // device copy of the intra kernel's parameters
  DevVec<int16_t> lmcs_lut;          // LMCS forward [0, 1024) and inverse [1024, 2048) luma LUTs
  int n_ijobs = 0, n_ictu = 0;
  DevVec<DbkSeg> dbk;
  int dbk_counts[4] = {0, 0, 0, 0};
  DevVec<int32_t> dbk_cnt;           // the host plan's list lengths, device copy (k_dbk reads them there)
  // device deblocking planning (vvcr_dbk_plan.hip): compact descriptors and the 4x4 motion field
  bool dbk_gpu = false, dbk_chroma_pass = false;
  DevVec<DbCu> dbcu;
  DevVec<DbPu> dbpu;
  DevVec<DbTu> dbtu;
  DevVec<MotionRec> dbmot;
  int n_dbcu = 0, n_dbtu = 0;
  size_t n_dbmot = 0;   // motion records staged (0: a picture without inter CUs)
  int32_t dbk_nitems[4] = {0, 0, 0, 0};
  DevVec<int32_t> sao;
  DevVec<int16_t> alf_luma_coef, alf_luma_clip, alf_chroma, alf_cc, alf_set;
  DevVec<uint8_t> alf_ctb;
  DevVec<uint8_t> lf_nb;             // lf_ctb_neighbours of the picture (SAO / ALF), n_lf_nb entries
  int n_lf_nb = 0;
  DevVec<int32_t> dmvr;
  DevVec<WpTable> wpt;               // the slice's weighted-prediction table (k_mc reads it per lane)
  McClassTable mc_ct;                // k_mc cell classes of mc_basic (edge jobs, tiles, blocks)
  DevVec<McClassTable> mc_ctd;       // the same in device memory (a batched k_mc reads each picture's)
  bool have_sao = false, have_alf = false;
  // exactly one of SAO / ALF and every stage in one prepared picture: the picture is reconstructed and
  // deblocked in the lane's loop-filter planes, and that one filter writes it into its slot (no copy-back)
  bool recon_tmp = false;
  bool zero_filled = false;   // the residual areas read are zeroed by TB_ZERO jobs: no plane clear
  int n_tb = 0, n_tb_small = 0, n_mctile = 0, n_basic = 0, n_bidir = 0, n_aff = 0, n_tiles = 0, n_dmvr = 0;
  hipEvent_t ev[NK][2] = {};
  hipEvent_t start = nullptr, done = nullptr;   // whole launch (events of this picture only: an event
                                                // shared by pictures of several lanes would serialise them)
  hipEvent_t ev_mc = nullptr;                   // after the inter stage on the lane
  hipEvent_t mc_done = nullptr;                 // the DMVR deltas of the launch are in h_dmvr
  int32_t *h_dmvr = nullptr;                    // pinned host copy of the DMVR deltas
  size_t h_dmvr_cap = 0;
  Staging up;                                   // the picture's host arrays, staged for one upload
  hipEvent_t up_done = nullptr;                 // the upload has landed in up.arena
  bool up_issued = false;
  bool ran[NK] = {};
  bool timed[NK] = {};              // the group's events were recorded by the last launch
  bool launched = false;
  int lane = 0;                      // execution lane of the last launch (its stream and scratch planes)
  int set = 0;                       // the lane's scratch set of the last launch (k: k-th picture of a batch)
  int kpics[NK] = {};                // pictures each kernel group's launch of this record carried (MC groups of a
                                     // frame-batched launch: the first picture's record holds the launch, its
                                     // time and bytes and the count; the others 0)
  uint32_t staged = 0;               // stages launched so far by vvcr_launch_picture_stages (0: none pending)
  double alg_bytes[NK] = {};
  int launches[NK] = {};

  Prepared() {
    for (auto &e : ev) { VVCR_CHECK_HIP(hipEventCreate(&e[0])); VVCR_CHECK_HIP(hipEventCreate(&e[1])); }
    VVCR_CHECK_HIP(hipEventCreateWithFlags(&done, wait_flags()));
    VVCR_CHECK_HIP(hipEventCreate(&start));
    VVCR_CHECK_HIP(hipEventCreateWithFlags(&mc_done, hipEventDisableTiming | wait_flags()));
    VVCR_CHECK_HIP(hipEventCreateWithFlags(&ev_mc, hipEventDisableTiming));
    VVCR_CHECK_HIP(hipEventCreateWithFlags(&up_done, hipEventDisableTiming | wait_flags()));
  }
  ~Prepared() {
    for (auto &e : ev) { (void)hipEventDestroy(e[0]); (void)hipEventDestroy(e[1]); }
    (void)hipEventDestroy(done);
    (void)hipEventDestroy(start);
    (void)hipEventDestroy(ev_mc);
    if (up_issued) (void)hipEventSynchronize(up_done);   // the DMA may still read the pinned staging buffer
    (void)hipEventDestroy(up_done);
    (void)hipEventSynchronize(mc_done);                   // nor may a queued DMVR delta read-back land in h_dmvr
    (void)hipEventDestroy(mc_done);
    if (h_dmvr) (void)hipHostFree(h_dmvr);
  }
  void wait() { if (launched) VVCR_CHECK_HIP(hipEventSynchronize(done)); }
  // back to the state of a new record, keeping its device buffers, events and pinned memory for reuse
  void recycle() {
    mask = 0;
    n_ijobs = n_ictu = 0;
    for (int &c : dbk_counts) c = 0;
    dbk_gpu = dbk_chroma_pass = false;
    n_dbcu = n_dbtu = 0;
    n_dbmot = 0;
    have_sao = have_alf = false;
    n_tb = n_tb_small = n_mctile = n_basic = n_bidir = n_aff = n_tiles = n_dmvr = 0;
    zero_filled = false;
    recon_tmp = false;
    for (int k = 0; k < NK; k++) { ran[k] = timed[k] = false; alg_bytes[k] = 0; launches[k] = 0; }
    launched = false;
    staged = 0;
    lane = 0;
    set = 0;
    for (int &k : kpics) k = 1;
  }
};

// Per-kernel-group HIP events (vvcr_kernel_stats). Every event record is a marker packet in the lane's
// queue, so the events are only recorded while timing is on (vvcr_set_timing; on by default).
struct KernelTimer {
  Prepared &r;
  int k;
  hipStream_t s;
  bool on;
  KernelTimer(Prepared &rr, int kk, hipStream_t ss, bool timing) : r(rr), k(kk), s(ss), on(timing) {
    r.ran[k] = true;
    r.timed[k] = on;
    if (on) VVCR_CHECK_HIP(hipEventRecord(r.ev[k][0], s));
  }
  ~KernelTimer() { if (on) (void)hipEventRecord(r.ev[k][1], s); }
};

}  // namespace

// A planned batch of the encoder RDO inner loop: Hadamard tiles sorted by kind (distortion) or the
// transform blocks (forward transform), resident on the device.
struct RdoPlan {
  bool fwd = false;
  int nblocks = 0, bd = 10;
  DevVec<RdBlockDev> blocks;
  DevVec<RdTile> tiles[RD_KINDS];
  int ntiles[RD_KINDS] = {};
  DevVec<FwdBlockDev> fblocks;      // sorted by class (w, h, tr_hor, tr_ver, lfnst)
  struct Cls { int start, n, w, h, trh, trv, lfnst; };
  std::vector<Cls> classes;
  int64_t coef_total = 0;
};

// A picture under construction on the host (vvcr_picture_*): its parameters, descriptors and loop-filter
// parameters, and after vvcr_picture_plan its work lists. Host memory only, no device or context: a
// producer may build and plan several pictures on several threads at once (one thread per picture) and
// hand them to vvcr_prepare_planned, which only uploads.
struct vvcr_picture {
  vvcr_seq_params sp{};
  vvcr_pic_params pp{};
  std::string err;
  PictureDescriptors desc;
  bool submitted = false;
  bool have_sao = false, have_alf = false;
  std::vector<int32_t> h_sao;
  std::vector<int16_t> h_alf_luma_coef, h_alf_luma_clip, h_alf_chroma, h_alf_cc, h_alf_set;
  std::vector<uint8_t> h_alf_ctb;
  uint32_t mask = 0;
  bool planned = false;
  WorkLists wl;
  IntraPlan intra;
  DbkLists dbk;
  bool dbk_gpu = false;              // the edges are planned on the device from dbkg (default; VVCR_DBK_GPU=0: host)
  DbkGpuInputs dbkg;
  std::vector<uint8_t> lf_nb;        // lf_ctb_neighbours (empty: loop filters across every tile / slice)
  // an upload that DMAs straight from this picture's page-locked arrays (Staging::add_big) is in flight
  // until up_ev: settle() before the arrays change or are freed
  mutable hipEvent_t up_ev = nullptr;
  mutable bool up_pending = false;
  vvcr_picture() = default;
  vvcr_picture(const vvcr_picture &) = delete;
  vvcr_picture &operator=(const vvcr_picture &) = delete;
  void settle() {
    if (up_pending) { (void)hipEventSynchronize(up_ev); up_pending = false; }
  }
  ~vvcr_picture() {
    settle();
    if (up_ev) (void)hipEventDestroy(up_ev);
  }
};

// deblocking planned on the device (vvcr_dbk_plan.hip) unless VVCR_DBK_GPU=0 (the host planner,
// vvcr_dbk_host.cpp: same lists, kept for A/B and as the parity reference of the device planner)
static bool dbk_on_device() {
  const char *e = getenv("VVCR_DBK_GPU");
  return !(e && e[0] == '0');
}

// Hadamard tile of RdCost::xGetHADs for a w x h block (RdCost.cpp:2818-2911), or -1 for odd sizes
static int rd_kind(int w, int h, int &tw, int &th) {
  if (w > h && (h & 7) == 0 && (w & 15) == 0) { tw = 16; th = 8; return RD_16x8; }
  if (w < h && (w & 7) == 0 && (h & 15) == 0) { tw = 8; th = 16; return RD_8x16; }
  if (w > h && (h & 3) == 0 && (w & 7) == 0) { tw = 8; th = 4; return RD_8x4; }
  if (w < h && (w & 3) == 0 && (h & 7) == 0) { tw = 4; th = 8; return RD_4x8; }
  if (h % 8 == 0 && w % 8 == 0) { tw = 8; th = 8; return RD_8x8; }
  if (h % 4 == 0 && w % 4 == 0) { tw = 4; th = 4; return RD_4x4; }
  if (h % 2 == 0 && w % 2 == 0) { tw = 2; th = 2; return RD_2x2; }
  return -1;
}

// Execution lanes: pictures are launched on nlane HIP streams (VVCR_LANES, default 4 = HIP's default
// hardware queues per process; up to MAXLANE when GPU_MAX_HW_QUEUES allows), each with its own scratch planes
// (prediction, residual, loop-filter ping-pong). A picture waits only for the pictures it depends on —
// the last writer of each reference slot (RAW), and the last writer and every reader since of its own
// slot (WAW / WAR) — so pictures that do not reference each other (the pictures of one temporal layer of
// an RA GOP, an intra picture and the B pictures decoded before it) reconstruct concurrently.
constexpr int MAXLANE = 16;
// A lane's scratch planes: set 0 serves every picture; set k (allocated at the lane's first batched launch) the
// k-th picture of a frame-batched launch (vvcr_launch_pictures), whose residual / prediction / loop-filter
// planes must stay intact while the batch's other pictures run.
struct ScratchSet {
  DPlane pred[3], resi[3], tmp[3];
};
struct Lane {
  hipStream_t s = nullptr;
  ScratchSet set[MC_MAXPIC];
  DevVec<uint8_t> dbkp;              // device deblocking planner's maps and lists (allocated at its first use)
  int dbkp_gen = 0;                  // generation of its maps' entries (0: the buffer is new, clear it)
  const void *held = nullptr;        // a picture launched stage by stage whose later stages are pending here
  int tail_slot = -1;                // DPB slot written by the lane's last picture
  uint64_t tail_seq = 0;             // launch sequence number of that picture
};

struct vvcr_ctx {
  vvcr_seq_params sp{};
  hipStream_t stream = nullptr;      // lane 0's stream (host copies, vvcr_stream)
  hipStream_t upload_stream = nullptr;   // prepared pictures' uploads (Staging)
  hipStream_t copy_stream = nullptr; // halo row export / import (vvcr_export_rows / vvcr_import_rows), output frames
  DevVec<uint8_t> out_stage;         // vvcr_write_output to host memory
  std::vector<std::array<DPlane, 3>> dpb;
  Lane lanes[MAXLANE];
  int nlane = 4, nintra = 2;         // lanes; the first nintra take pictures without references
  int intra_wg = 0;                  // k_intra workgroups (VVCR_INTRA_WG, default set in vvcr_create)
  uint64_t seq = 0;
  bool timing = true;                // record per-kernel-group events (vvcr_set_timing)
  // Dependency markers, owned per DPB slot so that no event is ever shared between slots: slot_w[s] is
  // re-recorded by every writer of slot s, slot_r[s][l] by every reader of s on lane l. A stream wait
  // captures the event's most recent record, so a later picture waits on exactly the last writer (RAW)
  // and, when it overwrites s, on the last reader of every lane (WAR) — a lane's stream is in order, so
  // its last reader follows all its earlier ones. Readers of s from before its previous writer are
  // covered by that writer (it waited on them). No launch count or host sync bounds this.
  std::vector<hipEvent_t> slot_w;                   // per DPB slot: its last writer
  std::vector<uint8_t> slot_w_set;                  // slot_w recorded at least once
  std::vector<std::array<hipEvent_t, MAXLANE>> slot_r;   // per DPB slot and lane: last reader
  std::vector<uint32_t> slot_r_set;                 // per DPB slot: lanes with a reader since the last write
  std::vector<uint64_t> slot_seq;                   // per DPB slot: launch sequence number of its last writer
  std::vector<int> slot_lane;                       // per DPB slot: lane of its last writer (-1 none, or a
                                                    // caller's stream: vvcr_import_rows_async)
  std::vector<hipEvent_t> slot_x;                   // per DPB slot: its last reader on a caller's stream
  std::vector<uint8_t> slot_x_set;                  // (vvcr_export_rows_async): the slot's next writer waits
  int lane_policy = 1;                              // VVCR_LANE_POLICY: 1 lane of the newest reference, 0 tail only
  bool in_picture = false;
  vvcr_picture cur;                  // the picture of vvcr_begin_picture .. vvcr_end_picture / vvcr_prepare_picture
  DevVec<uint16_t> d_scans;
  DevVec<const int16_t *> d_ref_table;   // DPB plane pointers [slot * 3 + comp] (RefPlanes)
  ScanTables scans;
  // prepared pictures: index 0 is the scratch record of vvcr_end_picture. The table is shared by the
  // threads calling vvcr_prepare_planned and the launching thread: `prepared_mu` guards it (a record
  // itself is only touched by the thread that prepares it, then by launch / release).
  std::vector<std::unique_ptr<Prepared>> prepared;
  std::mutex prepared_mu;
  // released records, kept with their device buffers: allocating and freeing device memory per picture
  // would cost a hipMalloc per buffer and a device-wide synchronisation per hipFree
  std::vector<std::unique_ptr<Prepared>> spare;
  std::mutex launch_mu;              // launches, releases and host reads / writes of the DPB may come from
                                     // several host threads (vvcp_decode of several streams at once)
  Prepared *last = nullptr;          // last launched (stage times, DMVR deltas)
  int n_cu = 256;                    // compute units (persistent intra launch width)
  std::vector<std::unique_ptr<struct RdoPlan>> rdo;   // encoder RDO plans (vvcr_rd_plan / vvcr_fwd_plan)
  // vvcr_rd_dist's staging: one page-locked host span and its device copy (results, block records, tiles,
  // samples), grown only, so that a call is one upload, its launches, one read-back and one synchronisation
  std::mutex rd_mu;
  char *rd_h = nullptr, *rd_d = nullptr;
  size_t rd_cap = 0;
  int32_t *d_err = nullptr;          // device error flag of the persistent intra kernel (checked by vvcr_sync)
};

// The device error words (after the lanes are idle): [0] the persistent intra kernel's dependency-wait
// timeout (its waits poll this word and give up when it is set), [1] the device deblocking planner
// (bit 2: a position no CU / TU covers, bit 4: list overflow, bit 8: not a wave64 device) — a word of its own, so that it never
// cuts the intra waits of other pictures short.
static void check_device_errors(vvcr_ctx *ctx) {
  int32_t e[2] = {0, 0};
  VVCR_CHECK_HIP(hipMemcpy(e, ctx->d_err, sizeof e, hipMemcpyDeviceToHost));
  if (e[0] | e[1]) {
    VVCR_CHECK_HIP(hipMemset(ctx->d_err, 0, sizeof e));
    if (e[0]) throw VvcrError(VVCR_E_STATE, "intra reconstruction: a step's dependency wait timed out (output invalid)");
    if (e[1] & 2) throw VvcrError(VVCR_E_STATE, "deblocking planner: no CU / TU covers a neighbouring position (inconsistent descriptors)");
    if (e[1] & 8) throw VvcrError(VVCR_E_STATE, "deblocking planner: built for 64-lane waves, the device runs another wave size");
    throw VvcrError(VVCR_E_STATE, "deblocking planner: segment list overflow");
  }
}

// every lane idle (host reads / writes of planes, vvcr_sync)
static void sync_lanes(vvcr_ctx *ctx) {
  for (int l = 0; l < ctx->nlane; l++) VVCR_CHECK_HIP(hipStreamSynchronize(ctx->lanes[l].s));
  // row copies enqueued on callers' streams (vvcr_*_rows_async)
  for (size_t k = 0; k < ctx->slot_w.size(); k++) {
    if (ctx->slot_w_set[k] && ctx->slot_lane[k] < 0) VVCR_CHECK_HIP(hipEventSynchronize(ctx->slot_w[k]));
    if (ctx->slot_x_set[k]) VVCR_CHECK_HIP(hipEventSynchronize(ctx->slot_x[k]));
  }
}

#define API_BEGIN try {
#define API_END                                                  \
  }                                                              \
  catch (const VvcrError &e) { g_ctx_error = e.msg; return e.code; } \
  catch (const std::exception &e) { g_ctx_error = e.what(); return VVCR_E_STATE; }

static int n_ctb(const vvcr_seq_params &sp) {
  const int ctu = 1 << sp.ctu_log2;
  return ((sp.width + ctu - 1) / ctu) * ((sp.height + ctu - 1) / ctu);
}

// WeightPrediction::getWpScaling (WeightPrediction.cpp:125-152): offsets scaled to the bit depth
static WpTable make_wp_table(const vvcr_pic_params &pp, int bit_depth) {
  WpTable T{};
  const int osc = 1 << (bit_depth - 8);
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < VVCR_MAX_REF; i++)
      for (int c = 0; c < 3; c++) {
        const int32_t *e = pp.wp[l][i][c];
        T.d[l][i][c] = (int8_t)e[1];
        T.w[l][i][c] = (int16_t)e[2];
        T.o[l][i][c] = (int16_t)(e[3] * osc);
      }
  return T;
}

// the planes a prepared picture is reconstructed (and deblocked) in on a lane's scratch set
static const DPlane *recon_planes(vvcr_ctx *ctx, const Prepared &r, int lane, int set) {
  return r.recon_tmp ? ctx->lanes[lane].set[set].tmp : ctx->dpb[r.pp.slot].data();
}

static McParams make_mc_params(vvcr_ctx *ctx, const Prepared &r, int lane, int set, const WpTable *wpd) {
  const vvcr_pic_params &pp = r.pp;
  McParams P{};
  P.ref.p = ctx->d_ref_table.p;
  for (int c = 0; c < 3; c++) {
    P.ref.stride[c] = ctx->dpb[0][c].stride; P.ref.w[c] = ctx->dpb[0][c].w; P.ref.h[c] = ctx->dpb[0][c].h;
  }
  const ScratchSet &S = ctx->lanes[lane].set[set];
  for (int c = 0; c < 3; c++) P.out[c] = S.pred[c];
  P.pic_w = ctx->sp.width;
  P.pic_h = ctx->sp.height;
  P.bd = ctx->sp.bit_depth;
  P.ctu = 1 << ctx->sp.ctu_log2;
  P.wpd = wpd;
  const DPlane *reco = recon_planes(ctx, r, lane, set);
  for (int c = 0; c < 3; c++) {
    P.reco[c] = reco[c];
    P.resi[c] = S.resi[c];
  }
  return P;
}

// k_mc's view of a prepared picture on a lane's scratch set (one picture of a frame-batched launch)
static McPic make_mc_pic(vvcr_ctx *ctx, const Prepared &r, int lane, int set) {
  McPic q{};
  const ScratchSet &S = ctx->lanes[lane].set[set];
  const DPlane *reco = recon_planes(ctx, r, lane, set);
  for (int c = 0; c < 3; c++) {
    q.out[c] = S.pred[c];
    q.reco[c] = reco[c];
    q.resi[c] = S.resi[c];
  }
  q.wpd = r.wpt.p;
  q.jobs = r.mc_basic.p;
  q.ct = r.mc_ctd.p;
  return q;
}

// parameters of the intra / inter-reconstruction kernels for a prepared picture
static IntraParams make_intra_params(vvcr_ctx *ctx, const Prepared &r, int lane, int set) {
  const vvcr_pic_params &pp = r.pp;
  IntraParams P{};
  const DPlane *reco = recon_planes(ctx, r, lane, set);
  const ScratchSet &S = ctx->lanes[lane].set[set];
  for (int c = 0; c < 3; c++) {
    P.reco[c] = reco[c];
    P.pred[c] = S.pred[c];
    P.resi[c] = S.resi[c];
  }
  P.bd = ctx->sp.bit_depth;
  P.ctu = 1 << ctx->sp.ctu_log2;
  P.ctu_log2 = ctx->sp.ctu_log2;
  if (pp.lmcs_enabled) {
    // forward mapping of inter predictions: slices other than I with the slice reshaper on (the CTU
    // flag of DecLib.cpp:1726-1742); chroma residual scaling: picture-header flag
    P.lmcs = (pp.slice_type != 2 ? 1 : 0) | (pp.lmcs_chroma_scale ? 2 : 0);
    P.lmcs_min_bin = pp.lmcs_min_bin;
    P.lmcs_max_bin = pp.lmcs_max_bin;
    for (int i = 0; i < 17; i++) P.lmcs_pivot[i] = pp.lmcs_pivot[i];
    for (int i = 0; i < 16; i++) P.lmcs_cadj[i] = pp.lmcs_cadj[i];
    P.lmcs_fwd = r.lmcs_lut.p;
  }
  return P;
}

// ---- algorithmic bytes: each logical input once, each output once, 2 B / sample
static double mc_bytes(const McJob &j) { return mc_alg_bytes(j.flags, j.w, j.h); }   // + the residual when fused

// Host phase, part 1 (no device): every work list of the picture.
static void plan_picture(vvcr_picture &b, uint32_t mask) {
  if (!b.submitted) throw VvcrError(VVCR_E_STATE, "picture planned before its descriptors were submitted");
  b.settle();
  const vvcr_seq_params &sp = b.sp;
  const vvcr_pic_params &pp = b.pp;
  b.wl.clear();
  b.intra.clear();
  b.dbk.clear();
  b.dbkg.clear();
  b.dbk_gpu = (mask & VVCR_STAGE_DBK) && dbk_on_device();
  // tiles / slices without loop filtering across them: the CTBs' neighbour availability (DBK, SAO, ALF)
  if (mask & (VVCR_STAGE_DBK | VVCR_STAGE_SAO | VVCR_STAGE_ALF)) lf_ctb_neighbours(sp, pp, b.desc, b.lf_nb);
  else b.lf_nb.clear();
  if (pp.lmcs_enabled && sp.bit_depth != 10) throw VvcrError(VVCR_E_UNSUPPORTED, "LMCS tables are captured for 10-bit luma");
  // With the residual, inter and intra stages together, plain inter CUs are reconstructed by k_mc (the
  // prediction plus the residual straight into the picture, fused_inter_cu); a subset of those stages
  // (the stage tests) keeps the separate prediction planes.
  const uint32_t recon3 = VVCR_STAGE_RESID | VVCR_STAGE_INTER | VVCR_STAGE_INTRA;
  const bool fuse = (mask & recon3) == recon3 && getenv("VVCR_NO_FUSE") == nullptr;
  // The three planners read the descriptors only and write disjoint outputs: deblocking runs on a
  // second thread beside the work lists and the intra plan (a 4K intra picture plans in ~100 ms each).
  std::exception_ptr dbk_err;
  std::thread dbk_thread;
  static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;   // diagnostics: phase times to stderr
  auto tp = std::chrono::steady_clock::now();
  auto mark = [&](const char *n) {
    if (!prof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "  plan %-10s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t - tp).count());
    tp = t;
  };
  if ((mask & VVCR_STAGE_DBK) && !b.dbk_gpu)
    dbk_thread = std::thread([&] {
      pthread_setname_np(pthread_self(), "vvcr-plan-dbk");
      try {
        plan_deblocking(sp, pp, b.desc, b.lf_nb, b.dbk);
      } catch (...) {
        dbk_err = std::current_exception();
      }
    });
  // the deblocking inputs and the work lists; for a large picture (an intra picture: thousands of CUs)
  // on a second thread beside the intra plan, which is the longest of the three (its latency is on a
  // single stream's critical path: the later pictures launch after it)
  std::exception_ptr side_err;
  auto side_work = [&] {
    try {
      if ((mask & VVCR_STAGE_DBK) && b.dbk_gpu) {
        // (a picture without inter CUs needs no motion field: the planner never reads it then)
        bool inter = false;
        if (b.desc.motion.empty())
          for (const vvcr_cu &c : b.desc.cu) inter |= c.predmode != 1;   // vvcr_cu::predmode: 1 intra
        if ((inter || !b.desc.motion.empty()) && b.desc.motion.size() != (size_t)(sp.width / 4) * (sp.height / 4))
          throw VvcrError(VVCR_E_ARG, "deblocking: the motion field does not cover the picture");
        pack_dbk_inputs(sp, pp, b.desc, b.lf_nb, b.dbkg);
      }
      if (mask & (VVCR_STAGE_RESID | VVCR_STAGE_INTER)) build_work_lists(sp, pp, b.desc, b.wl, fuse);
    } catch (...) {
      side_err = std::current_exception();
    }
  };
  static const bool serial = getenv("VVCR_PLAN_SERIAL") != nullptr;
  std::thread side;
  if ((mask & VVCR_STAGE_INTRA) && b.desc.cu.size() >= 16384 && !serial) side = std::thread(side_work);
  else side_work();
  mark(side.joinable() ? "side_start" : "dbk+lists");
  try {
    if (mask & VVCR_STAGE_INTRA) plan_intra(sp, pp, b.desc, b.intra, fuse);
    mark("intra");
  } catch (...) {
    if (side.joinable()) side.join();
    if (dbk_thread.joinable()) dbk_thread.join();
    throw;
  }
  if (side.joinable()) side.join();
  mark("side_join");
  if (side_err) {
    if (dbk_thread.joinable()) dbk_thread.join();
    std::rethrow_exception(side_err);
  }
  if ((mask & VVCR_STAGE_INTER) && b.wl.n_unsupported_inter) {
    if (dbk_thread.joinable()) dbk_thread.join();
    throw VvcrError(VVCR_E_UNSUPPORTED, std::to_string(b.wl.n_unsupported_inter) + " inter CUs use tools not supported yet");
  }
  if (dbk_thread.joinable()) dbk_thread.join();
  if (dbk_err) std::rethrow_exception(dbk_err);
  const bool saoOn = pp.sao_luma || pp.sao_chroma;
  const bool alfOn = pp.alf_en[0] || pp.alf_en[1] || pp.alf_en[2];
  if ((mask & VVCR_STAGE_SAO) && saoOn && !b.have_sao)
    throw VvcrError(VVCR_E_STATE, "SAO is enabled for the picture but no SAO parameters were set");
  if ((mask & VVCR_STAGE_ALF) && alfOn && !b.have_alf)
    throw VvcrError(VVCR_E_STATE, "ALF is enabled for the picture but no ALF parameters were set");
  b.mask = mask;
  b.planned = true;
}

// Diagnostics (VVCR_PREP_PROF): summed wall time of prepare()'s phases over all calls, printed at exit.
namespace prep_prof {
constexpr int N = 9;
const char *const names[N] = {"wait", "resid", "inter-lists", "mc_done", "dmvr-bufs", "inter-bytes", "intra+dbk+lf", "place", "copy"};
std::atomic<uint64_t> ns[N], calls;
const bool on = getenv("VVCR_PREP_PROF") != nullptr;
// wall time, or with VVCP_CPU_TIMES the calling thread's CPU time (as vvcp_decode's phase times)
const bool cpu = getenv("VVCP_CPU_TIMES") != nullptr;
struct Report {
  ~Report() {
    if (!on || !calls) return;
    fprintf(stderr, "prepare: %llu calls, %s ms per call:", (unsigned long long)calls.load(), cpu ? "thread CPU" : "wall");
    for (int k = 0; k < N; k++) fprintf(stderr, " %s %.3f", names[k], ns[k].load() * 1e-6 / calls.load());
    fprintf(stderr, "; %llu device / pinned allocations, %.1f MB\n", (unsigned long long)g_prep_allocs.load(), g_prep_alloc_bytes.load() * 1e-6);
  }
} report;
inline uint64_t now_ns() {
  if (cpu) {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
  }
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct Timer {
  uint64_t t = on ? now_ns() : 0;
  void mark(int k) {
    if (!on) return;
    const uint64_t n = now_ns();
    ns[k] += n - t;
    t = n;
  }
};
}  // namespace prep_prof

// Host phase, part 2: upload the planned lists of b into the device buffers of r.
static void prepare(vvcr_ctx *ctx, Prepared &r, const vvcr_picture &bp) {
  prep_prof::Timer pt;
  if (prep_prof::on) prep_prof::calls++;
  if (!bp.planned) throw VvcrError(VVCR_E_STATE, "picture not planned");
  if (bp.sp.width != ctx->sp.width || bp.sp.height != ctx->sp.height || bp.sp.ctu_log2 != ctx->sp.ctu_log2 ||
      bp.sp.bit_depth != ctx->sp.bit_depth || bp.sp.dpb_slots > ctx->sp.dpb_slots)
    throw VvcrError(VVCR_E_ARG, "picture built for other sequence parameters than the context's");
  r.wait();
  if (r.up_issued) VVCR_CHECK_HIP(hipEventSynchronize(r.up_done));   // a prepared, never launched picture
  pt.mark(0);
  Staging &st = r.up;
  st.begin();
  r.pp = bp.pp;
  const uint32_t mask = bp.mask;
  r.mask = mask;
  r.launched = false;
  r.staged = 0;
  {
    std::lock_guard<std::mutex> g(ctx->launch_mu);   // lane state
    for (int l = 0; l < ctx->nlane; l++)
      if (ctx->lanes[l].held == &r) ctx->lanes[l].held = nullptr;
  }
  for (int k = 0; k < NK; k++) { r.alg_bytes[k] = 0; r.launches[k] = 0; r.ran[k] = false; }
  const vvcr_seq_params &sp = ctx->sp;
  const vvcr_pic_params &pp = bp.pp;
  const WorkLists &wl = bp.wl;
  const double pix = (double)sp.width * sp.height * 1.5;   // samples of the three planes
  size_t iparams_off = SIZE_MAX;   // staged intra parameters, rewritten after place()
  if (mask & VVCR_STAGE_RESID) {
    // the packed levels of the transform blocks: the producer's pool when it arrived packed
    st.add_big(r.coef, bp.desc.coef_box.empty() ? bp.wl.coef : bp.desc.coef);
    st.add_big(r.tb, wl.tb);
    r.n_tb = (int)wl.tb.size();
    r.n_tb_small = wl.tb_small;
    r.zero_filled = wl.zero_filled;
    double b = 0;
    for (const TbJob &t : wl.tb) b += (double)t.w * t.h * ((t.flags & TB_ZERO) ? 2 : 4 + 2);   // int32 levels in, int16 residual out
    r.alg_bytes[K_RESID] = b;
  }
  pt.mark(1);
  if (mask & VVCR_STAGE_INTER) {
    // 32x32 tiles first, then the small jobs, in one array
    st.add(r.mc_basic, {{wl.mc_edge.data(), wl.mc_edge.size()}, {wl.mc_tile.data(), wl.mc_tile.size()},
                        {wl.mc_basic.data(), wl.mc_basic.size()}});
    st.add(r.mc_bidir, wl.mc_bidir);
    {
      const WpTable wt = make_wp_table(pp, sp.bit_depth);
      st.add(r.wpt, &wt, 1);
    }
    r.mc_ct = wl.mc_ct;
    st.add(r.mc_ctd, &wl.mc_ct, 1);
    st.add(r.aff_pu, wl.aff_pu);
    st.add(r.aff_jobs, wl.aff_jobs);
    r.n_mctile = (int)wl.mc_tile.size();
    r.n_basic = (int)(wl.mc_basic.size() + wl.mc_edge.size());
    r.n_bidir = (int)wl.mc_bidir.size();
    r.n_aff = (int)wl.aff_jobs.size();
    r.n_dmvr = wl.n_dmvr;
    pt.mark(2);
    // the previous launch's delta read-back (copy stream, after its inter stage) may still be queued
    VVCR_CHECK_HIP(hipEventSynchronize(r.mc_done));
    pt.mark(3);
    // DMVR deltas: sized once for the most a picture can have (a sub-block per 128 luma samples: DMVR
    // needs w, h >= 8 and w * h >= 128), so that a recycled record never reallocates them
    const size_t ndm = std::max(2 * (size_t)r.n_dmvr + 2, 2 * ((size_t)sp.width * sp.height / 128) + 2);
    r.dmvr.ensure(ndm);
    if (r.h_dmvr_cap < ndm) {
      if (r.h_dmvr) VVCR_CHECK_HIP(hipHostFree(r.h_dmvr));
      r.h_dmvr = nullptr;
      r.h_dmvr_cap = ndm;
      VVCR_CHECK_HIP(hipHostMalloc((void **)&r.h_dmvr, r.h_dmvr_cap * sizeof(int32_t), hipHostMallocDefault));
    }
    pt.mark(4);
    r.alg_bytes[K_MC] = wl.mc_alg;
    double b = 0;
    for (const McJob &j : wl.mc_bidir) b += mc_bytes(j);
    r.alg_bytes[K_MC_BIDIR] = b;
    b = 0;
    for (const AffJob &j : wl.aff_jobs) {
      const AffPu &U = wl.aff_pu[j.pu];
      const int lists = U.l[0].present + U.l[1].present;
      const double nsb = (j.w / 4.0) * (j.h / 4.0);
      b += 2.0 * (lists * nsb * (81 + 2 * 0.25 * 49) + 1.5 * j.w * j.h);   // 6-tap (4+5)^2 luma, 4-tap chroma
      b += resi_bytes(U.recon, j.w, j.h);                                      // the residual of a fused reconstruction
    }
    r.alg_bytes[K_MC_AFFINE] = b;
  }
  pt.mark(5);
  if (pp.lmcs_enabled) {
    st.add(r.lmcs_lut, {{pp.lmcs_fwd, 1024}, {pp.lmcs_inv, 1024}});
  }
  if (mask & VVCR_STAGE_INTRA) {
    const IntraPlan &ip = bp.intra;
    st.add(r.tiles, ip.inter_tiles);
    st.add_big(r.ijobs, ip.jobs);
    st.add_big(r.idep_start, ip.dep_start);
    st.add_big(r.ideps, ip.deps);
    r.istate.ensure(std::max<size_t>(16 + ip.jobs.size(), (size_t)sp.width * sp.height / 64));   // (an intra picture's steps)
    // one device copy per lane and scratch set (the plane pointers differ; [set * MAXLANE + lane]), written
    // after place(): they hold the arena address of the LMCS table (staged above), which is only known then
    {
      static const IntraParams blank[MAXLANE * MC_MAXPIC] = {};
      st.add(r.iparams, blank, MAXLANE * MC_MAXPIC);
    }
    iparams_off = st.last_off();
    r.n_ijobs = (int)ip.jobs.size();
    st.add(r.ictu_list, ip.ctu_list);
    st.add(r.ictu_start, ip.ctu_start);
    r.n_ictu = (int)ip.ctu_list.size();
    r.n_tiles = (int)ip.inter_tiles.size();
    double b = 0;
    for (const ReconTile &t : ip.inter_tiles) b += (double)t.w * t.h * 1.5 * 2 * 3;   // pred + resi in, reco out
    r.alg_bytes[K_RECON] = b;
    b = 0;
    for (const IntraJob &j : ip.jobs) {   // resi in, reco out, refs (an ISP job covers isp_k regions)
      const int nreg = (j.flags & (IJ_ISP_HOR | IJ_ISP_VER)) ? j.isp_k : 1;
      b += nreg * ((double)j.w * j.h * 2 * 2 + 2.0 * 2 * (2 * j.w + 2 * j.h));
    }
    r.alg_bytes[K_INTRA] = b;
  }
  if ((mask & VVCR_STAGE_DBK) && bp.dbk_gpu) {
    r.dbk_gpu = true;
    r.dbk_chroma_pass = bp.dbkg.chroma_pass;
    r.n_dbcu = (int)bp.dbkg.cu.size();
    r.n_dbtu = (int)bp.dbkg.tu.size();
    for (int k = 0; k < 4; k++) r.dbk_nitems[k] = bp.dbkg.nitems[k];
    if (r.n_dbcu > 0) {
      st.add_big(r.dbcu, bp.dbkg.cu);
      st.add_big(r.dbpu, bp.dbkg.pu);
      st.add_big(r.dbtu, bp.dbkg.tu);
      st.add_big(r.dbmot, bp.desc.motion.data(), bp.desc.motion.size());
    }
    r.n_dbmot = bp.desc.motion.size();
    r.alg_bytes[K_DBK] = pix * 2 * 2;
    // the planner reads the records and the motion field once
    r.alg_bytes[K_DBKP] = (double)r.n_dbcu * sizeof(DbCu) + (double)bp.dbkg.pu.size() * sizeof(DbPu) +
                          (double)r.n_dbtu * sizeof(DbTu) + (double)bp.desc.motion.size() * sizeof(MotionRec);
  } else if (mask & VVCR_STAGE_DBK) {
    const bigbuf::vec<DbkSeg> *parts[4] = {&bp.dbk.luma[0], &bp.dbk.chroma[0], &bp.dbk.luma[1], &bp.dbk.chroma[1]};
    for (int k = 0; k < 4; k++) r.dbk_counts[k] = (int)parts[k]->size();
    st.add(r.dbk, {{parts[0]->data(), parts[0]->size()}, {parts[1]->data(), parts[1]->size()},
                   {parts[2]->data(), parts[2]->size()}, {parts[3]->data(), parts[3]->size()}});
    st.add(r.dbk_cnt, r.dbk_counts, 4);
    r.alg_bytes[K_DBK] = pix * 2 * 2;
  }
  const bool saoOn = pp.sao_luma || pp.sao_chroma;
  const bool alfOn = pp.alf_en[0] || pp.alf_en[1] || pp.alf_en[2];
  r.have_sao = (mask & VVCR_STAGE_SAO) && saoOn;
  r.have_alf = (mask & VVCR_STAGE_ALF) && alfOn;
  static const bool copy_back = getenv("VVCR_COPY_BACK") != nullptr;   // diagnostics: the r04 copy-back
  r.recon_tmp = r.have_sao != r.have_alf && (mask & VVCR_STAGE_ALL) == VVCR_STAGE_ALL && pp.shard_y1 == 0 && !copy_back;
  r.n_lf_nb = (r.have_sao || r.have_alf) ? (int)bp.lf_nb.size() : 0;
  if (r.n_lf_nb) st.add(r.lf_nb, bp.lf_nb);
  if (r.have_sao) {
    st.add(r.sao, bp.h_sao);
    r.alg_bytes[K_SAO] = pix * 2 * 2;
  }
  if (r.have_alf) {
    st.add(r.alf_luma_coef, bp.h_alf_luma_coef);
    st.add(r.alf_luma_clip, bp.h_alf_luma_clip);
    st.add(r.alf_chroma, bp.h_alf_chroma);
    st.add(r.alf_cc, bp.h_alf_cc);
    st.add(r.alf_ctb, bp.h_alf_ctb);
    st.add(r.alf_set, bp.h_alf_set);
    r.alg_bytes[K_ALF] = pix * 2 * 2;
  }
  pt.mark(6);
  // the device arena: at least 4 bytes per luma sample (a 4K intra picture stages ~30 MB), so that a record
  // recycled from inter to intra pictures does not regrow it
  st.place((size_t)sp.width * sp.height * 4);
  if (iparams_off != SIZE_MAX)
    for (int k = 0; k < MC_MAXPIC; k++)
      for (int l = 0; l < MAXLANE; l++) st.host_at<IntraParams>(iparams_off)[k * MAXLANE + l] = make_intra_params(ctx, r, l, k);
  pt.mark(7);
  st.copy(ctx->upload_stream, r.up_done);
  r.up_issued = true;
  if (!st.ext.empty()) {   // the picture's own arrays are read by the DMA until this event
    if (!bp.up_ev) VVCR_CHECK_HIP(hipEventCreateWithFlags(&bp.up_ev, hipEventDisableTiming));
    VVCR_CHECK_HIP(hipEventRecord(bp.up_ev, ctx->upload_stream));
    bp.up_pending = true;
  }
  pt.mark(8);
}

// The device deblocking planner's arguments for a prepared picture on a lane: the lane's maps and lists
// (allocated at its first use; its pictures run one after the other, so one set serves them all).
static DbkPlanArgs dbk_plan_args(vvcr_ctx *ctx, Lane &ln, const Prepared &r) {
  const vvcr_seq_params &sp = ctx->sp;
  const vvcr_pic_params &pp = r.pp;
  const int W4 = sp.width / 4, H4 = sp.height / 4;
  const size_t n4 = (size_t)W4 * H4, a4 = (n4 + 255) & ~(size_t)255;
  const size_t maps = 4 * a4 * sizeof(int32_t), state = 2 * a4, items = 4 * a4 * sizeof(uint32_t);
  const size_t lists = 4 * a4 * sizeof(DbkSeg);
  const uint8_t *old = ln.dbkp.p;
  ln.dbkp.ensure(maps + state + items + lists + 256);
  uint8_t *p = ln.dbkp.p;
  if (p != old) ln.dbkp_gen = 0;   // a new buffer: cleared with the next generation
  DbkPlanArgs a{};
  a.cu = r.dbcu.p; a.pu = r.dbpu.p; a.tu = r.dbtu.p; a.motion = r.n_dbmot ? r.dbmot.p : nullptr;
  a.ncu = r.n_dbcu; a.ntu = r.n_dbtu; a.W4 = W4; a.H4 = H4; a.ctu_log2 = sp.ctu_log2;
  a.slice_type = pp.slice_type; a.dual_tree = pp.dual_tree; a.dbk_disable = pp.dbk_disable;
  std::memcpy(a.ref_poc, pp.ref_poc, sizeof a.ref_poc);
  a.shard = pp.shard_y1 > 0;
  a.ly0 = pp.shard_y0 - VVCR_LF_HALO; a.ly1 = pp.shard_y1 + VVCR_LF_HALO;
  a.chroma_pass = r.dbk_chroma_pass;
  for (int k = 0; k < 2; k++) {
    a.cu_map[k] = (int32_t *)p + k * a4;
    a.tu_map[k] = (int32_t *)p + (2 + k) * a4;
  }
  a.state[0] = p + maps; a.state[1] = p + maps + a4; a.state_pitch = a4;
  a.items = (uint32_t *)(p + maps + state);
  a.out = (DbkSeg *)(p + maps + state + items);
  a.cap = (int32_t)a4;
  a.counts = (int32_t *)(p + maps + state + items + lists);
  for (int k = 0; k < 4; k++) a.nitems[k] = r.dbk_nitems[k];
  a.err = ctx->d_err + 1;
  // the maps' generation: 1 .. 255, the maps cleared when it restarts
  a.fill = ln.dbkp_gen == 0 || ln.dbkp_gen >= 255;
  ln.dbkp_gen = a.fill ? 1 : ln.dbkp_gen + 1;
  a.gen = ln.dbkp_gen;
  a.num_vb[0] = pp.vb_disabled ? std::min(3, pp.num_vb_ver) : 0;
  a.num_vb[1] = pp.vb_disabled ? std::min(3, pp.num_vb_hor) : 0;
  for (int i = 0; i < 3; i++) { a.vb[0][i] = pp.vb_ver[i]; a.vb[1][i] = pp.vb_hor[i]; }
  return a;
}

// ---- Device phase: the kernels of prepared pictures on a lane ----------------------------------------

// the distinct DPB slots a picture references
static std::vector<int> ref_slots(const vvcr_pic_params &pp) {
  std::vector<int> refs;
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < pp.num_ref[l]; i++)
      if (std::find(refs.begin(), refs.end(), pp.ref_slot[l][i]) == refs.end()) refs.push_back(pp.ref_slot[l][i]);
  return refs;
}

// Lane choice: pictures without references (intra) take lanes [0, nintra), which only intra pictures use, so
// an intra picture never queues behind B pictures and two intra-started segments may overlap; the others take
// the lane of [nintra, nlane) that wrote their newest reference (stream order then costs nothing;
// VVCR_LANE_POLICY=0: only a lane whose last picture is a reference), else the least recently used of those
// lanes. Dependencies on pictures of the chosen lane need no event wait.
static int choose_lane(vvcr_ctx *ctx, const Prepared &r, const std::vector<int> &refs) {
  const int lo = refs.empty() ? 0 : ctx->nintra, hi = refs.empty() ? ctx->nintra : ctx->nlane;
  // the later stages of a picture launched stage by stage stay on its lane: they read that lane's
  // residual / prediction planes
  int L = r.staged ? r.lane : -1;
  // (lanes holding another picture's pending stages are never chosen)
  auto held = [&](int l) { return ctx->lanes[l].held != nullptr && ctx->lanes[l].held != &r; };
  if (L < 0 && !refs.empty() && ctx->lane_policy == 1) {
    // the B lane that wrote the newest of the references (still in its slot): the pictures of one
    // segment then stay on one lane even when other segments' pictures are interleaved on it, and their
    // dependencies are stream order instead of cross-lane event waits
    uint64_t best = 0;
    for (int rs : refs) {
      const int wl = ctx->slot_lane[rs];
      if (wl >= lo && wl < hi && !held(wl) && ctx->slot_seq[rs] > best) { best = ctx->slot_seq[rs]; L = wl; }
    }
  }
  if (!refs.empty() && L < 0)
    for (int l = lo; l < hi && L < 0; l++) {
      const int ts = ctx->lanes[l].tail_slot;
      if (ts >= 0 && !held(l) && std::find(refs.begin(), refs.end(), ts) != refs.end() && ctx->lanes[l].tail_seq == ctx->slot_seq[ts]) L = l;
    }
  if (L < 0) {
    uint64_t best = ~0ull;
    for (int l = lo; l < hi; l++)
      if (!held(l) && ctx->lanes[l].tail_seq < best) { best = ctx->lanes[l].tail_seq; L = l; }
  }
  // every lane of the picture's kind holds another picture's pending stages: its residual / prediction /
  // loop-filter planes are still to be read by those stages, so no lane may take this picture (a held lane
  // would have its planes overwritten and the held picture's later stages would read them: wrong output)
  if (L < 0)
    throw VvcrError(VVCR_E_STATE, "every " + std::string(refs.empty() ? "intra" : "inter") +
                                      " lane holds a picture launched stage by stage whose later stages are pending; "
                                      "launch those stages first (or raise VVCR_LANES)");
  return L;
}

// The picture's rows: a spatial shard reconstructs and filters its own rows; its SAO also covers the 8 rows
// around them that its ALF reads (their deblocked inputs come from the VVCR_LF_HALO rows the caller imported).
struct Rows {
  int own0, own1, sao0, sao1;
};
static Rows pic_rows(const vvcr_ctx *ctx, const vvcr_pic_params &pp) {
  const int H = ctx->sp.height;
  const bool shard = pp.shard_y1 > 0;
  Rows w;
  w.own0 = shard ? pp.shard_y0 : 0;
  w.own1 = shard ? pp.shard_y1 : H;
  w.sao0 = shard ? std::max(0, w.own0 - 8) : 0;
  w.sao1 = shard ? std::min(H, w.own1 + 8) : H;
  return w;
}

// The picture's dependencies on pictures of other lanes (same-lane work is ordered by the stream anyway),
// its upload, and its start marker.
static void launch_begin(vvcr_ctx *ctx, Prepared &r, int L, int set, const std::vector<int> &refs) {
  const vvcr_pic_params &pp = r.pp;
  Lane &ln = ctx->lanes[L];
  hipStream_t s = ln.s;
  r.lane = L;
  r.set = set;
  for (int &k : r.kpics) k = 1;
  ln.tail_slot = pp.slot;
  ln.tail_seq = ++ctx->seq;
  for (int rs : refs)
    if (ctx->slot_w_set[rs] && ctx->slot_lane[rs] != L) VVCR_CHECK_HIP(hipStreamWaitEvent(s, ctx->slot_w[rs], 0));
  if (ctx->slot_w_set[pp.slot] && ctx->slot_lane[pp.slot] != L) VVCR_CHECK_HIP(hipStreamWaitEvent(s, ctx->slot_w[pp.slot], 0));
  for (int l = 0; l < ctx->nlane; l++)
    if (l != L && (ctx->slot_r_set[pp.slot] >> l & 1)) VVCR_CHECK_HIP(hipStreamWaitEvent(s, ctx->slot_r[pp.slot][l], 0));
  if (ctx->slot_x_set[pp.slot]) VVCR_CHECK_HIP(hipStreamWaitEvent(s, ctx->slot_x[pp.slot], 0));   // rows exported on a caller's stream
  VVCR_CHECK_HIP(hipStreamWaitEvent(s, r.up_done, 0));   // the picture's upload
  VVCR_CHECK_HIP(hipEventRecord(r.start, s));
}

static void launch_resid_stage(vvcr_ctx *ctx, Prepared &r) {
  const ScratchSet &S = ctx->lanes[r.lane].set[r.set];
  hipStream_t s = ctx->lanes[r.lane].s;
  const Rows rw = pic_rows(ctx, r.pp);
  KernelTimer t(r, K_RESID, s, ctx->timing);
  if (!r.zero_filled) {
    Planes3 clr{};
    for (int c = 0; c < 3; c++) clr.dst[c] = S.resi[c];
    clr.y0 = rw.own0; clr.y1 = rw.own1;
    launch_planes3(clr, s);
  }
  TbParams tp{};
  for (int c = 0; c < 3; c++) tp.out[c] = S.resi[c];
  tp.bd = ctx->sp.bit_depth;
  memcpy(tp.scan_off, ctx->scans.off, sizeof(tp.scan_off));
  memcpy(tp.lfnst_scan_off, ctx->scans.lfnst_off, sizeof(tp.lfnst_scan_off));
  launch_resid(tp, r.tb.p, r.n_tb, r.n_tb_small, r.coef.p, ctx->d_scans.p, s);
  VVCR_CHECK_HIP(hipGetLastError());
  r.launches[K_RESID] = r.n_tb > 0 ? 1 : 0;
}

// plain MC (k_mc) of n pictures of one lane in one launch; the first picture's record holds the kernel time
// and the algorithmic bytes of all of them
static void launch_plain_mc(vvcr_ctx *ctx, Prepared *const *rs, int n) {
  Prepared &r0 = *rs[0];
  hipStream_t s = ctx->lanes[r0.lane].s;
  McBatch b{};
  b.ref.p = ctx->d_ref_table.p;
  for (int c = 0; c < 3; c++) {
    b.ref.stride[c] = ctx->dpb[0][c].stride; b.ref.w[c] = ctx->dpb[0][c].w; b.ref.h[c] = ctx->dpb[0][c].h;
  }
  b.bd = ctx->sp.bit_depth;
  b.npic = n;
  double bytes = 0;
  int jobs = 0;
  const McClassTable *hct[MC_MAXPIC];
  for (int k = 0; k < n; k++) {
    b.pic[k] = make_mc_pic(ctx, *rs[k], rs[k]->lane, rs[k]->set);
    hct[k] = &rs[k]->mc_ct;
    bytes += rs[k]->alg_bytes[K_MC];
    jobs += rs[k]->n_mctile + rs[k]->n_basic;
    if (k) {
      rs[k]->ran[K_MC] = true;
      rs[k]->timed[K_MC] = false;
      rs[k]->launches[K_MC] = 0;
      rs[k]->kpics[K_MC] = 0;
    }
  }
  KernelTimer t(r0, K_MC, s, ctx->timing);
  launch_mc_batch(b, hct, s);
  VVCR_CHECK_HIP(hipGetLastError());
  r0.launches[K_MC] = jobs ? 1 : 0;
  r0.kpics[K_MC] = n;
  if (n > 1) {
    r0.alg_bytes[K_MC] = bytes;
    for (int k = 1; k < n; k++) rs[k]->alg_bytes[K_MC] = 0;
  }
}

// The accounting of one MC kernel group launched over the pictures rs[0, n) (frame batching): the first
// record holds the launch (its events, launch count, the pictures with work and the bytes of all)
static void batch_stats(Prepared *const *rs, int n, int k, int njobs_total, int pics_with_work) {
  Prepared &r0 = *rs[0];
  r0.launches[k] = njobs_total ? 1 : 0;
  if (n == 1) return;
  r0.kpics[k] = pics_with_work;
  double bytes = 0;
  for (int q = 0; q < n; q++) bytes += rs[q]->alg_bytes[k];
  r0.alg_bytes[k] = bytes;
  for (int q = 1; q < n; q++) {
    rs[q]->ran[k] = true;
    rs[q]->timed[k] = false;
    rs[q]->launches[k] = 0;
    rs[q]->kpics[k] = 0;
    rs[q]->alg_bytes[k] = 0;
  }
}

// DMVR / BDOF and affine MC of the pictures rs[0, n) on the first one's lane (one launch each over all of
// them: frame batching), then each picture's DMVR deltas' read-back on the copy stream (the lane goes on)
static void launch_mc_ext_stage(vvcr_ctx *ctx, Prepared *const *rs, int n) {
  Prepared &r0 = *rs[0];
  hipStream_t s = ctx->lanes[r0.lane].s;
  ExtBatch bb, ab;
  bb.npic = ab.npic = n;
  int nb = 0, na = 0, pb = 0, pa = 0;
  for (int q = 0; q < n; q++) {
    Prepared &r = *rs[q];
    bb.pic[q] = ab.pic[q] = make_mc_params(ctx, r, r.lane, r.set, r.wpt.p);
    bb.njobs[q] = r.n_bidir; bb.jobs[q] = r.mc_bidir.p; bb.dmvr[q] = r.dmvr.p;
    ab.njobs[q] = r.n_aff; ab.jobs[q] = r.aff_jobs.p; ab.pus[q] = r.aff_pu.p;
    nb += r.n_bidir; na += r.n_aff;
    pb += r.n_bidir > 0; pa += r.n_aff > 0;
  }
  {
    KernelTimer t(r0, K_MC_BIDIR, s, ctx->timing);
    launch_mc_bidir(bb, s);
    VVCR_CHECK_HIP(hipGetLastError());
  }
  batch_stats(rs, n, K_MC_BIDIR, nb, pb);
  {
    KernelTimer t(r0, K_MC_AFFINE, s, ctx->timing);
    launch_mc_affine(ab, s);
    VVCR_CHECK_HIP(hipGetLastError());
  }
  batch_stats(rs, n, K_MC_AFFINE, na, pa);
  for (int q = 0; q < n; q++) {
    Prepared &r = *rs[q];
    VVCR_CHECK_HIP(hipEventRecord(r.ev_mc, s));
    VVCR_CHECK_HIP(hipStreamWaitEvent(ctx->copy_stream, r.ev_mc, 0));
    if (r.n_dmvr > 0)
      VVCR_CHECK_HIP(hipMemcpyAsync(r.h_dmvr, r.dmvr.p, (size_t)r.n_dmvr * 2 * sizeof(int32_t), hipMemcpyDeviceToHost,
                                    ctx->copy_stream));
    VVCR_CHECK_HIP(hipEventRecord(r.mc_done, ctx->copy_stream));
  }
}

// intra / inter reconstruction, LMCS inverse, deblocking, SAO, ALF (stages of mask), the picture's final
// copy into its slot, and the dependency markers
static void launch_rest(vvcr_ctx *ctx, Prepared &r, uint32_t mask, const std::vector<int> &refs) {
  const vvcr_pic_params &pp = r.pp;
  const int L = r.lane;
  Lane &ln = ctx->lanes[L];
  const ScratchSet &S = ln.set[r.set];
  hipStream_t s = ln.s;
  const Rows rw = pic_rows(ctx, pp);
  if (mask & VVCR_STAGE_INTRA) {
    const IntraParams P = make_intra_params(ctx, r, L, r.set);
    {
      KernelTimer t(r, K_RECON, s, ctx->timing);
      launch_recon_inter(P, r.tiles.p, r.n_tiles, s);
      VVCR_CHECK_HIP(hipGetLastError());
      r.launches[K_RECON] = r.n_tiles ? 1 : 0;
    }
    {
      KernelTimer t(r, K_INTRA, s, ctx->timing);
      launch_intra(r.iparams.p + r.set * MAXLANE + L, r.ijobs.p, r.n_ijobs, r.ictu_list.p, r.ictu_start.p, r.n_ictu, r.idep_start.p,
                   r.ideps.p, r.istate.p, ctx->d_err, ctx->intra_wg, s);
      VVCR_CHECK_HIP(hipGetLastError());
      r.launches[K_INTRA] = r.n_ijobs ? 1 : 0;
    }
  }
  const DPlane *A = recon_planes(ctx, r, L, r.set);   // the picture until the last loop filter
  const DPlane *slot = ctx->dpb[pp.slot].data();
  if ((mask & VVCR_STAGE_LMCS_INV) && pp.lmcs_enabled) {
    launch_lmcs_inverse(A[0], r.lmcs_lut.p + 1024, rw.own0, rw.own1, s);   // back to the original domain before the loop filters
    VVCR_CHECK_HIP(hipGetLastError());
  }
  if ((mask & VVCR_STAGE_DBK) && (r.dbk_gpu ? r.n_dbcu > 0 : (r.dbk_counts[0] + r.dbk_counts[1] + r.dbk_counts[2] + r.dbk_counts[3]) > 0)) {
    DbkParams dp{};
    for (int c = 0; c < 3; c++) dp.pl[c] = A[c];
    dp.bd = ctx->sp.bit_depth;
    dp.beta_offset_div2 = pp.dbk_beta_offset_div2;
    dp.tc_offset_div2 = pp.dbk_tc_offset_div2;
    dp.ladf_num = std::min(5, pp.ladf_num);
    for (int k = 0; k < 5; k++) { dp.ladf_qp_offset[k] = pp.ladf_qp_offset[k]; dp.ladf_lower_bound[k] = pp.ladf_lower_bound[k]; }
    if (r.dbk_gpu) {
      DbkPlanArgs a;
      {
        KernelTimer t(r, K_DBKP, s, ctx->timing);
        a = dbk_plan_args(ctx, ln, r);
        launch_dbk_plan(a, s);
        r.launches[K_DBKP] = 1;
      }
      KernelTimer t(r, K_DBK, s, ctx->timing);
      const DbkSeg *segs[2][2] = {{a.out, a.out + a.cap}, {a.out + 2 * (size_t)a.cap, a.out + 3 * (size_t)a.cap}};
      // workgroups per list: at most one segment per item of the direction (both passes), 64 per workgroup
      // and pass, capped (they loop); a direction without items launches nothing
      int g[2][2];
      for (int d = 0; d < 2; d++) {
        const int n = std::min(a.cap, a.nitems[d] + a.nitems[2 + d]);
        g[d][0] = g[d][1] = std::min(1024, (n + 63) / 64);
      }
      launch_dbk(dp, segs, a.counts, g, s);
      r.launches[K_DBK] = 2;
    } else {
      KernelTimer t(r, K_DBK, s, ctx->timing);
      const DbkSeg *segs[2][2] = {{r.dbk.p, r.dbk.p + r.dbk_counts[0]},
                                  {r.dbk.p + r.dbk_counts[0] + r.dbk_counts[1], r.dbk.p + r.dbk_counts[0] + r.dbk_counts[1] + r.dbk_counts[2]}};
      int g[2][2];
      for (int d = 0; d < 2; d++)
        for (int k = 0; k < 2; k++) g[d][k] = (r.dbk_counts[2 * d + k] + 63) / 64;
      for (int d = 0; d < 2; d++)
        if (g[d][0] + g[d][1]) { g[d][0] = std::max(1, g[d][0]); g[d][1] = std::max(1, g[d][1]); }
      launch_dbk(dp, segs, r.dbk_cnt.p, g, s);
      r.launches[K_DBK] = (r.dbk_counts[0] + r.dbk_counts[1] > 0) + (r.dbk_counts[2] + r.dbk_counts[3] > 0);
    }
  }
  // SAO and ALF ping-pong between the slot and the lane's planes; the final picture always ends in the slot
  // (a picture with one of the two was reconstructed in the lane's planes: recon_tmp)
  const int ctu = 1 << ctx->sp.ctu_log2;
  const int wc = (ctx->sp.width + ctu - 1) / ctu, n = n_ctb(ctx->sp);
  bool inTmp = A != slot;
  if (r.have_sao && (mask & VVCR_STAGE_SAO)) {
    KernelTimer t(r, K_SAO, s, ctx->timing);
    SaoParams sp{};
    for (int c = 0; c < 3; c++) { sp.src[c] = inTmp ? S.tmp[c] : slot[c]; sp.dst[c] = inTmp ? slot[c] : S.tmp[c]; }
    sp.sao = r.sao.p; sp.bd = ctx->sp.bit_depth; sp.ctu = ctu; sp.wc = wc;
    sp.y0 = rw.sao0; sp.y1 = rw.sao1;
    sp.nb = r.n_lf_nb ? r.lf_nb.p : nullptr;
    sp.nvb[0] = pp.vb_disabled ? std::min(3, pp.num_vb_ver) : 0;
    sp.nvb[1] = pp.vb_disabled ? std::min(3, pp.num_vb_hor) : 0;
    for (int i = 0; i < 3; i++) { sp.vb[0][i] = pp.vb_ver[i]; sp.vb[1][i] = pp.vb_hor[i]; }
    launch_sao(sp, s);
    VVCR_CHECK_HIP(hipGetLastError());
    inTmp = !inTmp;
    r.launches[K_SAO] = 3;
  }
  if (r.have_alf && (mask & VVCR_STAGE_ALF)) {
    KernelTimer t(r, K_ALF, s, ctx->timing);
    AlfParams ap{};
    for (int c = 0; c < 3; c++) { ap.src[c] = inTmp ? S.tmp[c] : slot[c]; ap.dst[c] = inTmp ? slot[c] : S.tmp[c]; }
    ap.bd = ctx->sp.bit_depth; ap.ctu_log2 = ctx->sp.ctu_log2; ap.wc = wc; ap.nctb = n;
    ap.vb_luma = pp.alf_vb_luma; ap.vb_chroma = pp.alf_vb_chroma;
    for (int c = 0; c < 3; c++) ap.en[c] = pp.alf_en[c];
    ap.en[3] = pp.ccalf_en[0]; ap.en[4] = pp.ccalf_en[1];
    ap.luma_coef = r.alf_luma_coef.p; ap.luma_clip = r.alf_luma_clip.p;
    ap.chroma_coef = r.alf_chroma.p; ap.chroma_clip = r.alf_chroma.p + 56; ap.cc_coef = r.alf_cc.p;
    ap.ctb_en = r.alf_ctb.p; ap.ctb_alt = r.alf_ctb.p + 3 * n; ap.cc_ctl = r.alf_ctb.p + 6 * n;
    ap.ctb_set = r.alf_set.p;
    ap.y0 = rw.own0; ap.y1 = rw.own1;
    ap.nb = r.n_lf_nb ? r.lf_nb.p : nullptr;
    ap.pad = r.n_lf_nb == 2 * n ? r.lf_nb.p + n : nullptr;   // lf_ctb_neighbours appends the corner flags
    ap.nvb[0] = pp.vb_disabled ? std::min(3, pp.num_vb_ver) : 0;
    ap.nvb[1] = pp.vb_disabled ? std::min(3, pp.num_vb_hor) : 0;
    for (int i = 0; i < 3; i++) { ap.vb[0][i] = pp.vb_ver[i]; ap.vb[1][i] = pp.vb_hor[i]; }
    launch_alf(ap, s);
    VVCR_CHECK_HIP(hipGetLastError());
    inTmp = !inTmp;
    r.launches[K_ALF] = 1;
  }
  // a picture still in the lane's planes goes to its slot once, by the call that completes its stages (a
  // stage-by-stage picture's earlier calls leave it in the lane: its held lane keeps those planes)
  if (inTmp && ((r.staged | mask) & r.mask) == r.mask) {
    Planes3 cp{};
    for (int c = 0; c < 3; c++) { cp.dst[c] = slot[c]; cp.src[c] = S.tmp[c]; }
    cp.copy = 1;
    cp.y0 = rw.own0; cp.y1 = rw.own1;
    launch_planes3(cp, s);
  }
  VVCR_CHECK_HIP(hipEventRecord(r.done, s));
  VVCR_CHECK_HIP(hipEventRecord(ctx->slot_w[pp.slot], s));
  ctx->slot_w_set[pp.slot] = 1;
  ctx->slot_seq[pp.slot] = ln.tail_seq;
  ctx->slot_lane[pp.slot] = L;
  ctx->slot_r_set[pp.slot] = 0;
  for (int rs : refs)
    if (rs != pp.slot) {
      VVCR_CHECK_HIP(hipEventRecord(ctx->slot_r[rs][L], s));
      ctx->slot_r_set[rs] |= 1u << L;
    }
  r.launched = true;
  r.staged |= mask;
  if ((r.staged & r.mask) == r.mask) r.staged = 0;
  ln.held = r.staged ? &r : nullptr;
  ctx->last = &r;
}

// Device phase of one picture (the stages of `stages` it was prepared with).
static void launch(vvcr_ctx *ctx, Prepared &r, uint32_t stages = VVCR_STAGE_ALL) {
  const uint32_t mask = r.mask & stages;
  const std::vector<int> refs = ref_slots(r.pp);
  const int L = choose_lane(ctx, r, refs);
  launch_begin(ctx, r, L, 0, refs);
  if (mask & VVCR_STAGE_RESID) launch_resid_stage(ctx, r);
  if (mask & VVCR_STAGE_INTER) {
    Prepared *one = &r;
    launch_plain_mc(ctx, &one, 1);
    launch_mc_ext_stage(ctx, &one, 1);
  }
  launch_rest(ctx, r, mask, refs);
}

// Frame-batched launch of n independent pictures (every stage; none references another's slot, all write
// different slots) on one lane: picture k on the lane's scratch set k. Their residuals, then ONE k_mc launch
// for all of their plain MC, then picture by picture DMVR / BDOF, affine and the remaining stages. Each
// picture's dependency markers are recorded after its own last stage.
static void launch_batch(vvcr_ctx *ctx, Prepared *const *rs, int n) {
  if (n < 1 || n > MC_MAXPIC) throw VvcrError(VVCR_E_ARG, "a batched launch takes 1 .. " + std::to_string(MC_MAXPIC) + " pictures");
  if (ctx->nlane - ctx->nintra < 1) throw VvcrError(VVCR_E_STATE, "no inter lane");
  std::vector<std::vector<int>> refs(n);
  for (int k = 0; k < n; k++) {
    const Prepared &r = *rs[k];
    if (r.staged) throw VvcrError(VVCR_E_STATE, "a picture with pending stages cannot be launched in a batch");
    if ((r.mask & VVCR_STAGE_ALL) != VVCR_STAGE_ALL) throw VvcrError(VVCR_E_ARG, "batched pictures are prepared with every stage");
    refs[k] = ref_slots(r.pp);
    if (n > 1 && refs[k].empty()) throw VvcrError(VVCR_E_ARG, "batched pictures are inter pictures");
    for (int j = 0; j < k; j++) {
      if (rs[j] == rs[k] || rs[j]->pp.slot == r.pp.slot) throw VvcrError(VVCR_E_ARG, "batched pictures write different slots");
      if (std::find(refs[k].begin(), refs[k].end(), rs[j]->pp.slot) != refs[k].end() ||
          std::find(refs[j].begin(), refs[j].end(), r.pp.slot) != refs[j].end())
        throw VvcrError(VVCR_E_ARG, "a batched picture references another picture of its batch");
    }
  }
  if (n == 1) { launch(ctx, *rs[0]); return; }
  // the lane of the first picture (its newest reference's); a picture of the batch whose references
  // were written on other lanes waits for them by events like any picture
  const int L = choose_lane(ctx, *rs[0], refs[0]);
  Lane &ln = ctx->lanes[L];
  for (int k = 1; k < n; k++)
    if (!ln.set[k].resi[0].p || !ln.set[k].pred[0].p || !ln.set[k].tmp[0].p)
      throw VvcrError(VVCR_E_STATE, "lane without the scratch sets of a batched launch");
  for (int k = 0; k < n; k++) launch_begin(ctx, *rs[k], L, k, refs[k]);
  for (int k = 0; k < n; k++) launch_resid_stage(ctx, *rs[k]);
  launch_plain_mc(ctx, rs, n);
  launch_mc_ext_stage(ctx, rs, n);
  for (int k = 0; k < n; k++) launch_rest(ctx, *rs[k], rs[k]->mask, refs[k]);
}

extern "C" {

int vvcr_create(const vvcr_seq_params *sp, vvcr_ctx **out) {
  if (!sp || !out) return VVCR_E_ARG;
  *out = nullptr;
  if (sp->chroma_format != 1 || sp->bit_depth < 8 || sp->bit_depth > 10 || sp->width <= 0 || sp->height <= 0 ||
      sp->dpb_slots <= 0 || sp->dpb_slots > VVCR_MAX_SLOTS || sp->width % 8 || sp->height % 8 || sp->width < 16 || sp->ctu_log2 < 5 ||
      sp->ctu_log2 > 7) {
    g_create_error = "unsupported sequence parameters (4:2:0, 8..10 bit, size multiple of 8 and width >= 16, CTU 32..128, <= 256 DPB slots)";
    return VVCR_E_UNSUPPORTED;
  }
  auto ctx = std::make_unique<vvcr_ctx>();
  ctx->sp = *sp;
  try {
    VVCR_CHECK_HIP(hipSetDevice(sp->device));
    // the host side's large per-picture arrays in page-locked memory from now on: the upload DMAs straight
    // from them (Staging::add_big) instead of copying them into the staging buffer (VVCR_PIN_HOST=0: off)
    if (const char *e = getenv("VVCR_PIN_HOST"); !(e && e[0] == '0'))
      bigbuf::set_pinned_allocator(
          [](size_t n) -> void * {
            void *p = nullptr;
            return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
          },
          [](void *p) { (void)hipHostFree(p); });
    if (const char *e = getenv("VVCR_LANES")) ctx->nlane = std::max(2, std::min(MAXLANE, atoi(e)));
    ctx->nintra = ctx->nlane / 2;
    if (const char *e = getenv("VVCR_INTRA_LANES")) ctx->nintra = std::max(1, std::min(ctx->nlane - 1, atoi(e)));
    if (const char *e = getenv("VVCR_INTRA_WG")) ctx->intra_wg = std::max(0, atoi(e));
    VVCR_CHECK_HIP(hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, sp->device));
    // VVCR_CU_INTRA=N: the intra lanes' streams run on N CUs (spread evenly over the device), the B lanes'
    // on the others, so that the intra chain's waves never share a CU with B-picture kernels
    int cu_intra = 0;
    if (const char *e = getenv("VVCR_CU_INTRA")) cu_intra = std::max(0, std::min(ctx->n_cu - 1, atoi(e)));
    for (int l = 0; l < ctx->nlane; l++) {
      if (cu_intra > 0) {
        std::vector<uint32_t> mask((ctx->n_cu + 31) / 32, 0);
        for (int i = 0; i < ctx->n_cu; i++) {
          const bool in = (i * cu_intra) / ctx->n_cu != ((i + 1) * cu_intra) / ctx->n_cu;
          if (in == (l < ctx->nintra)) mask[i >> 5] |= 1u << (i & 31);
        }
        VVCR_CHECK_HIP(hipExtStreamCreateWithCUMask(&ctx->lanes[l].s, (uint32_t)mask.size(), mask.data()));
      } else {
        VVCR_CHECK_HIP(hipStreamCreateWithFlags(&ctx->lanes[l].s, hipStreamNonBlocking));
      }
    }
    ctx->stream = ctx->lanes[0].s;
    VVCR_CHECK_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    VVCR_CHECK_HIP(hipStreamCreateWithFlags(&ctx->upload_stream, hipStreamNonBlocking));
    const int W = sp->width, H = sp->height;
    ctx->dpb.resize(sp->dpb_slots);
    for (auto &s : ctx->dpb) {
      s[0] = alloc_plane(W, H);
      s[1] = alloc_plane(W / 2, H / 2);
      s[2] = alloc_plane(W / 2, H / 2);
    }
    {
      std::vector<const int16_t *> t;
      for (auto &s : ctx->dpb)
        for (int c = 0; c < 3; c++) t.push_back(s[c].p);
      ctx->d_ref_table.upload(t);
    }
    ctx->slot_w.assign(sp->dpb_slots, nullptr);
    ctx->slot_w_set.assign(sp->dpb_slots, 0);
    ctx->slot_r.assign(sp->dpb_slots, {});
    ctx->slot_r_set.assign(sp->dpb_slots, 0);
    ctx->slot_seq.assign(sp->dpb_slots, 0);
    ctx->slot_lane.assign(sp->dpb_slots, -1);
    ctx->slot_x.assign(sp->dpb_slots, nullptr);
    ctx->slot_x_set.assign(sp->dpb_slots, 0);
    if (const char *e = getenv("VVCR_LANE_POLICY")) ctx->lane_policy = atoi(e);
    for (int k = 0; k < sp->dpb_slots; k++) {
      VVCR_CHECK_HIP(hipEventCreateWithFlags(&ctx->slot_w[k], hipEventDisableTiming));
      VVCR_CHECK_HIP(hipEventCreateWithFlags(&ctx->slot_x[k], hipEventDisableTiming));
      for (int l = 0; l < MAXLANE; l++) VVCR_CHECK_HIP(hipEventCreateWithFlags(&ctx->slot_r[k][l], hipEventDisableTiming));
    }
    for (int l = 0; l < ctx->nlane; l++)
      for (int c = 0; c < 3; c++) {
        Lane &ln = ctx->lanes[l];
        int w = c ? W / 2 : W, h = c ? H / 2 : H;
        // set 0 on every lane; the batch sets on the B lanes (frame-batched launches take inter pictures
        // only). Allocated here, not at the first batch: the intra parameters of every prepared picture hold
        // every set's plane pointers (vvcr_prepare_*), so the planes must exist before any picture is prepared.
        for (int k = 0; k < (l >= ctx->nintra ? MC_MAXPIC : 1); k++) {
          ln.set[k].pred[c] = alloc_plane(w, h);
          ln.set[k].resi[c] = alloc_plane(w, h);
          ln.set[k].tmp[c] = alloc_plane(w, h);
        }
      }
    if (ctx->intra_wg <= 0) {
      // k_intra takes CTUs in wavefront order: the CTUs in flight are those of a few anti-diagonals
      // (x + 2y), so four diagonals' worth of workgroups keeps the wavefront busy (1080p, CTU 128: 32,
      // as fast in isolation as one per CU), and the other lanes' kernels get the CUs the idle workgroups
      // held: with five intra lanes in flight, 32 workgroups per launch 12.1 Gpx/s, 48 11.0
      const int ctu = 1 << sp->ctu_log2, wc = (sp->width + ctu - 1) / ctu, hc = (sp->height + ctu - 1) / ctu;
      ctx->intra_wg = std::min(ctx->n_cu, 4 * std::min(hc, (wc + 1) / 2));
    }
    VVCR_CHECK_HIP(hipMalloc(&ctx->d_err, 2 * sizeof(int32_t)));
    VVCR_CHECK_HIP(hipMemset(ctx->d_err, 0, 2 * sizeof(int32_t)));
    build_scan_tables(ctx->scans);
    ctx->d_scans.upload(ctx->scans.data);
    ctx->prepared.emplace_back(new Prepared());   // scratch record of vvcr_end_picture
  } catch (const VvcrError &e) {
    g_create_error = e.msg;
    return e.code;
  }
  *out = ctx.release();
  g_live_ctx.fetch_add(1);
  return VVCR_OK;
}

static void reap_pictures(bool all);
int vvcr_destroy(vvcr_ctx *ctx) {
  if (!ctx) return VVCR_E_ARG;
  reap_pictures(true);
  for (int l = 0; l < ctx->nlane; l++) (void)hipStreamSynchronize(ctx->lanes[l].s);
  ctx->prepared.clear();
  for (auto &s : ctx->dpb)
    for (auto &p : s) (void)hipFree(p.p);
  for (int l = 0; l < ctx->nlane; l++)
    for (int c = 0; c < 3; c++) {
      Lane &ln = ctx->lanes[l];
      for (ScratchSet &S : ln.set) { (void)hipFree(S.pred[c].p); (void)hipFree(S.resi[c].p); (void)hipFree(S.tmp[c].p); }
    }
  for (auto &e : ctx->slot_w) if (e) (void)hipEventDestroy(e);
  for (auto &e : ctx->slot_x) if (e) (void)hipEventDestroy(e);
  for (auto &a : ctx->slot_r)
    for (auto &e : a) if (e) (void)hipEventDestroy(e);
  if (ctx->d_err) (void)hipFree(ctx->d_err);
  if (ctx->rd_h) (void)hipHostFree(ctx->rd_h);
  if (ctx->rd_d) (void)hipFree(ctx->rd_d);
  for (int l = 0; l < ctx->nlane; l++) (void)hipStreamDestroy(ctx->lanes[l].s);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  if (ctx->upload_stream) (void)hipStreamDestroy(ctx->upload_stream);
  delete ctx;
  if (g_live_ctx.fetch_sub(1) == 1) bigbuf::trim_pinned();
  return VVCR_OK;
}

const char *vvcr_last_error(vvcr_ctx *ctx) { return ctx ? g_ctx_error.c_str() : g_create_error.c_str(); }

void *vvcr_stream(vvcr_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// ---- picture builder: shared by the context's current picture and the host-only vvcr_picture_* API
static void pic_begin(vvcr_picture &b, const vvcr_seq_params &sp, const vvcr_pic_params &pp) {
  if (pp.slot < 0 || pp.slot >= sp.dpb_slots) throw VvcrError(VVCR_E_ARG, "picture slot out of range");
  for (int l = 0; l < 2; l++) {
    if (pp.num_ref[l] < 0 || pp.num_ref[l] > VVCR_MAX_REF) throw VvcrError(VVCR_E_ARG, "bad num_ref");
    for (int i = 0; i < pp.num_ref[l]; i++)
      if (pp.ref_slot[l][i] < 0 || pp.ref_slot[l][i] >= sp.dpb_slots) throw VvcrError(VVCR_E_ARG, "ref slot out of range");
  }
  // virtual boundaries (at most 3 per direction, multiples of 8 inside the picture) and LADF intervals
  // (2..5, bounds increasing from 0): the filters' interval and boundary searches rely on both
  if (pp.vb_disabled) {
    for (int d = 0; d < 2; d++) {
      const int n = d ? pp.num_vb_hor : pp.num_vb_ver, lim = d ? sp.height : sp.width;
      const int32_t *v = d ? pp.vb_hor : pp.vb_ver;
      if (n < 0 || n > 3) throw VvcrError(VVCR_E_ARG, "virtual boundary count");
      for (int i = 0; i < n; i++)
        if (v[i] <= 0 || v[i] >= lim || (v[i] & 7)) throw VvcrError(VVCR_E_ARG, "virtual boundary position");
    }
  }
  if (pp.ladf_num) {
    if (pp.ladf_num < 2 || pp.ladf_num > 5 || pp.ladf_lower_bound[0] != 0) throw VvcrError(VVCR_E_ARG, "LADF intervals");
    for (int k = 1; k < pp.ladf_num; k++)
      if (pp.ladf_lower_bound[k] <= pp.ladf_lower_bound[k - 1]) throw VvcrError(VVCR_E_ARG, "LADF bounds not increasing");
  }
  b.sp = sp;
  b.pp = pp;
  b.desc.clear();
  b.submitted = false;
  b.have_sao = b.have_alf = false;   // loop-filter parameters are per picture
  b.planned = false;
  b.mask = 0;
}

static void pic_submit(vvcr_picture &b, const vvcr_cu *cu, int32_t ncu, const vvcr_pu *pu, int32_t npu, const vvcr_tu *tu,
                       int32_t ntu, const int32_t *coef, int64_t ncoef, const vvcr_motion *motion, const vvcr_geo *geo,
                       int32_t ngeo) {
  b.settle();
  if (ncu < 0 || npu < 0 || ntu < 0 || ncoef < 0 || ngeo < 0 || (ncu && !cu) || (npu && !pu) || (ntu && !tu) ||
      (ncoef && !coef) || (ngeo && !geo))
    throw VvcrError(VVCR_E_ARG, "bad descriptor array");
  auto &d = b.desc;
  d.cu.assign(cu, cu + ncu);
  d.pu.assign(pu, pu + npu);
  d.tu.assign(tu, tu + ntu);
  d.coef.assign(coef, coef + ncoef);
  d.coef_box.clear();   // the dense pool
  d.cu_map[0].clear();
  d.cu_map[1].clear();
  const size_t nm = (size_t)(b.sp.width / 4) * (b.sp.height / 4);
  if (motion) {
    d.motion.alloc(nm, false);
    for (size_t i = 0; i < nm; i++) d.motion[i] = to_rec(motion[i]);
  } else {
    d.motion.clear();
  }
  d.geo.assign(geo, geo + ngeo);
  b.planned = false;
  validate_descriptors(b.sp, b.pp, d);
  b.submitted = true;
}

// In-library producers (the host parser, vvcp_plan.cpp) hand their arrays over instead of copying them.
extern "C++" void vvcr_picture_adopt(vvcr_picture *pic, PictureDescriptors &&d) {
  if (!pic) throw VvcrError(VVCR_E_ARG, "null picture");
  pic->settle();
  pic->desc = std::move(d);
  pic->planned = false;
  validate_descriptors(pic->sp, pic->pp, pic->desc);
  pic->submitted = true;
}

static void pic_set_lf(vvcr_picture &b, const vvcr_sao *sao, const vvcr_alf *alf) {
  b.settle();
  const int n = n_ctb(b.sp);
  b.planned = false;
  b.have_sao = sao != nullptr;
  if (sao) b.h_sao.assign((const int32_t *)sao, (const int32_t *)sao + (size_t)n * 3 * 35);
  b.have_alf = false;
  if (alf) {
    if (alf->num_luma_sets < 16 || alf->num_luma_sets > 24) throw VvcrError(VVCR_E_ARG, "bad ALF luma set count");
    const size_t L = (size_t)alf->num_luma_sets * 25 * 13;
    b.h_alf_luma_coef.assign(alf->luma_coef, alf->luma_coef + L);
    b.h_alf_luma_clip.assign(alf->luma_clip, alf->luma_clip + L);
    b.h_alf_chroma.assign(alf->chroma_coef, alf->chroma_coef + 56);
    b.h_alf_chroma.insert(b.h_alf_chroma.end(), alf->chroma_clip, alf->chroma_clip + 56);
    b.h_alf_cc.assign(alf->cc_coef, alf->cc_coef + 64);
    auto &ctb = b.h_alf_ctb;
    ctb.assign(alf->ctb_en, alf->ctb_en + 3 * n);
    ctb.insert(ctb.end(), alf->ctb_alt, alf->ctb_alt + 3 * n);
    ctb.insert(ctb.end(), alf->cc_ctl, alf->cc_ctl + 2 * n);
    for (int i = 0; i < 3 * n; i++) if (ctb[3 * n + i] > 7) throw VvcrError(VVCR_E_ARG, "bad ALF chroma alternative");
    for (int i = 0; i < 2 * n; i++) if (ctb[6 * n + i] > 4) throw VvcrError(VVCR_E_ARG, "bad CC-ALF filter index");
    b.h_alf_set.assign(alf->ctb_filter_set, alf->ctb_filter_set + n);
    for (int v : b.h_alf_set) if (v < 0 || v >= alf->num_luma_sets) throw VvcrError(VVCR_E_ARG, "bad ALF filter set index");
    b.have_alf = true;
  }
}

// a free prepared-picture handle (> 0) holding a fresh record
static int32_t new_prepared(vvcr_ctx *ctx) {
  std::lock_guard<std::mutex> g(ctx->prepared_mu);
  int h = -1;
  for (size_t i = 1; i < ctx->prepared.size(); i++)
    if (!ctx->prepared[i]) { h = (int)i; break; }
  if (h < 0) { h = (int)ctx->prepared.size(); ctx->prepared.emplace_back(); }
  if (!ctx->spare.empty()) {
    ctx->prepared[h] = std::move(ctx->spare.back());
    ctx->spare.pop_back();
    ctx->prepared[h]->recycle();
  } else {
    ctx->prepared[h].reset(new Prepared());
  }
  return h;
}

static Prepared &get_prepared(vvcr_ctx *ctx, int32_t h) {
  std::lock_guard<std::mutex> g(ctx->prepared_mu);
  if (h <= 0 || h >= (int)ctx->prepared.size() || !ctx->prepared[h]) throw VvcrError(VVCR_E_ARG, "bad prepared-picture handle");
  return *ctx->prepared[h];
}

int vvcr_begin_picture(vvcr_ctx *ctx, const vvcr_pic_params *pp) {
  if (!ctx || !pp) return VVCR_E_ARG;
  API_BEGIN
  vvcr_seq_params sp = ctx->sp;
  pic_begin(ctx->cur, sp, *pp);
  ctx->in_picture = true;
  return VVCR_OK;
  API_END
}

int vvcr_submit(vvcr_ctx *ctx, const vvcr_cu *cu, int32_t ncu, const vvcr_pu *pu, int32_t npu, const vvcr_tu *tu,
                int32_t ntu, const int32_t *coef, int64_t ncoef, const vvcr_motion *motion, const vvcr_geo *geo,
                int32_t ngeo) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_submit outside begin/end picture");
  pic_submit(ctx->cur, cu, ncu, pu, npu, tu, ntu, coef, ncoef, motion, geo, ngeo);
  return VVCR_OK;
  API_END
}

int vvcr_set_loop_filter_params(vvcr_ctx *ctx, const vvcr_sao *sao, const vvcr_alf *alf) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_set_loop_filter_params outside begin/end picture");
  pic_set_lf(ctx->cur, sao, alf);
  return VVCR_OK;
  API_END
}

int vvcr_end_picture_stages(vvcr_ctx *ctx, uint32_t mask) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_end_picture without begin");
  Prepared *rp;
  {   // the table may be reallocated by new_prepared on another thread; the record at index 0 is not
    std::lock_guard<std::mutex> g(ctx->prepared_mu);
    rp = ctx->prepared[0].get();
  }
  Prepared &r = *rp;
  plan_picture(ctx->cur, mask);
  prepare(ctx, r, ctx->cur);
  {
    std::lock_guard<std::mutex> g(ctx->launch_mu);   // launch() updates the shared slot / lane state
    launch(ctx, r);
  }
  ctx->in_picture = false;
  return VVCR_OK;
  API_END
}

int vvcr_end_picture(vvcr_ctx *ctx) { return vvcr_end_picture_stages(ctx, VVCR_STAGE_ALL); }

int vvcr_prepare_picture(vvcr_ctx *ctx, uint32_t mask, int32_t *handle) {
  if (!ctx || !handle) return VVCR_E_ARG;
  API_BEGIN
  if (!ctx->in_picture) throw VvcrError(VVCR_E_STATE, "vvcr_prepare_picture without begin");
  plan_picture(ctx->cur, mask);
  const int32_t h = new_prepared(ctx);
  try {
    prepare(ctx, get_prepared(ctx, h), ctx->cur);
  } catch (...) {
    std::lock_guard<std::mutex> g(ctx->prepared_mu);
    ctx->prepared[h].reset();
    throw;
  }
  ctx->in_picture = false;
  *handle = h;
  return VVCR_OK;
  API_END
}

int vvcr_prepare_planned(vvcr_ctx *ctx, const vvcr_picture *pic, int32_t *handle) {
  if (!ctx || !pic || !handle) return VVCR_E_ARG;
  API_BEGIN
  const int32_t h = new_prepared(ctx);
  try {
    prepare(ctx, get_prepared(ctx, h), *pic);
  } catch (...) {
    std::lock_guard<std::mutex> g(ctx->prepared_mu);
    ctx->prepared[h].reset();
    throw;
  }
  *handle = h;
  return VVCR_OK;
  API_END
}

int vvcr_launch_picture(vvcr_ctx *ctx, int32_t handle) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> g(ctx->launch_mu);
  launch(ctx, get_prepared(ctx, handle));
  return VVCR_OK;
  API_END
}

int vvcr_launch_picture_stages(vvcr_ctx *ctx, int32_t handle, uint32_t stage_mask) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> g(ctx->launch_mu);
  launch(ctx, get_prepared(ctx, handle), stage_mask);
  return VVCR_OK;
  API_END
}

int vvcr_launch_pictures(vvcr_ctx *ctx, const int32_t *handles, int32_t n) {
  if (!ctx || !handles || n < 1 || n > MC_MAXPIC) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> g(ctx->launch_mu);
  Prepared *rs[MC_MAXPIC];
  for (int k = 0; k < n; k++) rs[k] = &get_prepared(ctx, handles[k]);
  launch_batch(ctx, rs, n);
  return VVCR_OK;
  API_END
}

int vvcr_release_picture(vvcr_ctx *ctx, int32_t handle) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  Prepared &r = get_prepared(ctx, handle);
  r.wait();
  std::lock_guard<std::mutex> lg(ctx->launch_mu);
  if (ctx->last == &r) ctx->last = nullptr;
  for (int l = 0; l < ctx->nlane; l++)
    if (ctx->lanes[l].held == &r) ctx->lanes[l].held = nullptr;
  std::lock_guard<std::mutex> g(ctx->prepared_mu);
  // released records keep their pinned staging and device arena for the next picture: pinning a 4K
  // picture's ~15 MB staging buffer takes milliseconds, and with the previous cap of 96 records the bench's
  // 272 pictures in flight re-allocated most of theirs every step (prepare 10.5 -> 4.1 ms per picture,
  // 3.76 -> 4.76 Gpx/s, gpurun_out/benchab_*). The pool never exceeds the peak number of records alive at
  // once; VVCR_SPARE caps it.
  static const size_t keep = getenv("VVCR_SPARE") ? (size_t)atol(getenv("VVCR_SPARE")) : SIZE_MAX;
  if (ctx->spare.size() < keep) ctx->spare.push_back(std::move(ctx->prepared[handle]));
  else ctx->prepared[handle].reset();
  return VVCR_OK;
  API_END
}

// ---- host-only picture builder (no device): see include/vvcr.h
#define PIC_BEGIN try {
#define PIC_END                                                  \
  }                                                              \
  catch (const VvcrError &e) { pic->err = e.msg; return e.code; } \
  catch (const std::exception &e) { pic->err = e.what(); return VVCR_E_STATE; }

int vvcr_picture_create(const vvcr_seq_params *sp, const vvcr_pic_params *pp, vvcr_picture **out) {
  if (!sp || !pp || !out) return VVCR_E_ARG;
  *out = nullptr;
  if (sp->chroma_format != 1 || sp->width <= 0 || sp->height <= 0 || sp->width % 8 || sp->height % 8 ||
      sp->bit_depth < 8 || sp->bit_depth > 10 ||
      sp->ctu_log2 < 5 || sp->ctu_log2 > 7 || sp->dpb_slots <= 0 || sp->dpb_slots > VVCR_MAX_SLOTS) {
    g_create_error = "unsupported sequence parameters (4:2:0, 8..10 bit, size multiple of 8, CTU 32..128)";
    return VVCR_E_UNSUPPORTED;
  }
  auto pic = std::make_unique<vvcr_picture>();
  try {
    pic_begin(*pic, *sp, *pp);
  } catch (const VvcrError &e) {
    g_create_error = e.msg;
    return e.code;
  }
  *out = pic.release();
  return VVCR_OK;
}

int vvcr_picture_submit(vvcr_picture *pic, const vvcr_cu *cu, int32_t ncu, const vvcr_pu *pu, int32_t npu, const vvcr_tu *tu,
                        int32_t ntu, const int32_t *coef, int64_t ncoef, const vvcr_motion *motion, const vvcr_geo *geo,
                        int32_t ngeo) {
  if (!pic) return VVCR_E_ARG;
  PIC_BEGIN
  pic_submit(*pic, cu, ncu, pu, npu, tu, ntu, coef, ncoef, motion, geo, ngeo);
  return VVCR_OK;
  PIC_END
}

int vvcr_picture_set_loop_filter_params(vvcr_picture *pic, const vvcr_sao *sao, const vvcr_alf *alf) {
  if (!pic) return VVCR_E_ARG;
  PIC_BEGIN
  pic_set_lf(*pic, sao, alf);
  return VVCR_OK;
  PIC_END
}

int vvcr_picture_plan(vvcr_picture *pic, uint32_t stage_mask) {
  if (!pic) return VVCR_E_ARG;
  PIC_BEGIN
  plan_picture(*pic, stage_mask);
  return VVCR_OK;
  PIC_END
}

int vvcr_picture_work_counts(const vvcr_picture *pic, int64_t *counts, int32_t n) {
  if (!pic || (!counts && n)) return VVCR_E_ARG;
  if (!pic->planned) return VVCR_E_STATE;
  const int64_t v[10] = {(int64_t)pic->wl.tb.size(), (int64_t)(pic->wl.mc_tile.size() + pic->wl.mc_basic.size() + pic->wl.mc_edge.size()), (int64_t)pic->wl.mc_bidir.size(),
                         (int64_t)pic->wl.aff_jobs.size(), (int64_t)pic->intra.inter_tiles.size(), (int64_t)pic->intra.jobs.size(),
                         (int64_t)pic->dbk.total(), (int64_t)pic->wl.n_dmvr, pic->wl.ref_y0, pic->wl.ref_y1};
  for (int k = 0; k < n && k < 10; k++) counts[k] = v[k];
  return 10;
}

// Diagnostics (host only): the raw 32-byte McJob records of a planned picture's inter work lists, which = 0
// 32x32 tiles, 1 small blocks, 2 DMVR / BDOF blocks (tools/mc_mix.py). Returns the number of records.
extern "C" int vvcr_debug_mc_jobs(const vvcr_picture *pic, int32_t which, void *out, int32_t cap) {
  if (!pic || which < 0 || which > 2 || (!out && cap)) return VVCR_E_ARG;
  if (!pic->planned) return VVCR_E_STATE;
  const auto &v = which == 0 ? pic->wl.mc_tile : which == 1 ? pic->wl.mc_basic : pic->wl.mc_bidir;
  const size_t n = std::min(v.size(), (size_t)std::max(cap, 0));
  if (n) std::memcpy(out, v.data(), n * sizeof(McJob));
  return (int)v.size();
}

// Diagnostics (host only): the planned deblocking segments, the four lists back to back (luma VER, chroma
// VER, luma HOR, chroma HOR) as the device receives them. Returns the number of segments.
extern "C" int vvcr_debug_dbk_segments(const vvcr_picture *pic, void *out, int32_t cap) {
  if (!pic || (!out && cap)) return VVCR_E_ARG;
  if (!pic->planned) return VVCR_E_STATE;
  const bigbuf::vec<DbkSeg> *parts[4] = {&pic->dbk.luma[0], &pic->dbk.chroma[0], &pic->dbk.luma[1], &pic->dbk.chroma[1]};
  int32_t n = 0;
  for (const auto *v : parts)
    for (const DbkSeg &sg : *v) {
      if (n < cap) static_cast<DbkSeg *>(out)[n] = sg;
      n++;
    }
  return n;
}

// Diagnostics (host only): the lengths of the host-planned deblocking lists (luma VER, chroma VER, luma HOR,
// chroma HOR) of vvcr_debug_dbk_segments.
extern "C" int vvcr_debug_dbk_list_sizes(const vvcr_picture *pic, int32_t *out) {
  if (!pic || !out) return VVCR_E_ARG;
  if (!pic->planned) return VVCR_E_STATE;
  out[0] = (int32_t)pic->dbk.luma[0].size(); out[1] = (int32_t)pic->dbk.chroma[0].size();
  out[2] = (int32_t)pic->dbk.luma[1].size(); out[3] = (int32_t)pic->dbk.chroma[1].size();
  return 4;
}

// Diagnostics (tests): the device deblocking planner run on a planned picture (planned with device
// deblocking, the default): its four segment lists back to back (luma VER, chroma VER, luma HOR, chroma
// HOR), each sorted by position, as vvcr_debug_dbk_segments gives the host planner's. Synchronous, on lane 0.
// Returns the number of segments.
extern "C" int vvcr_debug_dbk_gpu_segments(vvcr_ctx *ctx, const vvcr_picture *pic, void *out, int32_t cap) {
  if (!ctx || !pic || (!out && cap)) return VVCR_E_ARG;
  if (!pic->planned || !pic->dbk_gpu) return VVCR_E_STATE;
  API_BEGIN
  // the device planner takes the context's geometry (CTU size: the CTU-row rule of the P-side length)
  if (pic->sp.width != ctx->sp.width || pic->sp.height != ctx->sp.height || pic->sp.ctu_log2 != ctx->sp.ctu_log2)
    throw VvcrError(VVCR_E_ARG, "picture planned for another sequence geometry than the context's");
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  sync_lanes(ctx);
  Prepared r;
  r.pp = pic->pp;
  r.dbk_gpu = true;
  r.dbk_chroma_pass = pic->dbkg.chroma_pass;
  r.n_dbcu = (int)pic->dbkg.cu.size();
  r.n_dbtu = (int)pic->dbkg.tu.size();
  for (int k = 0; k < 4; k++) r.dbk_nitems[k] = pic->dbkg.nitems[k];
  r.dbcu.upload(pic->dbkg.cu);
  r.dbpu.upload(pic->dbkg.pu);
  r.dbtu.upload(pic->dbkg.tu);
  r.dbmot.upload(pic->desc.motion.data(), pic->desc.motion.size());
  r.n_dbmot = pic->desc.motion.size();
  Lane &ln = ctx->lanes[0];
  DbkPlanArgs a = dbk_plan_args(ctx, ln, r);
  int32_t cnt[4] = {0, 0, 0, 0};
  if (r.n_dbcu > 0) {
    launch_dbk_plan(a, ln.s);
    VVCR_CHECK_HIP(hipStreamSynchronize(ln.s));
    check_device_errors(ctx);
    VVCR_CHECK_HIP(hipMemcpy(cnt, a.counts, sizeof cnt, hipMemcpyDeviceToHost));
  }
  int32_t n = 0;
  std::vector<DbkSeg> v;
  for (int k = 0; k < 4; k++) {
    v.resize(cnt[k]);
    if (cnt[k]) VVCR_CHECK_HIP(hipMemcpy(v.data(), a.out + (size_t)k * a.cap, cnt[k] * sizeof(DbkSeg), hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const DbkSeg &x, const DbkSeg &y) { return x.y4 != y.y4 ? x.y4 < y.y4 : x.x4 < y.x4; });
    for (const DbkSeg &sg : v) {
      if (n < cap) static_cast<DbkSeg *>(out)[n] = sg;
      n++;
    }
  }
  return n;
  API_END
}

// Diagnostics (host only): the DPB slots the planned inter work lists read, one entry per (job, list) in
// job order (MC tiles and blocks, bi-directional blocks, affine PUs). Returns the number of entries.
extern "C" int vvcr_debug_mc_slots(const vvcr_picture *pic, int32_t *out, int32_t cap) {
  if (!pic || (!out && cap)) return VVCR_E_ARG;
  if (!pic->planned) return VVCR_E_STATE;
  int32_t n = 0;
  auto put = [&](int v) { if (n < cap) out[n] = v; n++; };
  for (const auto *v : {&pic->wl.mc_tile, &pic->wl.mc_basic, &pic->wl.mc_edge, &pic->wl.mc_bidir})
    for (const McJob &j : *v) {
      if (j.flags & MC_L0) put(j.slot[0]);
      if (j.flags & MC_L1) put(j.slot[1]);
    }
  for (const AffPu &u : pic->wl.aff_pu)
    for (int l = 0; l < 2; l++)
      if (u.l[l].present) put(u.l[l].slot);
  return n;
}

const char *vvcr_picture_last_error(const vvcr_picture *pic) { return pic ? pic->err.c_str() : g_create_error.c_str(); }

// Pictures destroyed while an upload still DMAs from their arrays: freed once its event has completed
// (the destroying thread does not wait for the upload queue).
static std::mutex g_grave_mu;
static std::vector<vvcr_picture *> g_grave;
static void reap_pictures(bool all) {
  std::vector<vvcr_picture *> done;
  {
    std::lock_guard<std::mutex> g(g_grave_mu);
    for (size_t i = 0; i < g_grave.size();) {
      if (all || hipEventQuery(g_grave[i]->up_ev) != hipErrorNotReady) {
        done.push_back(g_grave[i]);
        g_grave[i] = g_grave.back();
        g_grave.pop_back();
      } else {
        i++;
      }
    }
  }
  for (vvcr_picture *p : done) delete p;   // (settle() waits if `all` took a pending one)
}

int vvcr_picture_destroy(vvcr_picture *pic) {
  if (!pic) return VVCR_E_ARG;
  if (pic->up_pending && hipEventQuery(pic->up_ev) == hipErrorNotReady) {
    std::lock_guard<std::mutex> g(g_grave_mu);
    g_grave.push_back(pic);
  } else {
    delete pic;
  }
  reap_pictures(false);
  return VVCR_OK;
}

int vvcr_kernel_stats(vvcr_ctx *ctx, int32_t handle, vvcr_kernel_stat *out, int32_t n) {
  if (!ctx || (!out && n)) return VVCR_E_ARG;
  API_BEGIN
  Prepared *r = handle == 0 ? ctx->last : &get_prepared(ctx, handle);
  if (!r) throw VvcrError(VVCR_E_STATE, "no launched picture");
  r->wait();
  for (int k = 0; k < NK && k < n; k++) {
    vvcr_kernel_stat &s = out[k];
    memset(&s, 0, sizeof s);
    strncpy(s.name, kKernelNames[k], sizeof(s.name) - 1);
    s.launches = r->ran[k] ? r->launches[k] : 0;
    s.alg_bytes = r->ran[k] ? r->alg_bytes[k] : 0.0;
    s.pictures = r->kpics[k];
    float ms = 0;
    // a stage with nothing to launch has an empty event pair: no kernel time
    if (r->ran[k] && r->timed[k] && r->launches[k] > 0) VVCR_CHECK_HIP(hipEventElapsedTime(&ms, r->ev[k][0], r->ev[k][1]));
    s.ms = ms;
  }
  return NK;
  API_END
}

int vvcr_set_timing(vvcr_ctx *ctx, int32_t on) {
  if (!ctx) return VVCR_E_ARG;
  ctx->timing = on != 0;
  return VVCR_OK;
}

int vvcr_sync(vvcr_ctx *ctx) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  sync_lanes(ctx);
  check_device_errors(ctx);
  return VVCR_OK;
  API_END
}

int vvcr_last_stage_times(vvcr_ctx *ctx, float *ms, int32_t n) {
  if (!ctx || !ms) return VVCR_E_ARG;
  API_BEGIN
  float t = 0;
  if (ctx->last) {
    VVCR_CHECK_HIP(hipEventSynchronize(ctx->last->done));
    VVCR_CHECK_HIP(hipEventElapsedTime(&t, ctx->last->start, ctx->last->done));
  }
  if (n > 0) ms[0] = t;
  for (int k = 1; k < n && k < 8; k++) ms[k] = 0;
  if (ctx->last) {
    Prepared &r = *ctx->last;
    for (int k = 0; k < NK; k++) {
      if (!r.ran[k] || !r.timed[k]) continue;
      float v = 0;
      VVCR_CHECK_HIP(hipEventElapsedTime(&v, r.ev[k][0], r.ev[k][1]));
      const int st = kKernelStage[k] + 1;
      if (st < n) ms[st] += v;
    }
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
    case VVCR_BUF_PRED: return &ctx->lanes[ctx->last ? ctx->last->lane : 0].set[ctx->last ? ctx->last->set : 0].pred[comp];   // of the last launched picture
    case VVCR_BUF_RESI: return &ctx->lanes[ctx->last ? ctx->last->lane : 0].set[ctx->last ? ctx->last->set : 0].resi[comp];
    default: throw VvcrError(VVCR_E_ARG, "bad buffer id");
  }
}

int vvcr_read_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, int16_t *dst, int32_t dst_stride) {
  if (!ctx || !dst) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  DPlane *p = select_plane(ctx, buf, slot, comp);
  sync_lanes(ctx);
  VVCR_CHECK_HIP(hipMemcpy2DAsync(dst, dst_stride * 2, p->p, p->stride * 2, p->w * 2, p->h, hipMemcpyDeviceToHost, ctx->stream));
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  check_device_errors(ctx);
  return VVCR_OK;
  API_END
}

int vvcr_write_plane(vvcr_ctx *ctx, int32_t buf, int32_t slot, int32_t comp, const int16_t *src, int32_t src_stride) {
  if (!ctx || !src) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  DPlane *p = select_plane(ctx, buf, slot, comp);
  sync_lanes(ctx);
  VVCR_CHECK_HIP(hipMemcpy2DAsync(p->p, p->stride * 2, src, src_stride * 2, p->w * 2, p->h, hipMemcpyHostToDevice, ctx->stream));
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  check_device_errors(ctx);
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
  Prepared *r = ctx->last;
  const int cnt = r ? r->n_dmvr : 0;
  const int64_t m = std::min<int64_t>(n, cnt);
  if (m > 0) {
    hipStream_t s = ctx->lanes[r->lane].s;
    VVCR_CHECK_HIP(hipMemcpyAsync(out, r->dmvr.p, (size_t)m * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    VVCR_CHECK_HIP(hipStreamSynchronize(s));
  }
  return cnt;
  API_END
}

int vvcr_picture_dmvr_deltas(vvcr_ctx *ctx, int32_t handle, int32_t *out, int64_t n) {
  if (!ctx || (!out && n)) return VVCR_E_ARG;
  API_BEGIN
  if (n < 0) throw VvcrError(VVCR_E_ARG, "negative count");
  Prepared &r = get_prepared(ctx, handle);
  if (!r.launched) throw VvcrError(VVCR_E_STATE, "picture not launched");
  if (!(r.mask & VVCR_STAGE_INTER)) throw VvcrError(VVCR_E_STATE, "picture launched without its inter stage");
  const int64_t m = std::min<int64_t>(n, r.n_dmvr);
  // waits for this picture's inter stage and the copy of its deltas only, not for the rest of its lane;
  // reads only the record of this picture, so several host threads may call it at once
  VVCR_CHECK_HIP(hipEventSynchronize(r.mc_done));
  if (m > 0) std::memcpy(out, r.h_dmvr, (size_t)m * 2 * sizeof(int32_t));
  return r.n_dmvr;
  API_END
}

// ---------------------------------------------------------------------------------------------------
// Halo exchange of spatial shards (include/vvcr.h): rows of a DPB slot <-> packed device buffer
// ---------------------------------------------------------------------------------------------------
int64_t vvcr_rows_bytes(const vvcr_ctx *ctx, int32_t n) {
  if (!ctx || n < 0) return VVCR_E_ARG;
  const int64_t W = ctx->sp.width;
  return (int64_t)n * W * 2 + 2 * (int64_t)(n / 2) * (W / 2) * 2;
}

// On stream cs (the library's copy stream, or a caller's: the _async forms). Host-synchronous unless async:
// then the copy is ordered by events instead (an export is the slot's reader on cs, slot_x; an import its
// writer, slot_w with no lane, which every later launch touching the slot waits for).
static void rows_copy(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, char *dev, bool to_slot, hipStream_t cs = nullptr,
                      bool async = false) {
  if (slot < 0 || slot >= (int)ctx->dpb.size()) throw VvcrError(VVCR_E_ARG, "bad slot");
  if (y0 < 0 || n <= 0 || (y0 | n) & 1 || y0 + n > ctx->sp.height) throw VvcrError(VVCR_E_ARG, "rows outside the picture (y0, n even)");
  if (!dev) throw VvcrError(VVCR_E_ARG, "null buffer");
  if (!async) cs = ctx->copy_stream;
  if (ctx->slot_w_set[slot]) VVCR_CHECK_HIP(hipStreamWaitEvent(cs, ctx->slot_w[slot], 0));
  if (to_slot) {   // write after read: every lane's last reader of the slot, and an export on a caller's stream
    for (int l = 0; l < ctx->nlane; l++)
      if (ctx->slot_r_set[slot] >> l & 1) VVCR_CHECK_HIP(hipStreamWaitEvent(cs, ctx->slot_r[slot][l], 0));
    if (ctx->slot_x_set[slot]) VVCR_CHECK_HIP(hipStreamWaitEvent(cs, ctx->slot_x[slot], 0));
  }
  for (int c = 0; c < 3; c++) {
    const DPlane &pl = ctx->dpb[slot][c];
    const int s = c ? 1 : 0, r0 = y0 >> s, nr = n >> s;
    int16_t *plane = pl.p + (size_t)r0 * pl.stride;
    const size_t rowb = (size_t)pl.w * 2;
    if (to_slot) VVCR_CHECK_HIP(hipMemcpy2DAsync(plane, pl.stride * 2, dev, rowb, rowb, nr, hipMemcpyDeviceToDevice, cs));
    else VVCR_CHECK_HIP(hipMemcpy2DAsync(dev, rowb, plane, pl.stride * 2, rowb, nr, hipMemcpyDeviceToDevice, cs));
    dev += rowb * nr;
  }
  if (!async) {
    VVCR_CHECK_HIP(hipStreamSynchronize(cs));
  } else if (to_slot) {
    VVCR_CHECK_HIP(hipEventRecord(ctx->slot_w[slot], cs));
    ctx->slot_w_set[slot] = 1;
    ctx->slot_lane[slot] = -1;   // no lane: every lane's next launch on the slot waits
    ctx->slot_r_set[slot] = 0;   // earlier readers: the import waited on them
  } else {
    VVCR_CHECK_HIP(hipEventRecord(ctx->slot_x[slot], cs));
    ctx->slot_x_set[slot] = 1;
  }
}

// ---------------------------------------------------------------------------------------------------
// Output frames (include/vvcr.h vvcr_write_output)
// ---------------------------------------------------------------------------------------------------
static void check_output(const vvcr_ctx *ctx, const vvcr_output_params *op) {
  if (!op) throw VvcrError(VVCR_E_ARG, "null output parameters");
  const int W = ctx->sp.width, H = ctx->sp.height;
  if (op->file_bit_depth < 0 || op->file_bit_depth > 16) throw VvcrError(VVCR_E_ARG, "file bit depth outside 0..16");
  if (op->conf_left < 0 || op->conf_right < 0 || op->conf_top < 0 || op->conf_bottom < 0 ||
      ((op->conf_left | op->conf_right | op->conf_top | op->conf_bottom) & 1) || op->conf_left + op->conf_right >= W ||
      op->conf_top + op->conf_bottom >= H)
    throw VvcrError(VVCR_E_ARG, "conformance window: even luma offsets (4:2:0) inside the picture");
}

int64_t vvcr_output_bytes(const vvcr_ctx *ctx, const vvcr_output_params *op) {
  if (!ctx || !op) return VVCR_E_ARG;
  const int bd = op->file_bit_depth ? op->file_bit_depth : ctx->sp.bit_depth;
  const int64_t W = ctx->sp.width, H = ctx->sp.height;
  return (bd > 8 ? 2 : 1) * (W * H + 2 * (W / 2) * (H / 2));
}

int vvcr_write_output(vvcr_ctx *ctx, int32_t slot, const vvcr_output_params *op, void *dst, int32_t dst_on_device) {
  if (!ctx || !dst) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  if (slot < 0 || slot >= (int)ctx->dpb.size()) throw VvcrError(VVCR_E_ARG, "bad slot");
  check_output(ctx, op);
  const int64_t nb = vvcr_output_bytes(ctx, op);
  hipStream_t cs = ctx->copy_stream;
  if (ctx->slot_w_set[slot]) VVCR_CHECK_HIP(hipStreamWaitEvent(cs, ctx->slot_w[slot], 0));
  uint8_t *out = (uint8_t *)dst;
  if (!dst_on_device) {
    ctx->out_stage.ensure((size_t)nb);
    out = ctx->out_stage.p;
  }
  launch_output(ctx->dpb[slot], *op, ctx->sp.bit_depth, out, cs);
  VVCR_CHECK_HIP(hipGetLastError());
  if (!dst_on_device) VVCR_CHECK_HIP(hipMemcpyAsync(dst, out, (size_t)nb, hipMemcpyDeviceToHost, cs));
  VVCR_CHECK_HIP(hipStreamSynchronize(cs));
  return VVCR_OK;
  API_END
}

int vvcr_export_rows(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, void *dev_dst) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  rows_copy(ctx, slot, y0, n, (char *)dev_dst, false);
  return VVCR_OK;
  API_END
}

int vvcr_import_rows(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, const void *dev_src) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  rows_copy(ctx, slot, y0, n, (char *)dev_src, true);
  return VVCR_OK;
  API_END
}

int vvcr_export_rows_async(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, void *dev_dst, void *stream) {
  if (!ctx || !stream) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  rows_copy(ctx, slot, y0, n, (char *)dev_dst, false, (hipStream_t)stream, true);
  return VVCR_OK;
  API_END
}

int vvcr_import_rows_async(vvcr_ctx *ctx, int32_t slot, int32_t y0, int32_t n, const void *dev_src, void *stream) {
  if (!ctx || !stream) return VVCR_E_ARG;
  API_BEGIN
  std::lock_guard<std::mutex> launch_guard(ctx->launch_mu);
  rows_copy(ctx, slot, y0, n, (char *)dev_src, true, (hipStream_t)stream, true);
  return VVCR_OK;
  API_END
}

// ---------------------------------------------------------------------------------------------------
// Encoder RDO inner loop (include/vvcr.h): plans, runs on device pointers, host-pointer conveniences
// ---------------------------------------------------------------------------------------------------
static RdoPlan &get_rdo(vvcr_ctx *ctx, int32_t h) {
  if (h < 0 || h >= (int)ctx->rdo.size() || !ctx->rdo[h]) throw VvcrError(VVCR_E_ARG, "bad RDO plan handle");
  return *ctx->rdo[h];
}
static int32_t new_rdo(vvcr_ctx *ctx) {
  for (size_t i = 0; i < ctx->rdo.size(); i++)
    if (!ctx->rdo[i]) { ctx->rdo[i].reset(new RdoPlan()); return (int32_t)i; }
  ctx->rdo.emplace_back(new RdoPlan());
  return (int32_t)ctx->rdo.size() - 1;
}

int vvcr_rd_plan(vvcr_ctx *ctx, const vvcr_rd_block *blocks, int32_t n, int32_t *plan) {
  if (!ctx || !plan || n < 0 || (n && !blocks)) return VVCR_E_ARG;
  API_BEGIN
  std::vector<RdBlockDev> bd(n);
  std::vector<RdTile> tl[RD_KINDS];
  for (int i = 0; i < n; i++) {
    const vvcr_rd_block &b = blocks[i];
    int tw, th;
    const int k = rd_kind(b.width, b.height, tw, th);
    if (k < 0 || b.width <= 0 || b.height <= 0 || b.width > 128 || b.height > 128)
      throw VvcrError(VVCR_E_ARG, "RDO block size not supported by xGetHADs (even sizes up to 128)");
    bd[i] = RdBlockDev{b.org_off, b.cur_off, b.org_stride, b.cur_stride};
    for (int y = 0; y < b.height; y += th)
      for (int x = 0; x < b.width; x += tw) tl[k].push_back(RdTile{i, (int16_t)x, (int16_t)y});
  }
  const int32_t h = new_rdo(ctx);
  RdoPlan &P = *ctx->rdo[h];
  P.nblocks = n;
  P.blocks.upload(bd);
  for (int k = 0; k < RD_KINDS; k++) { P.tiles[k].upload(tl[k]); P.ntiles[k] = (int)tl[k].size(); }
  *plan = h;
  return VVCR_OK;
  API_END
}

int vvcr_rd_run(vvcr_ctx *ctx, int32_t plan, const int16_t *org_dev, const int16_t *cur_dev, uint32_t *sad_dev,
                uint32_t *satd_dev) {
  if (!ctx || !org_dev || !cur_dev || !sad_dev || !satd_dev) return VVCR_E_ARG;
  API_BEGIN
  RdoPlan &P = get_rdo(ctx, plan);
  if (P.fwd) throw VvcrError(VVCR_E_ARG, "plan is a forward-transform plan");
  hipStream_t s = ctx->stream;
  VVCR_CHECK_HIP(hipMemsetAsync(sad_dev, 0, (size_t)P.nblocks * 4, s));
  VVCR_CHECK_HIP(hipMemsetAsync(satd_dev, 0, (size_t)P.nblocks * 4, s));
  for (int k = 0; k < RD_KINDS; k++)
    launch_rd_tiles(k, org_dev, cur_dev, P.tiles[k].p, P.ntiles[k], P.blocks.p, sad_dev, satd_dev, s);
  VVCR_CHECK_HIP(hipGetLastError());
  return VVCR_OK;
  API_END
}

int vvcr_fwd_plan(vvcr_ctx *ctx, const vvcr_fwd_block *blocks, int32_t n, int32_t bit_depth, int32_t *plan) {
  if (!ctx || !plan || n < 0 || (n && !blocks)) return VVCR_E_ARG;
  API_BEGIN
  if (bit_depth < 8 || bit_depth > 10) throw VvcrError(VVCR_E_UNSUPPORTED, "bit depth 8..10");
  std::vector<FwdBlockDev> fb(n);
  int64_t total = 0;
  for (int i = 0; i < n; i++) {
    const vvcr_fwd_block &b = blocks[i];
    const bool pow2 = b.width >= 4 && b.height >= 4 && !(b.width & (b.width - 1)) && !(b.height & (b.height - 1));
    const int maxH = b.tr_hor == 0 ? 64 : 32, maxV = b.tr_ver == 0 ? 64 : 32;
    if (!pow2 || b.width > maxH || b.height > maxV || b.tr_hor < 0 || b.tr_hor > 2 || b.tr_ver < 0 || b.tr_ver > 2)
      throw VvcrError(VVCR_E_ARG, "forward transform block: power-of-two 4..64 (DCT2) / 4..32 (DST7, DCT8)");
    fb[i] = FwdBlockDev{b.src_off, b.dst_off, b.src_stride, (uint8_t)b.width, (uint8_t)b.height, (uint8_t)b.tr_hor,
                        (uint8_t)b.tr_ver, b.lfnst ? 1 : 0};
    total = std::max<int64_t>(total, b.dst_off + (int64_t)b.width * b.height);
  }
  // group by class: one launch per class (vvcr_rdo.hip launch_fwd_tr)
  auto key = [](const FwdBlockDev &b) { return (b.w << 24) | (b.h << 16) | (b.tr_hor << 8) | (b.tr_ver << 4) | b.lfnst; };
  std::stable_sort(fb.begin(), fb.end(), [&](const FwdBlockDev &a, const FwdBlockDev &b) { return key(a) < key(b); });
  const int32_t h = new_rdo(ctx);
  RdoPlan &P = *ctx->rdo[h];
  P.fwd = true;
  P.nblocks = n;
  P.bd = bit_depth;
  P.coef_total = total;
  for (int i = 0; i < n;) {
    int j = i;
    while (j < n && key(fb[j]) == key(fb[i])) j++;
    P.classes.push_back({i, j - i, fb[i].w, fb[i].h, fb[i].tr_hor, fb[i].tr_ver, fb[i].lfnst});
    i = j;
  }
  P.fblocks.upload(fb);
  *plan = h;
  return VVCR_OK;
  API_END
}

int vvcr_fwd_run(vvcr_ctx *ctx, int32_t plan, const int16_t *resi_dev, int32_t *coef_dev) {
  if (!ctx || !resi_dev || !coef_dev) return VVCR_E_ARG;
  API_BEGIN
  RdoPlan &P = get_rdo(ctx, plan);
  if (!P.fwd) throw VvcrError(VVCR_E_ARG, "plan is a distortion plan");
  for (const RdoPlan::Cls &c : P.classes)
    launch_fwd_tr(resi_dev, coef_dev, P.fblocks.p + c.start, c.n, P.bd, c.w, c.h, c.trh, c.trv, c.lfnst, ctx->stream);
  VVCR_CHECK_HIP(hipGetLastError());
  return VVCR_OK;
  API_END
}

int vvcr_rdo_release(vvcr_ctx *ctx, int32_t plan) {
  if (!ctx) return VVCR_E_ARG;
  API_BEGIN
  get_rdo(ctx, plan);
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  ctx->rdo[plan].reset();
  return VVCR_OK;
  API_END
}

int vvcr_rd_dist(vvcr_ctx *ctx, const vvcr_rd_block *blocks, int32_t n, const int16_t *org, int64_t norg,
                 const int16_t *cur, int64_t ncur, uint32_t *sad, uint32_t *satd) {
  if (!ctx || !org || !cur || !sad || !satd || norg <= 0 || ncur <= 0 || n < 0 || (n && !blocks)) return VVCR_E_ARG;
  API_BEGIN
  // the same tiling as vvcr_rd_plan, written straight into the staging span: [sad | satd] zeroed (the
  // kernels accumulate into them), block records, tiles by kind, original and prediction samples. The
  // per-call cost is then one upload, the launches, one read-back and one synchronisation (the plan /
  // run / release route allocates and frees device memory per call: ~137 us per 8x8 SATD in the
  // EncoderApp binding, profiles/r06/enc_dropin_speed_r06x.json)
  int ntl[RD_KINDS] = {};
  for (int i = 0; i < n; i++) {
    const vvcr_rd_block &b = blocks[i];
    int tw, th;
    const int k = rd_kind(b.width, b.height, tw, th);
    if (k < 0 || b.width <= 0 || b.height <= 0 || b.width > 128 || b.height > 128)
      throw VvcrError(VVCR_E_ARG, "RDO block size not supported by xGetHADs (even sizes up to 128)");
    const int64_t eo = b.org_off + (int64_t)(b.height - 1) * b.org_stride + b.width, ec = b.cur_off + (int64_t)(b.height - 1) * b.cur_stride + b.width;
    if (b.org_off < 0 || b.cur_off < 0 || eo > norg || ec > ncur) throw VvcrError(VVCR_E_ARG, "RDO block outside its sample pool");
    ntl[k] += ((b.width + tw - 1) / tw) * ((b.height + th - 1) / th);
  }
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  const size_t o_res = 0, o_blk = al(2 * (size_t)n * 4);
  size_t o_tl[RD_KINDS], off = o_blk + al((size_t)n * sizeof(RdBlockDev));
  for (int k = 0; k < RD_KINDS; k++) { o_tl[k] = off; off += al((size_t)ntl[k] * sizeof(RdTile)); }
  const size_t o_org = off, o_cur = o_org + al((size_t)norg * 2), total = o_cur + al((size_t)ncur * 2);
  std::lock_guard<std::mutex> lk(ctx->rd_mu);
  if (total > ctx->rd_cap) {
    if (ctx->rd_h) VVCR_CHECK_HIP(hipHostFree(ctx->rd_h));
    if (ctx->rd_d) VVCR_CHECK_HIP(hipFree(ctx->rd_d));
    ctx->rd_h = ctx->rd_d = nullptr;
    ctx->rd_cap = 0;
    const size_t c = std::max<size_t>(total, 1 << 20);
    VVCR_CHECK_HIP(hipHostMalloc((void **)&ctx->rd_h, c, hipHostMallocDefault));
    VVCR_CHECK_HIP(hipMalloc((void **)&ctx->rd_d, c));
    ctx->rd_cap = c;
  }
  char *h = ctx->rd_h, *d = ctx->rd_d;
  std::memset(h + o_res, 0, 2 * (size_t)n * 4);
  RdBlockDev *bd = (RdBlockDev *)(h + o_blk);
  RdTile *tl[RD_KINDS];
  int fill[RD_KINDS] = {};
  for (int k = 0; k < RD_KINDS; k++) tl[k] = (RdTile *)(h + o_tl[k]);
  for (int i = 0; i < n; i++) {
    const vvcr_rd_block &b = blocks[i];
    int tw, th;
    const int k = rd_kind(b.width, b.height, tw, th);
    bd[i] = RdBlockDev{b.org_off, b.cur_off, b.org_stride, b.cur_stride};
    for (int y = 0; y < b.height; y += th)
      for (int x = 0; x < b.width; x += tw) tl[k][fill[k]++] = RdTile{i, (int16_t)x, (int16_t)y};
  }
  std::memcpy(h + o_org, org, (size_t)norg * 2);
  std::memcpy(h + o_cur, cur, (size_t)ncur * 2);
  hipStream_t st = ctx->stream;
  VVCR_CHECK_HIP(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, st));
  uint32_t *dsad = (uint32_t *)(d + o_res), *dsatd = dsad + n;
  for (int k = 0; k < RD_KINDS; k++)
    launch_rd_tiles(k, (const int16_t *)(d + o_org), (const int16_t *)(d + o_cur), (const RdTile *)(d + o_tl[k]), ntl[k],
                    (const RdBlockDev *)(d + o_blk), dsad, dsatd, st);
  VVCR_CHECK_HIP(hipGetLastError());
  VVCR_CHECK_HIP(hipMemcpyAsync(h + o_res, d + o_res, 2 * (size_t)n * 4, hipMemcpyDeviceToHost, st));
  VVCR_CHECK_HIP(hipStreamSynchronize(st));
  std::memcpy(sad, h + o_res, (size_t)n * 4);
  std::memcpy(satd, h + o_res + (size_t)n * 4, (size_t)n * 4);
  return VVCR_OK;
  API_END
}

int vvcr_fwd_transform(vvcr_ctx *ctx, const vvcr_fwd_block *blocks, int32_t n, int32_t bit_depth, const int16_t *resi,
                       int64_t nresi, int32_t *coef, int64_t ncoef) {
  if (!ctx || !resi || !coef || nresi <= 0 || ncoef <= 0) return VVCR_E_ARG;
  int32_t plan = -1;
  int r = vvcr_fwd_plan(ctx, blocks, n, bit_depth, &plan);
  if (r) return r;
  API_BEGIN
  for (int i = 0; i < n; i++) {
    const vvcr_fwd_block &b = blocks[i];
    const int64_t er = b.src_off + (int64_t)(b.height - 1) * b.src_stride + b.width;
    if (b.src_off < 0 || b.dst_off < 0 || er > nresi || b.dst_off + (int64_t)b.width * b.height > ncoef)
      throw VvcrError(VVCR_E_ARG, "transform block outside its buffer");
  }
  DevVec<int16_t> rd;
  DevVec<int32_t> cd;
  rd.upload(resi, nresi);
  cd.ensure(ncoef + 1);
  const int rr = vvcr_fwd_run(ctx, plan, rd.p, cd.p);
  if (rr) { vvcr_rdo_release(ctx, plan); return rr; }
  VVCR_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  VVCR_CHECK_HIP(hipMemcpy(coef, cd.p, (size_t)ncoef * 4, hipMemcpyDeviceToHost));
  vvcr_rdo_release(ctx, plan);
  return VVCR_OK;
  API_END
}

}  // extern "C"

