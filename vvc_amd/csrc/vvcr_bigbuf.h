// vvcr_bigbuf.h — a process-wide cache of large host buffers for the per-picture arrays of the host
// side (parser rows and coefficient pool, motion fields, planner maps and work lists). Every picture
// allocates and frees the same few dozen arrays of similar sizes; served from fresh memory each time,
// their first touches are page faults that cost more than the work on them (4K: ~100 MB per picture).
// Blocks of at least kMin bytes are rounded up to a size class (eighths of a power of two) and, when
// freed, kept for the next request of that class, up to cache_cap() bytes in all.
// With a pinned allocator installed (the reconstruction context does it: hipHostMalloc), new blocks of at
// least kPinMin bytes are page-locked, so that the upload can DMA straight from them (is_pinned) instead of
// copying them into its staging buffer first.
#pragma once
#include <atomic>
#include <unordered_set>
#include <unistd.h>
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

namespace bigbuf {

constexpr size_t kMin = 256 << 10;
// the cache's capacity: VVCR_BIGBUF_CAP_GB (default 24: with 16 decodes in flight the freed blocks of
// the pictures between their parse and their upload exceed 3 GB; a smaller cache then frees and
// re-allocates page-locked blocks, whose allocation is slow and serialised in the runtime — 4K bench
// 5.56 Gpx/s unpinned at 3 GB, 6.38 pinned at 24 GB, 3.41 pinned at 3 GB), bounded by the host memory per
// process: a node's ranks (LOCAL_WORLD_SIZE) share its RAM
inline size_t cache_cap() {
  static const size_t cap = [] {
    if (const char *e = std::getenv("VVCR_BIGBUF_CAP_GB")) return (size_t)std::atoll(e) << 30;
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    const char *lw = std::getenv("LOCAL_WORLD_SIZE");
    if (!lw) lw = std::getenv("WORLD_SIZE");
    const size_t ranks = lw && std::atoi(lw) > 0 ? (size_t)std::atoi(lw) : 1;
    const size_t share = pages > 0 && psz > 0 ? (size_t)pages * (size_t)psz / (4 * ranks) : (size_t(24) << 30);
    return std::min(size_t(24) << 30, share);
  }();
  return cap;
}
constexpr size_t kPinMin = 1 << 20;

using PinAlloc = void *(*)(size_t);
using PinFree = void (*)(void *);

inline size_t size_class(size_t n) {
  size_t p = 1;
  while (p < n) p <<= 1;
  const size_t step = p >> 3;   // eighths of the power of two at or above n
  return (n + step - 1) / step * step;
}

struct Cache {
  std::mutex mu;
  std::unordered_map<size_t, std::vector<void *>> free;
  size_t cached = 0;
  std::atomic<PinAlloc> pin_alloc{nullptr};
  PinFree pin_free = nullptr;
  std::unordered_set<const void *> pinned;   // blocks from pin_alloc
  static Cache &get() {
    static Cache *c = new Cache();   // never destroyed: buffers may be released during static teardown
    return *c;
  }
};

inline void *alloc(size_t bytes) {
  if (bytes < kMin) {
    void *p = std::malloc(bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    return p;
  }
  const size_t sc = size_class(bytes);
  Cache &c = Cache::get();
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.free.find(sc);
    if (it != c.free.end() && !it->second.empty()) {
      void *p = it->second.back();
      it->second.pop_back();
      c.cached -= sc;
      return p;
    }
  }
  if (sc >= kPinMin) {
    if (PinAlloc pa = c.pin_alloc.load(std::memory_order_acquire)) {
      if (void *p = pa(sc)) {
        std::lock_guard<std::mutex> g(c.mu);
        c.pinned.insert(p);
        return p;
      }
    }
  }
  void *p = std::malloc(sc);
  if (!p) throw std::bad_alloc();
  return p;
}

// installs the allocator of page-locked blocks (once; later calls are ignored)
inline void set_pinned_allocator(PinAlloc a, PinFree f) {
  Cache &c = Cache::get();
  std::lock_guard<std::mutex> g(c.mu);
  if (c.pin_alloc.load()) return;
  c.pin_free = f;
  c.pin_alloc.store(a, std::memory_order_release);
}

// whether p is the start of a page-locked block
inline bool is_pinned(const void *p) {
  Cache &c = Cache::get();
  if (!p || !c.pin_alloc.load(std::memory_order_acquire)) return false;
  std::lock_guard<std::mutex> g(c.mu);
  return c.pinned.count(p) != 0;
}

inline void release(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < kMin) {
    std::free(p);
    return;
  }
  const size_t sc = size_class(bytes);
  Cache &c = Cache::get();
  PinFree pf = nullptr;
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (c.cached + sc <= cache_cap()) {
      c.free[sc].push_back(p);
      c.cached += sc;
      return;
    }
    if (c.pinned.erase(p)) pf = c.pin_free;
  }
  if (pf) pf(p);
  else std::free(p);
}

// frees every cached (unused) page-locked block: the reconstruction context calls it when its last
// instance is destroyed, so a process that stops decoding does not keep gigabytes of pinned memory that
// co-located processes and the page cache could use. Blocks still in use are freed on their release as usual.
inline void trim_pinned() {
  Cache &c = Cache::get();
  std::vector<void *> drop;
  PinFree pf = nullptr;
  {
    std::lock_guard<std::mutex> g(c.mu);
    pf = c.pin_free;
    for (auto &kv : c.free) {
      auto &v = kv.second;
      for (size_t i = 0; i < v.size();) {
        if (c.pinned.erase(v[i])) {
          drop.push_back(v[i]);
          c.cached -= kv.first;
          v[i] = v.back();
          v.pop_back();
        } else {
          i++;
        }
      }
    }
  }
  if (pf)
    for (void *p : drop) pf(p);
}

// std::vector allocator drawing large arrays from the cache
template <class T>
struct Alloc {
  using value_type = T;
  Alloc() = default;
  template <class U> Alloc(const Alloc<U> &) {}
  T *allocate(size_t n) { return static_cast<T *>(alloc(n * sizeof(T))); }
  void deallocate(T *p, size_t n) { release(p, n * sizeof(T)); }
  template <class U> bool operator==(const Alloc<U> &) const { return true; }
  template <class U> bool operator!=(const Alloc<U> &) const { return false; }
};

template <class T> using vec = std::vector<T, Alloc<T>>;

// an array of trivially copyable T from the cache, NOT initialised unless asked (alloc(n, true) zeroes)
template <class T>
struct raw {
  T *p = nullptr;
  size_t n = 0;
  raw() = default;
  raw(const raw &) = delete;
  raw &operator=(const raw &) = delete;
  raw(raw &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  raw &operator=(raw &&o) noexcept {
    if (this != &o) { reset(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~raw() { reset(); }
  void reset() { release(p, n * sizeof(T)); p = nullptr; n = 0; }
  void clear() { reset(); }
  void alloc(size_t count, bool zero) {
    reset();
    p = static_cast<T *>(bigbuf::alloc(count * sizeof(T)));
    n = count;
    if (zero) std::memset((void *)p, 0, count * sizeof(T));
  }
  // takes over the buffer of an array of a type with the same size (a layout-compatible record)
  template <class U>
  void adopt(raw<U> &&o) {
    static_assert(sizeof(U) == sizeof(T), "adopt: element sizes differ");
    reset();
    p = reinterpret_cast<T *>(o.p);
    n = o.n;
    o.p = nullptr;
    o.n = 0;
  }
  void assign(const T *b, const T *e) {
    alloc((size_t)(e - b), false);
    if (n) std::memcpy((void *)p, b, n * sizeof(T));
  }
  T *data() { return p; }
  const T *data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
};

}  // namespace bigbuf
