// vvcr_bigbuf.h — a process-wide cache of large host buffers for the per-picture arrays of the host
// side (parser rows and coefficient pool, motion fields, planner maps and work lists). Every picture
// allocates and frees the same few dozen arrays of similar sizes; served from fresh memory each time,
// their first touches are page faults that cost more than the work on them (4K: ~100 MB per picture).
// Blocks of at least kMin bytes are rounded up to a size class (eighths of a power of two) and, when
// freed, kept for the next request of that class, up to kCacheCap bytes in all.
#pragma once
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

namespace bigbuf {

constexpr size_t kMin = 256 << 10;
constexpr size_t kCacheCap = size_t(3) << 30;

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
  void *p = std::malloc(sc);
  if (!p) throw std::bad_alloc();
  return p;
}

inline void release(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < kMin) {
    std::free(p);
    return;
  }
  const size_t sc = size_class(bytes);
  Cache &c = Cache::get();
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (c.cached + sc <= kCacheCap) {
      c.free[sc].push_back(p);
      c.cached += sc;
      return;
    }
  }
  std::free(p);
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
