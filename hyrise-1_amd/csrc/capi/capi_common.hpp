// Shared host-side plumbing of the C-ABI translation units: error reporting, workspace carving and per-kernel
// HIP-event timing. State lives in hyrise_amd.hip; every other TU only includes this header.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hyrise_amd.h"

namespace hyc {

extern thread_local std::string g_last_error;

inline hy_status fail(hy_status code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HY_HIP(call)                                                                                       \
  do {                                                                                                     \
    hipError_t e_ = (call);                                                                                \
    if (e_ != hipSuccess) return ::hyc::fail(HY_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline hipStream_t S(hy_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Chunk kinds every row-wise reader (join, aggregate, projection, column compare) takes: values and dictionaries.
// Compressed RunLength / FrameOfReference chunks are scanned only (hy_table_scan family); the others read their
// decoded value mirrors.
inline bool row_readable(const hy_column_chunk& c) {
  return c.size == 0 || c.kind == HY_COL_VALUE || c.kind == HY_COL_DICT;
}

inline bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return cap != hipStreamCaptureStatusNone;
}

// Host -> device copies of the descriptors a call builds on the host (chunk / side / column tables, offsets): staged
// through a per-thread pinned ring so that hipMemcpyAsync is a real asynchronous DMA (a pageable source makes the
// runtime stage it synchronously, at a fraction of the bandwidth - measurable with tens of thousands of chunks), and
// so that the source may go out of scope right after the call. Every copy re-records its stream's event (one event
// per (stream, device) the thread has staged on: stream order makes the latest record cover the earlier copies); when
// the ring wraps it waits on those events only - the ring's own DMAs - instead of the whole device, so other threads'
// operator streams are not stalled, and copies staged for another GPU are covered too.
struct PinnedRing;
// Every thread's ring, so that hy_stream_destroy can drop the fences of a stream it destroys from all of them (a fence
// event whose stream is gone is not safe to wait on: the runtime follows the event to its recording stream).
struct RingRegistry {
  std::mutex m;
  std::vector<PinnedRing*> rings;
};
inline RingRegistry& ring_registry() {
  static RingRegistry* r = new RingRegistry;  // (leaked: thread-local rings may outlive static destruction)
  return *r;
}
struct PinnedRing {
  struct Fence {
    hipStream_t stream;
    int device;
    hipEvent_t event;
  };
  std::mutex m;  // the owner's staging against another thread's forget_stream
  char* buf = nullptr;
  size_t cap = 0, used = 0;
  std::vector<Fence> fences;
  PinnedRing() {
    auto& r = ring_registry();
    std::lock_guard<std::mutex> lock(r.m);
    r.rings.push_back(this);
  }
  ~PinnedRing() {
    {
      auto& r = ring_registry();
      std::lock_guard<std::mutex> lock(r.m);
      r.rings.erase(std::remove(r.rings.begin(), r.rings.end(), this), r.rings.end());
    }
    for (auto& f : fences) (void)hipEventDestroy(f.event);
    if (buf) (void)hipHostFree(buf);
  }
  // (the stream has been synchronised: its fences are complete)
  void forget_stream(hipStream_t s) {
    std::lock_guard<std::mutex> lock(m);
    for (auto& f : fences)
      if (f.stream == s) (void)hipEventDestroy(f.event);
    fences.erase(std::remove_if(fences.begin(), fences.end(), [&](const Fence& f) { return f.stream == s; }),
                 fences.end());
  }
  hy_status wait_all() {
    for (auto& f : fences) {
      const hipError_t e = hipEventSynchronize(f.event);
      if (e == hipSuccess) continue;
      (void)hipGetLastError();
      // a fence the runtime will not wait on (its stream destroyed outside hy_stream_destroy, or in a state the
      // runtime refuses): the whole device covers the ring's copies; the event is re-created
      if (std::getenv("HY_DEBUG_RING"))
        std::fprintf(stderr, "hyrise-amd ring: fence on stream %p device %d: %s\n", static_cast<void*>(f.stream),
                     f.device, hipGetErrorString(e));
      int cur = 0;
      HY_HIP(hipGetDevice(&cur));
      HY_HIP(hipSetDevice(f.device));
      const hipError_t w = hipDeviceSynchronize();
      (void)hipEventDestroy(f.event);
      f.event = nullptr;
      const hipError_t c = hipEventCreateWithFlags(&f.event, hipEventDisableTiming);
      HY_HIP(hipSetDevice(cur));
      HY_HIP(w);
      HY_HIP(c);
    }
    return HY_OK;
  }
  hy_status fence(hipStream_t s) {
    int dev = 0;
    HY_HIP(hipGetDevice(&dev));
    for (auto& f : fences)
      if (f.stream == s && f.device == dev) {
        HY_HIP(hipEventRecord(f.event, s));
        return HY_OK;
      }
    if (fences.size() >= 32) {  // many short-lived streams: retire the fences (their copies are waited for first)
      const hy_status w = wait_all();
      if (w != HY_OK) return w;
      for (auto& f : fences) (void)hipEventDestroy(f.event);
      fences.clear();
    }
    Fence f{s, dev, nullptr};
    HY_HIP(hipEventCreateWithFlags(&f.event, hipEventDisableTiming));
    HY_HIP(hipEventRecord(f.event, s));
    fences.push_back(f);
    return HY_OK;
  }
};
// hy_stream_destroy: no ring keeps a fence on the stream afterwards
inline void ring_forget_stream(hipStream_t s) {
  auto& r = ring_registry();
  std::lock_guard<std::mutex> lock(r.m);
  for (PinnedRing* ring : r.rings) ring->forget_stream(s);
}
// A stream being captured into a graph is refused: the copy would become a graph node reading a ring slot that later
// staging reuses (or frees), so every replay would upload whatever the slot then holds. Captured regions (a prepared
// plan's execution, hyrise_amd_join.hip) stage nothing; their descriptors are in the plan's workspace beforehand.
inline hy_status staged_htod(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return HY_OK;
  if (stream_capturing(s)) {
#ifdef HYRISE_DEBUG
    assert(!"staged_htod on a capturing stream");  // debug builds stop at the offending call
#endif
    return fail(HY_ERR_INVALID_ARGUMENT, "host-staged copy on a stream being captured into a graph");
  }
  thread_local PinnedRing ring;
  std::lock_guard<std::mutex> ring_lock(ring.m);
  const size_t need = (bytes + 255) & ~size_t(255);
  if (ring.used + need > ring.cap) {
    const hy_status w = ring.wait_all();  // every copy out of the ring has completed
    if (w != HY_OK) return w;
    if (need > ring.cap) {
      if (ring.buf) HY_HIP(hipHostFree(ring.buf));
      ring.buf = nullptr;
      ring.cap = std::max<size_t>(size_t(16) << 20, 2 * need);
      HY_HIP(hipHostMalloc(reinterpret_cast<void**>(&ring.buf), ring.cap, hipHostMallocDefault));
    }
    ring.used = 0;
  }
  char* stage = ring.buf + ring.used;
  std::memcpy(stage, src, bytes);
  ring.used += need;
  HY_HIP(hipMemcpyAsync(dst, stage, bytes, hipMemcpyHostToDevice, s));
  return ring.fence(s);
}
#define HY_STAGE(dst, src, bytes, stream)                                              \
  do {                                                                                 \
    const hy_status st_ = ::hyc::staged_htod((dst), (src), (bytes), (stream));         \
    if (st_ != HY_OK) return st_;                                                      \
  } while (0)

// Bump allocator over the caller's workspace. Every carve is 256-byte aligned.
struct Carver {
  char* base;
  size_t cap;
  size_t used = 0;
  bool ok = true;
  template <typename T>
  T* take(size_t count) {
    used = (used + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base ? base + used : nullptr);
    used += count * sizeof(T);
    if (base && used > cap) ok = false;
    return p;
  }
};

// ---- per-kernel timing (HIP events on the launching stream), enabled by hy_kernel_stats_enable ----
struct KernelTiming {
  std::string name;
  hipEvent_t start, stop;
  uint64_t units;
  hipStream_t stream;  // (hy_stream_destroy resolves the stream's pending timings before the handle dies)
};
struct KStat {
  uint64_t count = 0;
  double total_ms = 0;
  uint64_t units = 0;
};
extern std::mutex g_kt_mutex;
// Held while a stream is being captured into a hipGraph (hy_scan_join_plan_execute) and while hy_free_async_after
// orders a free after other streams: that function records events on every operator stream - from any thread, e.g.
// the background chunk reaper - and an event recorded on a stream under capture becomes a node of that capture, and
// a stream that waits on it joins the capture (its own later work is then captured instead of executed, and the
// capture ends unjoined). Recursive: a thread never blocks itself.
extern std::recursive_mutex g_capture_m;
extern uint64_t* g_join_trace;  // hy_debug_set_join_trace
extern thread_local const uint32_t* g_key_hash;  // hy_join_params.key_hash of the join running on this thread
extern bool g_kt_enabled;
extern std::vector<KernelTiming> g_kt_pending;
extern std::vector<hipEvent_t> g_kt_pool;
extern std::vector<std::pair<std::string, KStat>> g_kt_stats;

inline hipEvent_t kt_event() {
  if (!g_kt_pool.empty()) {
    hipEvent_t e = g_kt_pool.back();
    g_kt_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

// Brackets one kernel launch: KTimer t("name", stream, units); launch; t.done();
struct KTimer {
  bool on;
  KernelTiming kt;
  hipStream_t s;
  KTimer(const char* name, hipStream_t stream, uint64_t units) : on(false), s(stream) {
    std::lock_guard<std::mutex> lock(g_kt_mutex);
    if (!g_kt_enabled) return;
    on = true;
    kt.name = name;
    kt.units = units;
    kt.stream = stream;
    kt.start = kt_event();
    kt.stop = kt_event();
    (void)hipEventRecord(kt.start, s);
  }
  void done() {
    if (!on) return;
    (void)hipEventRecord(kt.stop, s);
    std::lock_guard<std::mutex> lock(g_kt_mutex);
    g_kt_pending.push_back(kt);
    on = false;
  }
};

inline int grid_for(uint64_t n, int threads) {
  const uint64_t g = (n + threads - 1) / threads;
  return static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(g, 256 * 16)));
}

}  // namespace hyc
