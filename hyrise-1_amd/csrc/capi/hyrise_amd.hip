// C-ABI implementation (include/hyrise_amd.h): runtime wrappers, launch orchestration and workspace carving for
// the gfx950 TableScan / JoinHash kernels. Nothing here throws across the boundary; every failure becomes an
// hy_status plus a thread-local message.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "hyrise_amd.h"
#include "../kernels/common.hpp"
#include "../kernels/scan.hip"
#include "../kernels/join.hip"

#include "capi_common.hpp"

namespace hyc {
thread_local std::string g_last_error;
std::mutex g_kt_mutex;
std::recursive_mutex g_capture_m;
uint64_t* g_join_trace = nullptr;
thread_local const uint32_t* g_key_hash = nullptr;
bool g_kt_enabled = false;
std::vector<KernelTiming> g_kt_pending;
std::vector<hipEvent_t> g_kt_pool;
std::vector<std::pair<std::string, KStat>> g_kt_stats;
}  // namespace hyc

using namespace hyc;

// ================================================================================================================
// Runtime
// ================================================================================================================
extern "C" {

hy_status hy_get_device_count(int* count) {
  if (!count) return fail(HY_ERR_INVALID_ARGUMENT, "count is NULL");
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return HY_OK;
}

hy_status hy_set_device(int device) {
  HY_HIP(hipSetDevice(device));
  return HY_OK;
}

hy_status hy_malloc(void** ptr, size_t bytes) {
  if (!ptr) return fail(HY_ERR_INVALID_ARGUMENT, "ptr is NULL");
  // round up so that 16-byte vector loads past the last element stay inside the allocation
  HY_HIP(hipMalloc(ptr, std::max<size_t>(256, (bytes + 255) & ~size_t(255))));
  return HY_OK;
}

hy_status hy_free(void* ptr) {
  if (ptr) HY_HIP(hipFree(ptr));
  return HY_OK;
}

// Stream-ordered allocations from the device's default memory pool, which keeps freed memory (release threshold =
// unlimited) for the next allocation instead of returning it to the driver: operator outputs of several GB per query
// step are then not a hipMalloc + hipFree (and the device-wide synchronisation hipFree implies) each time.
hy_status hy_malloc_async(void** ptr, size_t bytes, hy_stream_t stream) {
  if (!ptr) return fail(HY_ERR_INVALID_ARGUMENT, "ptr is NULL");
  static std::once_flag once;
  static hipError_t pool_err = hipSuccess;
  std::call_once(once, [] {
    int dev = 0;
    hipMemPool_t pool;
    pool_err = hipGetDevice(&dev);
    if (pool_err == hipSuccess) pool_err = hipDeviceGetDefaultMemPool(&pool, dev);
    if (pool_err == hipSuccess) {
      uint64_t threshold = UINT64_MAX;
      pool_err = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold);
    }
  });
  HY_HIP(pool_err);
  HY_HIP(hipMallocAsync(ptr, std::max<size_t>(256, (bytes + 255) & ~size_t(255)), S(stream)));
  return HY_OK;
}

hy_status hy_free_async(void* ptr, hy_stream_t stream) {
  if (ptr) HY_HIP(hipFreeAsync(ptr, S(stream)));
  return HY_OK;
}

hy_status hy_free_async_after(void* ptr, hy_stream_t free_stream, const hy_stream_t* wait_streams, uint32_t n_wait) {
  if (!ptr) return HY_OK;
  if (n_wait && !wait_streams) return fail(HY_ERR_INVALID_ARGUMENT, "wait_streams is NULL");
  // (not while another thread captures one of these streams: see g_capture_m)
  std::lock_guard<std::recursive_mutex> capture_lock(g_capture_m);
  for (uint32_t i = 0; i < n_wait; ++i) {
    if (wait_streams[i] == free_stream) continue;
    hipEvent_t ev;
    HY_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, S(wait_streams[i]));
    if (e == hipSuccess) e = hipStreamWaitEvent(S(free_stream), ev, 0);
    (void)hipEventDestroy(ev);  // (the wait holds what it needs)
    HY_HIP(e);
  }
  HY_HIP(hipFreeAsync(ptr, S(free_stream)));
  return HY_OK;
}

hy_status hy_device_memory(uint64_t* free_bytes, uint64_t* total_bytes) {
  if (!free_bytes || !total_bytes) return fail(HY_ERR_INVALID_ARGUMENT, "NULL output");
  size_t f = 0, t = 0;
  HY_HIP(hipMemGetInfo(&f, &t));
  *free_bytes = f;
  *total_bytes = t;
  return HY_OK;
}

hy_status hy_pool_stats(uint64_t* reserved_bytes, uint64_t* used_bytes) {
  if (!reserved_bytes || !used_bytes) return fail(HY_ERR_INVALID_ARGUMENT, "NULL output");
  int dev = 0;
  hipMemPool_t pool;
  HY_HIP(hipGetDevice(&dev));
  HY_HIP(hipDeviceGetDefaultMemPool(&pool, dev));
  HY_HIP(hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, reserved_bytes));
  HY_HIP(hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, used_bytes));
  return HY_OK;
}

hy_status hy_memcpy_htod(void* dst, const void* src, size_t bytes, hy_stream_t stream) {
  if (bytes) HY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream)));
  return HY_OK;
}

hy_status hy_memcpy_dtoh(void* dst, const void* src, size_t bytes, hy_stream_t stream) {
  if (bytes) HY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream)));
  return HY_OK;
}

hy_status hy_memcpy_dtod(void* dst, const void* src, size_t bytes, hy_stream_t stream) {
  if (bytes) HY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, S(stream)));
  return HY_OK;
}

hy_status hy_memset(void* dst, int value, size_t bytes, hy_stream_t stream) {
  if (bytes) HY_HIP(hipMemsetAsync(dst, value, bytes, S(stream)));
  return HY_OK;
}

hy_status hy_stream_create(hy_stream_t* stream) {
  hipStream_t s;
  HY_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return HY_OK;
}

namespace {
// one pending kernel timing into the stats (g_kt_mutex held; its stop event has completed or is waited for)
hy_status kt_resolve_locked(const KernelTiming& k) {
  HY_HIP(hipEventSynchronize(k.stop));
  float ms = 0;
  HY_HIP(hipEventElapsedTime(&ms, k.start, k.stop));
  auto it = std::find_if(g_kt_stats.begin(), g_kt_stats.end(), [&](const auto& e) { return e.first == k.name; });
  if (it == g_kt_stats.end()) {
    g_kt_stats.emplace_back(k.name, KStat{});
    it = g_kt_stats.end() - 1;
  }
  it->second.count += 1;
  it->second.total_ms += ms;
  it->second.units += k.units;
  g_kt_pool.push_back(k.start);
  g_kt_pool.push_back(k.stop);
  return HY_OK;
}
}  // namespace

hy_status hy_stream_destroy(hy_stream_t stream) {
  // Every event this library recorded on the stream is finished with before the handle dies: the runtime follows an
  // event to the stream it was last recorded on when the event is waited for, and a destroyed stream there is a read
  // - and, when the freed memory happens to look like an active capture, a write - of freed runtime memory
  // (the staging rings' fences and the pending kernel timings).
  HY_HIP(hipStreamSynchronize(S(stream)));
  ring_forget_stream(S(stream));
  {
    std::lock_guard<std::mutex> lock(g_kt_mutex);
    hy_status st = HY_OK;
    for (const auto& k : g_kt_pending)
      if (k.stream == S(stream) && st == HY_OK) st = kt_resolve_locked(k);
    g_kt_pending.erase(std::remove_if(g_kt_pending.begin(), g_kt_pending.end(),
                                      [&](const KernelTiming& k) { return k.stream == S(stream); }),
                       g_kt_pending.end());
    if (st != HY_OK) return st;
  }
  HY_HIP(hipStreamDestroy(S(stream)));
  return HY_OK;
}

hy_status hy_stream_synchronize(hy_stream_t stream) {
  HY_HIP(hipStreamSynchronize(S(stream)));
  return HY_OK;
}

const char* hy_last_error_message(void) { return g_last_error.c_str(); }

hy_status hy_debug_set_join_trace(uint64_t* device_trace) {
  g_join_trace = device_trace;
  return HY_OK;
}

hy_status hy_kernel_stats_enable(int enable) {
  std::lock_guard<std::mutex> lock(g_kt_mutex);
  g_kt_enabled = enable != 0;
  return HY_OK;
}

hy_status hy_kernel_stats_reset(void) {
  std::lock_guard<std::mutex> lock(g_kt_mutex);
  for (auto& k : g_kt_pending) {
    (void)hipEventSynchronize(k.stop);
    g_kt_pool.push_back(k.start);
    g_kt_pool.push_back(k.stop);
  }
  g_kt_pending.clear();
  g_kt_stats.clear();
  return HY_OK;
}

// Resolves all recorded launches (waits for them) and returns the number of distinct kernels.
hy_status hy_kernel_stats_collect(uint32_t* n_kernels) {
  std::lock_guard<std::mutex> lock(g_kt_mutex);
  for (auto& k : g_kt_pending) {
    const hy_status st = kt_resolve_locked(k);
    if (st != HY_OK) return st;
  }
  g_kt_pending.clear();
  if (n_kernels) *n_kernels = static_cast<uint32_t>(g_kt_stats.size());
  return HY_OK;
}

hy_status hy_kernel_stats_get(uint32_t index, const char** name, uint64_t* launches, double* total_ms,
                              uint64_t* units) {
  std::lock_guard<std::mutex> lock(g_kt_mutex);
  if (index >= g_kt_stats.size()) return fail(HY_ERR_INVALID_ARGUMENT, "kernel stats index");
  *name = g_kt_stats[index].first.c_str();
  *launches = g_kt_stats[index].second.count;
  *total_ms = g_kt_stats[index].second.total_ms;
  *units = g_kt_stats[index].second.units;
  return HY_OK;
}

const char* hy_build_info(void) { return "hyrise-amd gfx950 (CDNA4) HIP kernels: table_scan, reference_scan, join_hash"; }

}  // extern "C"

// ================================================================================================================
// TableScan
// ================================================================================================================
namespace {

enum ScanClass { SC_DICT8, SC_DICT16, SC_DICT32, SC_VALUE, SC_FOR8, SC_FOR16, SC_FOR32, SC_RLE, SC_COUNT };

int width_class(int32_t w, int base) { return w == 1 ? base : w == 2 ? base + 1 : w == 4 ? base + 2 : -1; }

int scan_class(const hy_scan_chunk& c) {
  switch (c.column.kind) {
    case HY_COL_VALUE:
      return SC_VALUE;
    case HY_COL_DICT:
      return width_class(c.column.vid_width, SC_DICT8);
    case HY_COL_FOR:
      return width_class(c.column.vid_width, SC_FOR8);
    case HY_COL_RLE:
      return SC_RLE;
  }
  return -1;
}

uint64_t scan_tiles(uint32_t size) { return (uint64_t(size) + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE; }

// tiles per workgroup of 1-byte columns: 4 (64 B of loads in flight per lane) - twice the workgroups of
// seg_tiles<uint8_t> (8), whose single round of long workgroups left the chip idle in its tail (TableScan SF10
// `scan_dict` 0.117 vs 0.153 ms; 2: 0.129 ms; profiles/r03d_scan_seg8_*). HY_SCAN_SEG8 = 2 / 8: A/B.
int seg8() {
  static const int v = [] {
    const char* e = std::getenv("HY_SCAN_SEG8");
    const int x = e ? std::atoi(e) : 4;
    return (x == 2 || x == 8) ? x : 4;
  }();
  return v;
}

// tiles per scan workgroup for a column class (hyk::seg_tiles<E> of the class's element type)
int class_seg(int cls, int32_t value_type) {
  switch (cls) {
    case SC_DICT8:
    case SC_FOR8:
      return seg8();
    case SC_DICT16:
    case SC_FOR16:
      return hyk::seg_tiles<uint16_t>();
    case SC_DICT32:
    case SC_FOR32:
      return hyk::seg_tiles<uint32_t>();
    default:
      return (value_type == HY_TYPE_INT64 || value_type == HY_TYPE_DOUBLE) ? hyk::seg_tiles<int64_t>()
                                                                          : hyk::seg_tiles<int32_t>();
  }
}

// HY_SCAN_TWO_PASS=0: the one-pass look-back kernel for every chunk (A/B); otherwise chunks of at most
// hyk::SCAN_TWO_PASS_SEGS segments (6.5 M rows at 1-byte ids) take the count + write kernels
bool scan_two_pass_enabled() {
  const char* e = std::getenv("HY_SCAN_TWO_PASS");  // (read per call: tests switch it)
  return !(e && std::atoi(e) == 0);
}

template <typename E, int MODE, bool OUT_ROWID, typename V, int SEG>
void launch_scan_seg(const hyk::ScanLaunchDesc& d, const hyk::ScanConst<V>& c, void* out, uint32_t* counts,
                     bool two_pass, hipStream_t s) {
  const dim3 grid(static_cast<uint32_t>(d.n_tiles)), block(hyk::SCAN_THREADS);
  if (two_pass) {
    hipLaunchKernelGGL((hyk::scan_count_kernel<E, MODE, V, SEG>), grid, block, 0, s, d, c);
    hipLaunchKernelGGL((hyk::scan_write_kernel<OUT_ROWID, SEG>), grid, block, 0, s, d, out, counts);
  } else {
    hipLaunchKernelGGL((hyk::scan_kernel<E, MODE, OUT_ROWID, V, SEG>), grid, block, 0, s, d, c, out, counts);
  }
}

// two_pass: every chunk of the class has at most hyk::SCAN_TWO_PASS_SEGS segments
template <typename E, int MODE, bool OUT_ROWID, typename V = E>
hy_status launch_scan(const hyk::ScanLaunchDesc& d, const void* constant, void* out, uint32_t* counts, bool two_pass,
                      hipStream_t s) {
  hyk::ScanConst<V> c{};
  if (MODE != hyk::MODE_DICT && constant) std::memcpy(&c.value, constant, sizeof(V));
  // (the two kernels of a two-pass scan are timed as one: the scan's time)
  KTimer t(MODE == hyk::MODE_DICT ? "scan_dict" : MODE == hyk::MODE_FOR ? "scan_frame_of_reference" : "scan_value", s,
           d.n_rows);
  if constexpr (sizeof(E) == 1) {
    if (seg8() == 2)
      launch_scan_seg<E, MODE, OUT_ROWID, V, 2>(d, c, out, counts, two_pass, s);
    else if (seg8() == 8)
      launch_scan_seg<E, MODE, OUT_ROWID, V, 8>(d, c, out, counts, two_pass, s);
    else
      launch_scan_seg<E, MODE, OUT_ROWID, V, 4>(d, c, out, counts, two_pass, s);
  } else {
    launch_scan_seg<E, MODE, OUT_ROWID, V, hyk::seg_tiles<E>()>(d, c, out, counts, two_pass, s);
  }
  t.done();
  HY_HIP(hipGetLastError());
  return HY_OK;
}

template <typename E, bool OUT_ROWID>
hy_status launch_for(const hyk::ScanLaunchDesc& d, int32_t value_type, const void* constant, void* out,
                     uint32_t* counts, bool two_pass, hipStream_t s) {
  if (value_type == HY_TYPE_INT32)
    return launch_scan<E, hyk::MODE_FOR, OUT_ROWID, int32_t>(d, constant, out, counts, two_pass, s);
  return launch_scan<E, hyk::MODE_FOR, OUT_ROWID, int64_t>(d, constant, out, counts, two_pass, s);
}

// RunLength chunks of one call (hyk::rle_* kernels): per-run predicate, prefix over the matching runs' lengths, then
// the row ranges expanded into each chunk's output. Run-level temporaries come from the stream-ordered pool (their
// size follows the run count, which the workspace query does not see).
template <bool OUT_ROWID>
hy_status rle_scan(const hyk::RleDesc& d, const uint32_t* chunk_index, const uint32_t* chunk_ids,
                   int32_t value_type, const void* constant, void* out, uint32_t* counts, uint64_t rows,
                   hipStream_t s) {
  const uint64_t n = d.n_runs;
  uint32_t* match_len = nullptr;
  uint64_t* prefix = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  HY_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, static_cast<const uint32_t*>(nullptr),
                                          static_cast<uint64_t*>(nullptr), static_cast<int>(n + 1), s));
  HY_HIP(hipMallocAsync(reinterpret_cast<void**>(&match_len), 4 * (n + 1), s));
  HY_HIP(hipMallocAsync(reinterpret_cast<void**>(&prefix), 8 * (n + 1), s));
  HY_HIP(hipMallocAsync(&temp, temp_bytes + 16, s));
  hyk::RleDesc dd = d;
  auto match = [&](auto tag) {
    using T = decltype(tag);
    hyk::ScanConst<T> c{};
    if (constant) std::memcpy(&c.value, constant, sizeof(T));
    hipLaunchKernelGGL((hyk::rle_match_kernel<T>), dim3(grid_for(n + 1, hyk::SCAN_THREADS)), dim3(hyk::SCAN_THREADS),
                       0, s, dd, c, match_len);
  };
  {
    KTimer kt("scan_run_length", s, rows);
    switch (value_type) {
      case HY_TYPE_INT32:
        match(int32_t{});
        break;
      case HY_TYPE_INT64:
        match(int64_t{});
        break;
      case HY_TYPE_FLOAT:
        match(float{});
        break;
      default:
        match(double{});
        break;
    }
    HY_HIP(hipGetLastError());
    HY_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, match_len, prefix, static_cast<int>(n + 1), s));
    hipLaunchKernelGGL(hyk::rle_counts_kernel, dim3((d.n_chunks + 255) / 256), dim3(256), 0, s, dd, prefix, chunk_index,
                       counts);
    HY_HIP(hipGetLastError());
    uint64_t total = 0;
    HY_HIP(hipMemcpyAsync(&total, prefix + n, 8, hipMemcpyDeviceToHost, s));
    HY_HIP(hipStreamSynchronize(s));
    if (total)
      hipLaunchKernelGGL((hyk::rle_expand_kernel<OUT_ROWID>), dim3(grid_for(total, hyk::SCAN_THREADS)),
                         dim3(hyk::SCAN_THREADS), 0, s, dd, prefix, total, chunk_ids, out);
    kt.done();
  }
  HY_HIP(hipGetLastError());
  HY_HIP(hipFreeAsync(match_len, s));
  HY_HIP(hipFreeAsync(prefix, s));
  HY_HIP(hipFreeAsync(temp, s));
  return HY_OK;
}

// workspace layout for one class: chunks, tile prefix, chunk index, status
size_t scan_class_bytes(uint32_t n_chunks, uint64_t n_tiles) {
  Carver cv{nullptr, 0};
  cv.take<hy_scan_chunk>(n_chunks);
  cv.take<uint64_t>(n_chunks + 1);
  cv.take<uint32_t>(n_chunks);
  cv.take<uint32_t>(n_chunks);
  cv.take<uint64_t>(n_tiles + 1);
  cv.take<uint32_t>(n_tiles + 1);
  cv.take<uint32_t>(64);
  // two-pass masks: per lane one 32-bit word per two tiles of a segment - at most one per tile, plus up to 4 for a
  // chunk's last, partial segment
  cv.take<uint32_t>((n_tiles + 4ull * n_chunks) * hyk::SCAN_THREADS);
  return cv.used + 256;
}

}  // namespace

extern "C" {

hy_status hy_table_scan_workspace_size(const uint32_t* chunk_sizes, uint32_t n_chunks, size_t* bytes) {
  if (!bytes || (n_chunks && !chunk_sizes)) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  uint64_t tiles = 0;
  for (uint32_t i = 0; i < n_chunks; ++i) tiles += scan_tiles(chunk_sizes[i]);
  // worst case: all chunks in one class, times the number of classes (carved sequentially)
  *bytes = SC_COUNT * scan_class_bytes(n_chunks, tiles);
  return HY_OK;
}

}  // extern "C"

namespace {
template <bool OUT_ROWID>
hy_status table_scan_impl(const hy_scan_chunk* chunks, uint32_t n_chunks, int32_t value_type, const void* constant,
                          void* out_offsets, uint32_t* counts, const uint32_t* chunk_ids, void* workspace,
                          size_t workspace_bytes, hy_stream_t stream) {
  if (n_chunks == 0) return HY_OK;
  if (!chunks || !out_offsets || !counts) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  hipStream_t s = S(stream);
  std::vector<std::vector<uint32_t>> by_class(SC_COUNT);
  for (uint32_t i = 0; i < n_chunks; ++i) {
    const int cls = scan_class(chunks[i]);
    if (cls < 0) return fail(HY_ERR_INVALID_ARGUMENT, "bad chunk kind / vid width");
    if ((cls == SC_RLE || cls >= SC_FOR8) && chunks[i].column.size && !chunks[i].column.dictionary)
      return fail(HY_ERR_INVALID_ARGUMENT, "compressed chunk without its minima / end positions");
    if (cls == SC_RLE && chunks[i].column.size &&
        (chunks[i].column.dictionary_size == 0 || chunks[i].column.dictionary_size > chunks[i].column.size))
      return fail(HY_ERR_INVALID_ARGUMENT, "run count");
    if (cls >= SC_FOR8 && cls <= SC_FOR32 && value_type != HY_TYPE_INT32 && value_type != HY_TYPE_INT64)
      return fail(HY_ERR_UNSUPPORTED, "FrameOfReference chunks hold int32 / int64");
    if (chunks[i].op < HY_OP_EQ || chunks[i].op > HY_OP_VID_SET) return fail(HY_ERR_INVALID_ARGUMENT, "scan op");
    if (chunks[i].op == HY_OP_VID_SET && (chunks[i].column.kind != HY_COL_DICT || !chunks[i].vid_set))
      return fail(HY_ERR_INVALID_ARGUMENT, "HY_OP_VID_SET needs a dictionary chunk and a vid_set");
    if (chunks[i].column.size && !aligned16(chunks[i].column.data))
      return fail(HY_ERR_ALIGNMENT, "column data not 16-byte aligned");
    if (chunks[i].column.nulls && !aligned16(chunks[i].column.nulls))
      return fail(HY_ERR_ALIGNMENT, "null vector not 16-byte aligned");
    by_class[cls].push_back(i);
  }
  if ((!by_class[SC_VALUE].empty() || !by_class[SC_RLE].empty()) &&
      !(value_type == HY_TYPE_INT32 || value_type == HY_TYPE_INT64 || value_type == HY_TYPE_FLOAT ||
        value_type == HY_TYPE_DOUBLE))
    return fail(HY_ERR_UNSUPPORTED, "value scan type");
  HY_HIP(hipMemsetAsync(counts, 0, sizeof(uint32_t) * n_chunks, s));

  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  // host staging must outlive the async copies: keep everything until the stream is synchronized below
  std::vector<std::vector<hy_scan_chunk>> h_chunks(SC_COUNT);
  std::vector<std::vector<uint64_t>> h_tiles(SC_COUNT);
  std::vector<std::vector<uint32_t>> h_cids(SC_COUNT);
  uint32_t* error = nullptr;
  for (int cls = 0; cls < SC_COUNT; ++cls) {
    const auto& idx = by_class[cls];
    if (idx.empty()) continue;
    const uint32_t nc = static_cast<uint32_t>(idx.size());
    auto& hc = h_chunks[cls];
    auto& ht = h_tiles[cls];
    hc.resize(nc);
    ht.resize(nc + 1);
    uint64_t run = 0, rows = 0, max_segs = 0;
    for (uint32_t k = 0; k < nc; ++k) {
      hc[k] = chunks[idx[k]];
      rows += hc[k].column.size;
      ht[k] = run;
      const uint64_t seg = static_cast<uint64_t>(class_seg(cls, value_type));
      if (cls == SC_RLE)  // runs, not tiles
        run += hc[k].column.size ? hc[k].column.dictionary_size : 0;
      else
        run += hc[k].op == HY_OP_NONE ? 0 : (scan_tiles(hc[k].column.size) + seg - 1) / seg;  // segments
      max_segs = std::max(max_segs, run - ht[k]);
    }
    ht[nc] = run;
    const bool two_pass = scan_two_pass_enabled() && max_segs <= hyk::SCAN_TWO_PASS_SEGS;
    hyk::ScanLaunchDesc d{};
    // descriptors, segment prefix, chunk indexes, chunk ids and segment owners carved back to back and uploaded as ONE
    // staged copy; then the look-back words and the ticket / error words cleared by one memset
    auto* dch = cv.take<hy_scan_chunk>(nc);
    auto* dti = cv.take<uint64_t>(nc + 1);
    auto* dix = cv.take<uint32_t>(nc);
    auto* dcid = cv.take<uint32_t>(nc);
    const uint64_t words = cls == SC_RLE ? 0 : run;  // RLE: run-level arrays come from rle_scan's own pool
    auto* downer = cv.take<uint32_t>(words + 1);
    auto* dst = cv.take<uint64_t>(words + 1);
    auto* dmisc = cv.take<uint32_t>(64);
    // the two-pass masks: mask_words(seg) 32-bit words per lane and segment (seg tiles of 4096 rows: <= one per tile)
    const uint64_t seg_of_class = cls == SC_RLE ? 0 : static_cast<uint64_t>(class_seg(cls, value_type));
    auto* dmasks = two_pass ? cv.take<uint32_t>(words * hyk::mask_words(static_cast<int>(seg_of_class)) * hyk::SCAN_THREADS)
                            : nullptr;
    if (!cv.ok) return fail(HY_ERR_WORKSPACE, "scan workspace too small");
    if (!error) error = dmisc + 1;  // (cleared by this class's memset below)
    auto& hcid = h_cids[cls];
    hcid.resize(nc);
    for (uint32_t k = 0; k < nc; ++k) hcid[k] = chunk_ids ? chunk_ids[idx[k]] : idx[k];
    {
      char* const base = reinterpret_cast<char*>(dch);
      std::vector<char> image(reinterpret_cast<char*>(downer + words + 1) - base, 0);
      auto put = [&](void* dev, const void* src, size_t bytes) {
        if (bytes) std::memcpy(image.data() + (static_cast<char*>(dev) - base), src, bytes);
      };
      put(dch, hc.data(), sizeof(hy_scan_chunk) * nc);
      put(dti, ht.data(), sizeof(uint64_t) * (nc + 1));
      put(dix, idx.data(), sizeof(uint32_t) * nc);
      put(dcid, hcid.data(), sizeof(uint32_t) * nc);
      uint32_t* owner = reinterpret_cast<uint32_t*>(image.data() + (reinterpret_cast<char*>(downer) - base));
      for (uint32_t k = 0; k < nc; ++k)
        for (uint64_t t = ht[k]; t < ht[k + 1] && cls != SC_RLE; ++t) owner[t] = k;  // (fill_tile_owner's result)
      HY_STAGE(dch, image.data(), image.size(), s);
    }
    HY_HIP(hipMemsetAsync(dst, 0, reinterpret_cast<char*>(dmisc + 64) - reinterpret_cast<char*>(dst), s));
    if (run == 0) continue;
    if (cls == SC_RLE) {
      uint32_t* run_chunk = nullptr;
      HY_HIP(hipMallocAsync(reinterpret_cast<void**>(&run_chunk), 4 * (run + 1), s));
      hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((nc + 255) / 256), dim3(256), 0, s, dti, nc, run_chunk);
      HY_HIP(hipGetLastError());
      const hyk::RleDesc rd{dch, dti, run_chunk, run, nc};
      const hy_status st = rle_scan<OUT_ROWID>(rd, dix, dcid, value_type, constant, out_offsets, counts, rows, s);
      HY_HIP(hipFreeAsync(run_chunk, s));
      if (st != HY_OK) return st;
      continue;
    }
    d.tile_chunk = downer;
    d.chunks = dch;
    d.chunk_tile_begin = dti;
    d.chunk_index = dix;
    d.chunk_ids = dcid;
    d.n_rows = rows;
    d.n_chunks = nc;
    d.n_tiles = run;
    d.status = dst;
    d.ticket = dmisc;
    d.error = error;
    d.masks = dmasks;
    hy_status st = HY_OK;
    constexpr int DICT = hyk::MODE_DICT, VALUE = hyk::MODE_VALUE;
    switch (cls) {
      case SC_DICT8:
        st = launch_scan<uint8_t, DICT, OUT_ROWID>(d, nullptr, out_offsets, counts, two_pass, s);
        break;
      case SC_DICT16:
        st = launch_scan<uint16_t, DICT, OUT_ROWID>(d, nullptr, out_offsets, counts, two_pass, s);
        break;
      case SC_DICT32:
        st = launch_scan<uint32_t, DICT, OUT_ROWID>(d, nullptr, out_offsets, counts, two_pass, s);
        break;
      case SC_FOR8:
        st = launch_for<uint8_t, OUT_ROWID>(d, value_type, constant, out_offsets, counts, two_pass, s);
        break;
      case SC_FOR16:
        st = launch_for<uint16_t, OUT_ROWID>(d, value_type, constant, out_offsets, counts, two_pass, s);
        break;
      case SC_FOR32:
        st = launch_for<uint32_t, OUT_ROWID>(d, value_type, constant, out_offsets, counts, two_pass, s);
        break;
      case SC_VALUE:
        switch (value_type) {
          case HY_TYPE_INT32:
            st = launch_scan<int32_t, VALUE, OUT_ROWID>(d, constant, out_offsets, counts, two_pass, s);
            break;
          case HY_TYPE_INT64:
            st = launch_scan<int64_t, VALUE, OUT_ROWID>(d, constant, out_offsets, counts, two_pass, s);
            break;
          case HY_TYPE_FLOAT:
            st = launch_scan<float, VALUE, OUT_ROWID>(d, constant, out_offsets, counts, two_pass, s);
            break;
          case HY_TYPE_DOUBLE:
            st = launch_scan<double, VALUE, OUT_ROWID>(d, constant, out_offsets, counts, two_pass, s);
            break;
        }
        break;
    }
    if (st != HY_OK) return st;
  }
  uint32_t herr = 0;
  if (error) {
    HY_HIP(hipMemcpyAsync(&herr, error, 4, hipMemcpyDeviceToHost, s));
  }
  HY_HIP(hipStreamSynchronize(s));
  if (herr) return fail(HY_ERR_KERNEL, "scan look-back did not complete");
  return HY_OK;
}
}  // namespace

extern "C" {

hy_status hy_table_scan(const hy_scan_chunk* chunks, uint32_t n_chunks, int32_t value_type, const void* constant,
                        uint32_t* out_offsets, uint32_t* counts, void* workspace, size_t workspace_bytes,
                        hy_stream_t stream) {
  return table_scan_impl<false>(chunks, n_chunks, value_type, constant, out_offsets, counts, nullptr, workspace,
                                workspace_bytes, stream);
}

hy_status hy_table_scan_row_ids(const hy_scan_chunk* chunks, uint32_t n_chunks, int32_t value_type,
                                const void* constant, const uint32_t* chunk_ids, hy_row_id* out_rows, uint32_t* counts,
                                void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  return table_scan_impl<true>(chunks, n_chunks, value_type, constant, out_rows, counts, chunk_ids, workspace,
                               workspace_bytes, stream);
}

hy_status hy_reference_scan_workspace_size(uint64_t pos_list_size, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  const uint64_t tiles = (pos_list_size + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE;
  Carver cv{nullptr, 0};
  cv.take<uint64_t>(tiles + 1);
  cv.take<uint32_t>(64);
  cv.take<hy_scan_chunk>(1 << 20);  // referenced chunk descriptors (bounded below by the call)
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_reference_scan(const hy_row_id* pos_list, uint64_t pos_list_size, const hy_scan_chunk* referenced_chunks,
                            uint32_t n_referenced_chunks, int32_t value_type, const void* constant,
                            uint32_t* out_positions, uint64_t* count, void* workspace, size_t workspace_bytes,
                            hy_stream_t stream) {
  if (!count) return fail(HY_ERR_INVALID_ARGUMENT, "null count");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(count, 0, 8, s));
  if (pos_list_size == 0) return HY_OK;
  if (n_referenced_chunks > (1u << 20)) return fail(HY_ERR_UNSUPPORTED, "too many referenced chunks");
  for (uint32_t i = 0; i < n_referenced_chunks; ++i) {
    const hy_scan_chunk& rc = referenced_chunks[i];
    if (rc.op < HY_OP_EQ || rc.op > HY_OP_VID_SET ||
        (rc.op == HY_OP_VID_SET && (rc.column.kind != HY_COL_DICT || !rc.vid_set)))
      return fail(HY_ERR_INVALID_ARGUMENT, "scan op");
    if (rc.column.kind == HY_COL_STRING) return fail(HY_ERR_UNSUPPORTED, "string chunks: hy_string_reference_scan");
    if ((rc.column.kind == HY_COL_RLE || rc.column.kind == HY_COL_FOR) && rc.column.size &&
        (!rc.column.dictionary || (rc.column.kind == HY_COL_RLE && rc.column.dictionary_size == 0)))
      return fail(HY_ERR_INVALID_ARGUMENT, "compressed chunk without its minima / end positions");
  }
  const uint64_t tiles = (pos_list_size + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE;
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  auto* dst = cv.take<uint64_t>(tiles + 1);
  auto* dmisc = cv.take<uint32_t>(64);
  auto* dch = cv.take<hy_scan_chunk>(std::max<uint32_t>(1, n_referenced_chunks));
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "reference scan workspace too small");
  HY_HIP(hipMemsetAsync(dst, 0, sizeof(uint64_t) * (tiles + 1), s));
  HY_HIP(hipMemsetAsync(dmisc, 0, 256, s));
  HY_STAGE(dch, referenced_chunks, sizeof(hy_scan_chunk) * n_referenced_chunks, s);
  hyk::RefScanDesc d{pos_list, pos_list_size, dch, n_referenced_chunks, tiles, dst, dmisc, dmisc + 1};
  auto go = [&](auto tag) -> hy_status {
    using T = decltype(tag);
    hyk::ScanConst<T> c{};
    if (constant) std::memcpy(&c.value, constant, sizeof(T));
    hipLaunchKernelGGL((hyk::ref_scan_kernel<T>), dim3(static_cast<uint32_t>(tiles)), dim3(hyk::SCAN_THREADS), 0, s, d,
                       c, out_positions, count);
    HY_HIP(hipGetLastError());
    return HY_OK;
  };
  hy_status st;
  switch (value_type) {
    case HY_TYPE_INT32:
      st = go(int32_t{});
      break;
    case HY_TYPE_INT64:
      st = go(int64_t{});
      break;
    case HY_TYPE_FLOAT:
      st = go(float{});
      break;
    case HY_TYPE_DOUBLE:
      st = go(double{});
      break;
    default: {
      // non-numeric columns (strings) are only scanned through their dictionaries: the comparison is on value ids
      for (uint32_t i = 0; i < n_referenced_chunks; ++i)
        if (referenced_chunks[i].column.kind != HY_COL_DICT && referenced_chunks[i].op != HY_OP_NONE &&
            referenced_chunks[i].op != HY_OP_IS_NULL)  // IS NULL reads only the null flags
          return fail(HY_ERR_UNSUPPORTED, "reference scan of an unencoded non-numeric column");
      st = go(int32_t{});
      break;
    }
  }
  if (st != HY_OK) return st;
  uint32_t herr = 0;
  HY_HIP(hipMemcpyAsync(&herr, dmisc + 1, 4, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  if (herr) return fail(HY_ERR_KERNEL, "reference scan look-back did not complete");
  return HY_OK;
}

hy_status hy_pos_list_null_positions(const hy_row_id* pos_list, uint64_t pos_list_size, uint32_t* out_positions,
                                     uint64_t* count, void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  if (!count) return fail(HY_ERR_INVALID_ARGUMENT, "null count");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(count, 0, 8, s));
  if (pos_list_size == 0) return HY_OK;
  if (!pos_list || !out_positions) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  const uint64_t tiles = (pos_list_size + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE;
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  auto* dst = cv.take<uint64_t>(tiles + 1);
  auto* dmisc = cv.take<uint32_t>(64);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "null-position workspace too small");
  HY_HIP(hipMemsetAsync(dst, 0, sizeof(uint64_t) * (tiles + 1), s));
  HY_HIP(hipMemsetAsync(dmisc, 0, 256, s));
  hyk::RefScanDesc d{pos_list, pos_list_size, nullptr, 0, tiles, dst, dmisc, dmisc + 1};
  hipLaunchKernelGGL((hyk::ref_scan_kernel<int32_t, true>), dim3(static_cast<uint32_t>(tiles)),
                     dim3(hyk::SCAN_THREADS), 0, s, d, hyk::ScanConst<int32_t>{}, out_positions, count);
  HY_HIP(hipGetLastError());
  uint32_t herr = 0;
  HY_HIP(hipMemcpyAsync(&herr, dmisc + 1, 4, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  if (herr) return fail(HY_ERR_KERNEL, "null-position look-back did not complete");
  return HY_OK;
}

hy_status hy_gather_row_ids(const hy_row_id* pos_list, const uint32_t* positions, uint64_t n, hy_row_id* out,
                            hy_stream_t stream) {
  if (n == 0) return HY_OK;
  hipLaunchKernelGGL(hyk::gather_row_ids_kernel, dim3(grid_for(n, 256)), dim3(256), 0, S(stream), pos_list, positions,
                     n, out);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_pos_list_chunk_first_seen(const hy_row_id* pos_list, uint64_t n, uint32_t n_chunks, uint64_t* first_seen,
                                       hy_stream_t stream) {
  if (n_chunks == 0) return HY_OK;
  HY_HIP(hipMemsetAsync(first_seen, 0xFF, 8ull * n_chunks, S(stream)));
  if (n == 0) return HY_OK;
  hipLaunchKernelGGL(hyk::first_seen_kernel, dim3(grid_for(n, 256)), dim3(256), 0, S(stream), pos_list, n, n_chunks,
                     reinterpret_cast<unsigned long long*>(first_seen));
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_expand_row_ids(uint32_t chunk_id, const uint32_t* offsets, uint64_t n, hy_row_id* out,
                            hy_stream_t stream) {
  if (n == 0) return HY_OK;
  hipLaunchKernelGGL(hyk::expand_row_ids_kernel, dim3(grid_for(n, 256)), dim3(256), 0, S(stream), chunk_id, offsets, n,
                     out);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_table_scan_count(const hy_scan_chunk* chunks, uint32_t n_chunks, uint32_t* counts, void* workspace,
                              size_t workspace_bytes, hy_stream_t stream) {
  if (n_chunks == 0) return HY_OK;
  if (!chunks || !counts) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  int width = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    const auto& ch = chunks[c];
    if (ch.column.kind != HY_COL_DICT || ch.op == HY_OP_IS_NULL || (ch.op == HY_OP_VID_SET && !ch.vid_set))
      return fail(HY_ERR_UNSUPPORTED, "hy_table_scan_count: dictionary predicates only");
    if (ch.column.size && (reinterpret_cast<uintptr_t>(ch.column.data) & 15u))
      return fail(HY_ERR_INVALID_ARGUMENT, "hy_table_scan_count: chunk data must be 16-byte aligned");
    if (ch.column.size) {
      if (width && width != ch.column.vid_width) return fail(HY_ERR_UNSUPPORTED, "hy_table_scan_count: mixed id widths");
      width = ch.column.vid_width;
    }
  }
  if (workspace_bytes < sizeof(hy_scan_chunk) * n_chunks) return fail(HY_ERR_INVALID_ARGUMENT, "workspace too small");
  hipStream_t s = S(stream);
  auto* d_chunks = static_cast<hy_scan_chunk*>(workspace);
  HY_STAGE(d_chunks, chunks, sizeof(hy_scan_chunk) * n_chunks, s);
  switch (width) {
    case 0:
      HY_HIP(hipMemsetAsync(counts, 0, 4ull * n_chunks, s));
      return HY_OK;
    case 1:
      hipLaunchKernelGGL(hyk::scan_count_kernel<uint8_t>, dim3(n_chunks), dim3(256), 0, s, d_chunks, counts);
      break;
    case 2:
      hipLaunchKernelGGL(hyk::scan_count_kernel<uint16_t>, dim3(n_chunks), dim3(256), 0, s, d_chunks, counts);
      break;
    default:
      hipLaunchKernelGGL(hyk::scan_count_kernel<uint32_t>, dim3(n_chunks), dim3(256), 0, s, d_chunks, counts);
      break;
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_expand_chunk_row_ids(const uint32_t* offsets, const uint64_t* chunk_begin, const uint32_t* chunk_ids,
                                  uint32_t n_chunks, hy_row_id* out, hy_stream_t stream) {
  if (n_chunks == 0) return HY_OK;
  if (!offsets || !chunk_begin || !out) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  hipLaunchKernelGGL(hyk::expand_chunk_row_ids_kernel, dim3(n_chunks), dim3(256), 0, S(stream), offsets, chunk_begin,
                     chunk_ids, out);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// ================================================================================================================
// Hashing
// ================================================================================================================
// MurmurHash2 over a byte string (reference murmur_hash.cpp:21-73; std::string keys, murmur_hash.hpp:16-20): the
// partitioning hash of string join keys, computed once per distinct string by the JoinHash operator.
uint32_t hy_murmur2_bytes(const void* bytes, uint32_t len, uint32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = seed ^ len;
  const auto* data = static_cast<const unsigned char*>(bytes);
  for (; len >= 4; data += 4, len -= 4) {
    uint32_t k;
    std::memcpy(&k, data, 4);
    h = hyk::murmur_mix_word(h, k);
  }
  switch (len) {
    case 3:
      h ^= static_cast<uint32_t>(data[2]) << 16;
      [[fallthrough]];
    case 2:
      h ^= static_cast<uint32_t>(data[1]) << 8;
      [[fallthrough]];
    case 1:
      h ^= data[0];
      h *= m;
  }
  return hyk::murmur_final(h);
}

hy_status hy_murmur2(const void* keys, uint64_t n, uint32_t key_bytes, uint32_t seed, uint32_t* out,
                     hy_stream_t stream) {
  if (n == 0) return HY_OK;
  if (key_bytes == 4) {
    hipLaunchKernelGGL(hyk::murmur_kernel_u32, dim3(grid_for(n, 256)), dim3(256), 0, S(stream),
                       static_cast<const uint32_t*>(keys), n, seed, out);
  } else if (key_bytes == 8) {
    hipLaunchKernelGGL(hyk::murmur_kernel_u64, dim3(grid_for(n, 256)), dim3(256), 0, S(stream),
                       static_cast<const uint64_t*>(keys), n, seed, out);
  } else {
    return fail(HY_ERR_UNSUPPORTED, "key_bytes must be 4 or 8");
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// JoinHashImpl ctor (reference join_hash.cpp:640-668), evaluated in the same float arithmetic:
//   size = B * (sizeof(T) + sizeof(void*)) + (B / 2) * (sizeof(PosList) + 2 * sizeof(RowID))
//   cluster_count = max(1.0f, (2.0f * size) / 256000); radix_bits = ceil(log2(cluster_count))
// sizeof(PosList) = 32 (std::vector with a polymorphic allocator), sizeof(RowID) = 8.
uint32_t hy_join_radix_bits(uint64_t build_rows, uint32_t key_bytes) {
  const uint64_t size = build_rows * (uint64_t(key_bytes) + 8) + (build_rows / 2) * (32 + 2 * 8);
  const float adaption = 2.0f;
  const float cluster_count = std::max(1.0f, (adaption * static_cast<float>(size)) / 256000);
  return static_cast<uint32_t>(std::ceil(std::log2(cluster_count)));
}

}  // extern "C"

// ================================================================================================================
// Measured HBM roofline: streaming read / copy kernels (16-byte nontemporal accesses, 4 per lane in flight)
// ================================================================================================================
namespace {

__global__ __launch_bounds__(256) void stream_read_kernel(const hyk::u32x4* __restrict__ src, uint64_t n16,
                                                          uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256 * 4;
  for (uint64_t i = blockIdx.x * 1024ull + threadIdx.x; i < n16; i += stride) {
    hyk::u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * 256 < n16 ? __builtin_nontemporal_load(src + i + k * 256) : hyk::u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x * 256 + threadIdx.x] = acc;  // keeps the loads live; practically never taken
}

__global__ __launch_bounds__(256) void stream_copy_kernel(const hyk::u32x4* __restrict__ src, hyk::u32x4* __restrict__ dst,
                                                          uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256 * 4;
  for (uint64_t i = blockIdx.x * 1024ull + threadIdx.x; i < n16; i += stride) {
    hyk::u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < n16) v[k] = __builtin_nontemporal_load(src + i + k * 256);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < n16) dst[i + k * 256] = v[k];
  }
}

}  // namespace

extern "C" {

hy_status hy_stream_bandwidth_probe(const void* src, void* dst, uint64_t bytes, int32_t mode, hy_stream_t stream) {
  if (!src || (mode == HY_PROBE_COPY && !dst)) return fail(HY_ERR_INVALID_ARGUMENT, "null buffer");
  if (!aligned16(src) || (dst && !aligned16(dst))) return fail(HY_ERR_ALIGNMENT, "buffers must be 16-byte aligned");
  const uint64_t n16 = bytes / 16;
  if (n16 == 0) return HY_OK;
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((n16 + 1023) / 1024, 256 * 32));
  if (mode == HY_PROBE_READ) {
    KTimer t("stream_read", S(stream), bytes);
    hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(256), 0, S(stream), static_cast<const hyk::u32x4*>(src), n16,
                       static_cast<uint32_t*>(dst));
    t.done();
  } else if (mode == HY_PROBE_COPY) {
    KTimer t("stream_copy", S(stream), bytes);
    hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, S(stream), static_cast<const hyk::u32x4*>(src),
                       static_cast<hyk::u32x4*>(dst), n16);
    t.done();
  } else {
    return fail(HY_ERR_INVALID_ARGUMENT, "mode");
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_dereference_row_ids(const hy_row_id* rows, uint64_t n, const hy_row_id* const* chunk_pos_lists,
                                 hy_row_id* out, hy_stream_t stream) {
  if (n == 0) return HY_OK;
  hipLaunchKernelGGL(hyk::dereference_kernel, dim3(grid_for(n, 256)), dim3(256), 0, S(stream), rows, n,
                     chunk_pos_lists, out);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

}  // extern "C"
