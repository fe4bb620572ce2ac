// C-ABI implementation (include/hyrise_amd.h): runtime wrappers, launch orchestration and workspace carving for
// the gfx950 TableScan / JoinHash kernels. Nothing here throws across the boundary; every failure becomes an
// hy_status plus a thread-local message.
#include <hip/hip_runtime.h>

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
uint64_t* g_join_trace = nullptr;
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

hy_status hy_stream_destroy(hy_stream_t stream) {
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

enum ScanClass { SC_DICT8, SC_DICT16, SC_DICT32, SC_VALUE, SC_COUNT };

int scan_class(const hy_scan_chunk& c) {
  if (c.column.kind == HY_COL_VALUE) return SC_VALUE;
  switch (c.column.vid_width) {
    case 1:
      return SC_DICT8;
    case 2:
      return SC_DICT16;
    case 4:
      return SC_DICT32;
  }
  return -1;
}

uint64_t scan_tiles(uint32_t size) { return (uint64_t(size) + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE; }

// tiles per scan workgroup for a column class (hyk::seg_tiles<E> of the class's element type)
int class_seg(int cls, int32_t value_type) {
  switch (cls) {
    case SC_DICT8:
      return hyk::seg_tiles<uint8_t>();
    case SC_DICT16:
      return hyk::seg_tiles<uint16_t>();
    case SC_DICT32:
      return hyk::seg_tiles<uint32_t>();
    default:
      return (value_type == HY_TYPE_INT64 || value_type == HY_TYPE_DOUBLE) ? hyk::seg_tiles<int64_t>()
                                                                          : hyk::seg_tiles<int32_t>();
  }
}

template <typename E, bool DICT, bool OUT_ROWID>
hy_status launch_scan(const hyk::ScanLaunchDesc& d, const void* constant, void* out, uint32_t* counts,
                      hipStream_t s) {
  hyk::ScanConst<E> c{};
  if (!DICT && constant) std::memcpy(&c.value, constant, sizeof(E));
  KTimer t(DICT ? "scan_dict" : "scan_value", s, d.n_rows);
  hipLaunchKernelGGL((hyk::scan_kernel<E, DICT, OUT_ROWID>), dim3(static_cast<uint32_t>(d.n_tiles)),
                     dim3(hyk::SCAN_THREADS), 0, s, d, c, out, counts);
  t.done();
  HY_HIP(hipGetLastError());
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
    if (cls < 0) return fail(HY_ERR_INVALID_ARGUMENT, "bad vid width");
    if (chunks[i].column.size && !aligned16(chunks[i].column.data))
      return fail(HY_ERR_ALIGNMENT, "column data not 16-byte aligned");
    if (chunks[i].column.nulls && !aligned16(chunks[i].column.nulls))
      return fail(HY_ERR_ALIGNMENT, "null vector not 16-byte aligned");
    by_class[cls].push_back(i);
  }
  if (!by_class[SC_VALUE].empty() &&
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
    uint64_t run = 0, rows = 0;
    for (uint32_t k = 0; k < nc; ++k) {
      hc[k] = chunks[idx[k]];
      rows += hc[k].column.size;
      ht[k] = run;
      const uint64_t seg = static_cast<uint64_t>(class_seg(cls, value_type));
      run += hc[k].op == HY_OP_NONE ? 0 : (scan_tiles(hc[k].column.size) + seg - 1) / seg;  // segments
    }
    ht[nc] = run;
    hyk::ScanLaunchDesc d{};
    auto* dch = cv.take<hy_scan_chunk>(nc);
    auto* dti = cv.take<uint64_t>(nc + 1);
    auto* dix = cv.take<uint32_t>(nc);
    auto* dcid = cv.take<uint32_t>(nc);
    auto* dst = cv.take<uint64_t>(run + 1);
    auto* downer = cv.take<uint32_t>(run + 1);
    auto* dmisc = cv.take<uint32_t>(64);
    if (!cv.ok) return fail(HY_ERR_WORKSPACE, "scan workspace too small");
    if (!error) {
      error = dmisc + 1;
      HY_HIP(hipMemsetAsync(error, 0, 4, s));
    }
    HY_HIP(hipMemcpyAsync(dch, hc.data(), sizeof(hy_scan_chunk) * nc, hipMemcpyHostToDevice, s));
    HY_HIP(hipMemcpyAsync(dti, ht.data(), sizeof(uint64_t) * (nc + 1), hipMemcpyHostToDevice, s));
    HY_HIP(hipMemcpyAsync(dix, idx.data(), sizeof(uint32_t) * nc, hipMemcpyHostToDevice, s));
    auto& hcid = h_cids[cls];
    hcid.resize(nc);
    for (uint32_t k = 0; k < nc; ++k) hcid[k] = chunk_ids ? chunk_ids[idx[k]] : idx[k];
    HY_HIP(hipMemcpyAsync(dcid, hcid.data(), sizeof(uint32_t) * nc, hipMemcpyHostToDevice, s));
    HY_HIP(hipMemsetAsync(dst, 0, sizeof(uint64_t) * (run + 1), s));
    HY_HIP(hipMemsetAsync(dmisc, 0, 4, s));
    if (run == 0) continue;
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((nc + 255) / 256), dim3(256), 0, s, dti, nc, downer);
    HY_HIP(hipGetLastError());
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
    hy_status st = HY_OK;
    switch (cls) {
      case SC_DICT8:
        st = launch_scan<uint8_t, true, OUT_ROWID>(d, nullptr, out_offsets, counts, s);
        break;
      case SC_DICT16:
        st = launch_scan<uint16_t, true, OUT_ROWID>(d, nullptr, out_offsets, counts, s);
        break;
      case SC_DICT32:
        st = launch_scan<uint32_t, true, OUT_ROWID>(d, nullptr, out_offsets, counts, s);
        break;
      case SC_VALUE:
        switch (value_type) {
          case HY_TYPE_INT32:
            st = launch_scan<int32_t, false, OUT_ROWID>(d, constant, out_offsets, counts, s);
            break;
          case HY_TYPE_INT64:
            st = launch_scan<int64_t, false, OUT_ROWID>(d, constant, out_offsets, counts, s);
            break;
          case HY_TYPE_FLOAT:
            st = launch_scan<float, false, OUT_ROWID>(d, constant, out_offsets, counts, s);
            break;
          case HY_TYPE_DOUBLE:
            st = launch_scan<double, false, OUT_ROWID>(d, constant, out_offsets, counts, s);
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
  const uint64_t tiles = (pos_list_size + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE;
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  auto* dst = cv.take<uint64_t>(tiles + 1);
  auto* dmisc = cv.take<uint32_t>(64);
  auto* dch = cv.take<hy_scan_chunk>(std::max<uint32_t>(1, n_referenced_chunks));
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "reference scan workspace too small");
  HY_HIP(hipMemsetAsync(dst, 0, sizeof(uint64_t) * (tiles + 1), s));
  HY_HIP(hipMemsetAsync(dmisc, 0, 256, s));
  HY_HIP(hipMemcpyAsync(dch, referenced_chunks, sizeof(hy_scan_chunk) * n_referenced_chunks, hipMemcpyHostToDevice, s));
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
        if (referenced_chunks[i].column.kind != HY_COL_DICT && referenced_chunks[i].op != HY_OP_NONE)
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

// ================================================================================================================
// Hashing
// ================================================================================================================
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
// JoinHash
// ================================================================================================================
namespace {

// Tiles per span of the pass from column chunks (sub1) and of the record passes (sub2); HY_PART_SUB1 / HY_PART_SUB2
// override them (tuning). Read once: workspace sizes and launches must agree.
uint32_t sub_from_env(const char* name, uint32_t dflt) {
  const char* e = std::getenv(name);
  const long v = e ? std::strtol(e, nullptr, 10) : 0;
  return v >= 1 && v <= hyk::PART_SUB_MAX ? static_cast<uint32_t>(v) : dflt;
}
uint32_t sub1() {
  static const uint32_t v = sub_from_env("HY_PART_SUB1", 1);
  return v;
}
uint32_t sub2() {
  static const uint32_t v = sub_from_env("HY_PART_SUB2", 1);
  return v;
}
uint64_t span1() { return uint64_t(sub1()) * hyk::PART_TILE; }
uint64_t span2() { return uint64_t(sub2()) * hyk::PART_TILE; }


struct SidePlan {
  uint64_t n_rows = 0;
  uint64_t n_tiles1 = 0;
  std::vector<hyk::SrcChunk> chunks;
  std::vector<uint64_t> tile_begin;
  std::vector<uint64_t> row_begin;       // this table
  std::vector<hyk::SrcChunk> referenced;
  std::vector<uint64_t> ref_row_begin;   // referenced table
  int32_t fuse = 0;
  uint32_t ref_base = 0;                 // referenced_chunk_base of the side
  uint32_t map_uniform = 0;              // output RowID map (this table or referenced table when fused)
};

uint32_t uniform_of(const std::vector<uint64_t>& row_begin) {
  const size_t n = row_begin.size() - 1;
  if (n == 0) return 0;
  if (n == 1) return static_cast<uint32_t>(std::max<uint64_t>(row_begin[1], 1));
  const uint64_t u = row_begin[1] - row_begin[0];
  if (u == 0) return 0;
  for (size_t i = 1; i + 1 < n; ++i)
    if (row_begin[i + 1] - row_begin[i] != u) return 0;
  if (row_begin[n] - row_begin[n - 1] > u) return 0;
  return static_cast<uint32_t>(u);
}

hyk::SrcChunk src_from(const hy_column_chunk& c, const hy_row_id* pos_list, uint32_t size, uint64_t row_begin,
                       uint32_t single_chunk = HY_MIXED_CHUNKS) {
  hyk::SrcChunk s{};
  s.single_chunk = single_chunk;
  s.data = c.data;
  s.nulls = c.nulls;
  s.dictionary = c.dictionary;
  s.pos_list = pos_list;
  s.size = size;
  s.dictionary_size = c.dictionary_size;
  s.kind = c.kind;
  s.vid_width = c.vid_width;
  s.row_begin = row_begin;
  return s;
}

hy_status plan_side(const hy_join_side* side, SidePlan& p) {
  if (!side || (side->n_chunks && !side->chunks)) return fail(HY_ERR_INVALID_ARGUMENT, "join side");
  p.ref_base = side->referenced_chunk_base;
  p.chunks.resize(side->n_chunks);
  p.tile_begin.resize(side->n_chunks + 1);
  p.row_begin.resize(side->n_chunks + 1);
  bool is_ref = false;
  uint64_t rows = 0, tiles = 0;
  for (uint32_t i = 0; i < side->n_chunks; ++i) {
    const hy_join_chunk& c = side->chunks[i];
    if (c.pos_list) is_ref = true;
    p.chunks[i] = src_from(c.column, c.pos_list, c.size, rows, c.single_chunk);
    p.chunks[i].chunk_id = c.chunk_id;
    p.row_begin[i] = rows;
    p.tile_begin[i] = tiles;
    rows += c.size;
    tiles += (uint64_t(c.size) + span1() - 1) / span1();
  }
  p.row_begin[side->n_chunks] = rows;
  p.tile_begin[side->n_chunks] = tiles;
  p.n_rows = rows;
  p.n_tiles1 = tiles;
  if (rows >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "join side exceeds 2^32-1 rows");
  if (is_ref) {
    p.referenced.resize(side->n_referenced);
    p.ref_row_begin.resize(side->n_referenced + 1);
    uint64_t rr = 0;
    for (uint32_t i = 0; i < side->n_referenced; ++i) {
      p.referenced[i] = src_from(side->referenced[i], nullptr, side->referenced[i].size, rr);
      p.ref_row_begin[i] = rr;
      rr += side->referenced[i].size;
    }
    p.ref_row_begin[side->n_referenced] = rr;
    for (const auto& c : p.chunks)
      if (c.pos_list && c.single_chunk != HY_MIXED_CHUNKS && c.single_chunk >= side->n_referenced)
        return fail(HY_ERR_INVALID_ARGUMENT, "single_chunk outside the referenced chunks");
    if (rr >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "referenced table exceeds 2^32-1 rows");
  }
  return HY_OK;
}

// Radix digits from the most significant: the partition id has `bits` bits; the first digit may be narrower than 8 so
// that the others are 8 bits wide; min_top forces the first digit to be at least that wide (the distributed join
// assigns whole first-digit buckets to ranks).
std::vector<uint32_t> digit_plan(uint32_t bits, uint32_t min_top) {
  std::vector<uint32_t> w;
  if (bits == 0) return w;
  uint32_t top = bits - 8 * ((bits - 1) / 8);
  if (top < min_top) top = std::min(min_top, bits);
  w.push_back(top);
  uint32_t rest = bits - top;
  if (rest) {
    const uint32_t q = (rest + 7) / 8;
    w.push_back(rest - 8 * (q - 1));
    for (uint32_t i = 1; i < q; ++i) w.push_back(8);
  }
  return w;
}

// Device pointers of one side inside the workspace.
template <typename H, typename P = uint32_t>
struct SideBufs {
  hyk::SrcChunk* chunks;
  uint64_t* tile_begin;
  uint64_t* row_begin;
  hyk::SrcChunk* referenced;
  uint64_t* ref_row_begin;
  uint32_t* hist;            // histogram of the current pass (largest pass)
  uint32_t* off;             // its exclusive scan
  hyk::Rec<H, P>* recA;
  hyk::Rec<H, P>* recB;
  uint32_t* segA;            // segment / partition bounds, ping-pong (2^bits + 1 entries)
  uint32_t* segB;
  uint64_t* seg_tile_begin;  // 2^bits + 1
  uint32_t* tile_counts;     // 2^bits
  uint32_t* tile_excl;       // 2^bits
  uint32_t* tile_owner;      // largest pass's tiles
  uint64_t* total;           // rows taking part (device)
};

struct SideSizes {
  uint64_t rows = 0, tiles1 = 0;   // pass-0 tiles (0: the side starts from received records)
  size_t n_chunks = 0, n_referenced = 0;
};

// Largest histogram of any pass, and the largest tile count of any record pass.
void pass_sizes(const SideSizes& z, const std::vector<uint32_t>& w, uint64_t first_segs, uint64_t* hist_words,
                uint64_t* max_tiles) {
  *hist_words = 1;
  *max_tiles = 1;
  uint64_t segs = first_segs;
  for (size_t i = 0; i < w.size(); ++i) {
    const uint64_t digits = 1ull << w[i];
    if (i == 0 && z.tiles1) {
      *hist_words = std::max(*hist_words, digits * z.tiles1);
      *max_tiles = std::max(*max_tiles, z.tiles1);
    } else {
      const uint64_t t = (z.rows + span2() - 1) / span2() + segs;
      *hist_words = std::max(*hist_words, digits * t);
      *max_tiles = std::max(*max_tiles, t);
      segs *= digits;
      continue;
    }
    segs = digits;
  }
}

template <typename H, typename P>
void carve_side(Carver& cv, const SideSizes& z, uint32_t bits, const std::vector<uint32_t>& w, uint64_t first_segs,
                bool own_recA, SideBufs<H, P>& b) {
  b.chunks = cv.take<hyk::SrcChunk>(std::max<size_t>(1, z.n_chunks));
  b.tile_begin = cv.take<uint64_t>(z.n_chunks + 1);
  b.row_begin = cv.take<uint64_t>(z.n_chunks + 1);
  b.referenced = cv.take<hyk::SrcChunk>(std::max<size_t>(1, z.n_referenced));
  b.ref_row_begin = cv.take<uint64_t>(z.n_referenced + 1);
  uint64_t hist_words, max_tiles;
  pass_sizes(z, w, first_segs, &hist_words, &max_tiles);
  b.hist = cv.take<uint32_t>(hist_words);
  b.off = cv.take<uint32_t>(hist_words);
  b.recA = own_recA ? cv.take<hyk::Rec<H, P>>(std::max<uint64_t>(1, z.rows)) : nullptr;
  b.recB = cv.take<hyk::Rec<H, P>>(std::max<uint64_t>(1, z.rows));
  const uint64_t parts = (uint64_t(1) << bits) + 1;
  b.segA = cv.take<uint32_t>(parts);
  b.segB = cv.take<uint32_t>(parts);
  b.seg_tile_begin = cv.take<uint64_t>(parts);
  b.tile_counts = cv.take<uint32_t>(parts);
  b.tile_excl = cv.take<uint32_t>(parts);
  b.tile_owner = cv.take<uint32_t>(max_tiles);
  b.total = cv.take<uint64_t>(1);
}

struct Common {
  uint64_t* scan_status;
  uint64_t scan_status_words;
  uint32_t* misc;  // [0] ticket [1] error [2] overflow ...
  uint64_t* totals;
  uint64_t* join_status;
};

void carve_common(Carver& cv, uint64_t max_scan, uint32_t bits, Common* c) {
  c->scan_status_words = max_scan / hyk::SCAN_BLOCK + 2;
  c->scan_status = cv.take<uint64_t>(c->scan_status_words);
  c->misc = cv.take<uint32_t>(64);
  c->totals = cv.take<uint64_t>(8);
  c->join_status = cv.take<uint64_t>((uint64_t(1) << bits) + 1);
}

hy_status run_scan(const uint32_t* in, uint32_t* out, uint64_t n, const Common& c, hipStream_t s,
                   uint64_t* total_out = nullptr) {
  if (n == 0) {
    if (total_out) HY_HIP(hipMemsetAsync(total_out, 0, 8, s));
    return HY_OK;
  }
  const uint64_t tiles = (n + hyk::SCAN_BLOCK - 1) / hyk::SCAN_BLOCK;
  if (tiles + 1 > c.scan_status_words) return fail(HY_ERR_WORKSPACE, "scan status");
  HY_HIP(hipMemsetAsync(c.scan_status, 0, sizeof(uint64_t) * (tiles + 1), s));
  HY_HIP(hipMemsetAsync(c.misc, 0, 4, s));
  KTimer kt_("exclusive_scan", s, n);
  const bool vec = reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
  hipLaunchKernelGGL(vec ? hyk::exclusive_scan_u32<true> : hyk::exclusive_scan_u32<false>,
                     dim3(static_cast<uint32_t>(tiles)), dim3(hyk::SCAN_T), 0, s, in, out, n, c.scan_status, c.misc,
                     c.misc + 1, total_out);
  kt_.done();
  HY_HIP(hipGetLastError());
  return HY_OK;
}

uint32_t full_mask(uint32_t bits) { return bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u); }

// The load path every chunk of the side allows (hyk::LP_*): lean kernels for the all-value and all-single-chunk
// reference sides, the general one otherwise.
int load_path(const SidePlan& p) {
  bool value = true, ref1 = true;
  for (const auto& c : p.chunks) {
    if (c.size == 0) continue;
    value = value && c.pos_list == nullptr && c.kind == HY_COL_VALUE && c.nulls == nullptr;
    ref1 = ref1 && c.pos_list != nullptr && c.single_chunk != HY_MIXED_CHUNKS &&
           p.referenced[c.single_chunk].kind == HY_COL_VALUE && p.referenced[c.single_chunk].nulls == nullptr &&
           p.referenced[c.single_chunk].size > 0;
  }
  if (value) return hyk::LP_VALUE;
  return ref1 ? hyk::LP_REF1 : hyk::LP_ANY;
}

// Pass 0: from column chunks into b.recA (or `out`), bucket bounds into b.segA (2^w0 buckets).
template <typename T, typename H, typename P>
hy_status pass0_side(const char* side_tag, const SidePlan& p, const SideBufs<H, P>& b, uint32_t bits, uint32_t w0,
                     uint32_t seed, bool keep_nulls, uint32_t ref_base, const Common& c, hipStream_t s,
                     hyk::Rec<H, P>* out) {
  hyk::Side sd{};
  sd.chunks = b.chunks;
  sd.n_chunks = static_cast<uint32_t>(p.chunks.size());
  sd.chunk_tile_begin = b.tile_begin;
  sd.tile_chunk = b.tile_owner;
  sd.n_tiles = p.n_tiles1;
  sd.referenced = b.referenced;
  sd.n_referenced = static_cast<uint32_t>(p.referenced.size());
  sd.referenced_row_begin = b.ref_row_begin;
  sd.fuse_deref = p.fuse;
  sd.keep_nulls = keep_nulls ? 1 : 0;
  sd.ref_base = ref_base;
  sd.sub = sub1();
  const uint32_t n_digits = 1u << w0;
  hyk::Digit d0{full_mask(bits), bits - w0, n_digits - 1u, seed};
  HY_HIP(hipMemsetAsync(b.total, 0, 8, s));
  if (p.n_tiles1 > 0) {
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((sd.n_chunks + 255) / 256), dim3(256), 0, s, b.tile_begin,
                       sd.n_chunks, b.tile_owner);
    HY_HIP(hipGetLastError());
    const int lp = load_path(p);
    {
      KTimer kt_((std::string("part1_hist.") + side_tag).c_str(), s, p.n_rows);
      auto kern = lp == hyk::LP_VALUE  ? hyk::part1_hist<T, H, hyk::LP_VALUE>
                  : lp == hyk::LP_REF1 ? hyk::part1_hist<T, H, hyk::LP_REF1>
                                       : hyk::part1_hist<T, H, hyk::LP_ANY>;
      hipLaunchKernelGGL(kern, dim3(static_cast<uint32_t>(p.n_tiles1)), dim3(hyk::PART_THREADS), 0, s, sd, d0,
                         n_digits, b.hist);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    hy_status st = run_scan(b.hist, b.off, uint64_t(n_digits) * p.n_tiles1, c, s, b.total);
    if (st != HY_OK) return st;
    {
      KTimer kt_((std::string("part1_scatter.") + side_tag).c_str(), s, p.n_rows);
      auto kern = lp == hyk::LP_VALUE  ? hyk::part1_scatter<T, H, P, hyk::LP_VALUE>
                  : lp == hyk::LP_REF1 ? hyk::part1_scatter<T, H, P, hyk::LP_REF1>
                                       : hyk::part1_scatter<T, H, P, hyk::LP_ANY>;
      hipLaunchKernelGGL(kern, dim3(static_cast<uint32_t>(p.n_tiles1)), dim3(hyk::PART_THREADS), 0, s, sd, d0,
                         static_cast<int>(w0), n_digits, b.off, out);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(hyk::seg_bounds, dim3((n_digits + 1 + 255) / 256), dim3(256), 0, s, b.off, p.n_tiles1, n_digits,
                     b.total, b.segA);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// One record pass over segments sg (tile prefix and owners filled, grid = an upper bound of its tiles): histogram,
// scan, stable scatter by digit (bits [shift, shift + w)), then the bounds of the n_groups * 2^w parts.
template <typename H, typename P>
hy_status record_pass(const char* side_tag, const SideBufs<H, P>& b, const hyk::Segs& sg, const hyk::Groups& gr,
                      uint32_t n_groups, uint64_t grid, uint32_t bits, uint32_t shift, uint32_t w, uint32_t seed,
                      const hyk::Rec<H, P>* in, hyk::Rec<H, P>* out, const uint64_t* total, uint32_t* bounds,
                      const Common& c, hipStream_t s, uint64_t rows) {
  const uint32_t n_digits = 1u << w;
  hyk::Digit dg{full_mask(bits), shift, n_digits - 1u, seed};
  if (grid) {
    {
      KTimer kt_((std::string("part2_hist.") + side_tag).c_str(), s, rows);
      hipLaunchKernelGGL((hyk::part2_hist<H, P>), dim3(static_cast<uint32_t>(grid)), dim3(hyk::PART_THREADS), 0, s,
                         sg, dg, n_digits, in, b.hist);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    hy_status st = run_scan(b.hist, b.off, grid * n_digits, c, s);
    if (st != HY_OK) return st;
    {
      KTimer kt_((std::string("part2_scatter.") + side_tag).c_str(), s, rows);
      hipLaunchKernelGGL((hyk::part2_scatter<H, P>), dim3(static_cast<uint32_t>(grid)), dim3(hyk::PART_THREADS), 0, s,
                         sg, dg, static_cast<int>(w), n_digits, in, b.off, out);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
  }
  const uint64_t nb = uint64_t(n_groups) * n_digits + 1;
  hipLaunchKernelGGL(hyk::pass_bounds, dim3(grid_for(nb, 256)), dim3(256), 0, s, b.off, sg, gr, n_groups, n_digits,
                     total, bounds);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// Record passes over contiguous segments (bounds in `seg`, n_segs of them) for digits w[first..]: ping-pong between
// the two record buffers. On return *recs / *bounds hold the final records and partition bounds.
template <typename H, typename P>
hy_status local_passes(const char* side_tag, SideBufs<H, P>& b, const std::vector<uint32_t>& w, size_t first,
                       uint32_t bits, uint32_t seed, hyk::Rec<H, P>* in, hyk::Rec<H, P>* spare, uint32_t* seg,
                       uint32_t* seg_spare, uint64_t n_segs, const uint64_t* total, uint64_t rows, const Common& c,
                       hipStream_t s, hyk::Rec<H, P>** recs, uint32_t** bounds) {
  uint32_t below = 0;
  for (size_t i = first; i < w.size(); ++i) below += w[i];
  for (size_t i = first; i < w.size(); ++i) {
    below -= w[i];
    hipLaunchKernelGGL(hyk::seg_tile_counts, dim3(grid_for(n_segs, 256)), dim3(256), 0, s, seg, nullptr,
                       static_cast<uint32_t>(n_segs), span2(), b.tile_counts);
    HY_HIP(hipGetLastError());
    hy_status st = run_scan(b.tile_counts, b.tile_excl, n_segs, c, s, c.totals + 4);
    if (st != HY_OK) return st;
    hipLaunchKernelGGL(hyk::widen_prefix, dim3(grid_for(n_segs + 1, 256)), dim3(256), 0, s, b.tile_excl,
                       static_cast<uint32_t>(n_segs), c.totals + 4, b.seg_tile_begin);
    HY_HIP(hipGetLastError());
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3(grid_for(n_segs, 256)), dim3(256), 0, s, b.seg_tile_begin,
                       static_cast<uint32_t>(n_segs), b.tile_owner);
    HY_HIP(hipGetLastError());
    const uint64_t grid = rows ? (rows + span2() - 1) / span2() + n_segs : 0;
    hyk::Segs sg{seg,     b.seg_tile_begin, b.tile_owner, static_cast<uint32_t>(n_segs), nullptr, nullptr, nullptr,
                 nullptr, sub2()};
    st = record_pass<H, P>(side_tag, b, sg, hyk::Groups{nullptr, nullptr, nullptr}, static_cast<uint32_t>(n_segs), grid,
                           bits, below, w[i], seed, in, spare, total, seg_spare, c, s, rows);
    if (st != HY_OK) return st;
    std::swap(in, spare);
    std::swap(seg, seg_spare);
    n_segs <<= w[i];
  }
  *recs = in;
  *bounds = seg;
  return HY_OK;
}

hyk::RowMap make_map(const uint64_t* dev_row_begin, const std::vector<uint64_t>& host_row_begin) {
  hyk::RowMap m{};
  m.row_begin = dev_row_begin;
  m.n_chunks = static_cast<uint32_t>(host_row_begin.size() - 1);
  m.uniform = uniform_of(host_row_begin);
  m.magic = 0;
  if (m.uniform >= 2) {
    // floor(2^64 / u) + 1
    const unsigned __int128 two64 = static_cast<unsigned __int128>(1) << 64;
    m.magic = static_cast<uint64_t>(two64 / m.uniform) + 1;
  }
  return m;
}

// Per-partition LDS build/probe over partitioned records (partition bounds on the device).
template <typename H, typename P>
hy_status run_join_partitions(const uint32_t* build_begin, const uint32_t* probe_begin, uint32_t n_parts,
                              const hyk::Rec<H, P>* brec, const hyk::Rec<H, P>* precs, const hyk::RowMap& bmap,
                              const hyk::RowMap& pmap, int32_t mode, hy_row_id* out_build, hy_row_id* out_probe,
                              uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,
                              hy_join_result* result, const Common& c, hipStream_t s, uint64_t units) {
  // largest build partition decides the LDS table size
  std::vector<uint32_t> hb(n_parts + 1), hp(n_parts + 1);
  HY_HIP(hipMemcpyAsync(hb.data(), build_begin, sizeof(uint32_t) * (n_parts + 1), hipMemcpyDeviceToHost, s));
  HY_HIP(hipMemcpyAsync(hp.data(), probe_begin, sizeof(uint32_t) * (n_parts + 1), hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  uint32_t max_build = 0, max_probe = 0;
  for (uint32_t i = 0; i < n_parts; ++i) {
    max_build = std::max(max_build, hb[i + 1] - hb[i]);
    max_probe = std::max(max_probe, hp[i + 1] - hp[i]);
  }
  // probe records per thread per pass: JP_PER, or 6 when the largest probe partition needs more than one pass
  const bool wide = max_probe > static_cast<uint32_t>(hyk::JP_PER * hyk::JOIN_THREADS);
  // LDS budget: two 1024-thread workgroups per CU; a partition with more build rows than one table holds (skewed
  // keys) is processed as several LDS sub-tables in sequence
  size_t kLdsBudget = sizeof(hyk::Rec<H, P>) > 8 ? 72 * 1024 : 40 * 1024;
  if (const char* e = std::getenv("HY_JOIN_LDS_BUDGET")) kLdsBudget = std::strtoull(e, nullptr, 10);  // test knob
  uint32_t lds_max = std::min<uint32_t>(std::max<uint32_t>(max_build, 1), hyk::LDS_MAX_ROWS);
  while (lds_max > 16 && hyk::table_bytes<H, P>(lds_max) > kLdsBudget) lds_max = lds_max * 7 / 8;
  const size_t lds = hyk::table_bytes<H, P>(lds_max);

  hyk::JoinDesc jd{};
  jd.build_begin = build_begin;
  jd.probe_begin = probe_begin;
  jd.n_parts = n_parts;
  jd.lds_max_build = lds_max;
  jd.mode = mode;
  jd.build_map = bmap;
  jd.probe_map = pmap;
  jd.capacity = out_capacity;
  jd.error = c.misc + 1;
  jd.overflow = c.misc + 2;
  jd.total = c.totals + 1;
  jd.trace = g_join_trace;
  HY_HIP(hipMemsetAsync(c.misc, 0, 64 * 4, s));
  HY_HIP(hipMemsetAsync(c.totals, 0, 8 * 2, s));
  if (n_parts) {
    KTimer kt_("join_partition", s, units);
    auto launch = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3(n_parts), dim3(hyk::JOIN_THREADS), lds, s, jd, brec, precs, out_build, out_probe,
                         partition_begin, partition_counts);
    };
    if (jd.trace)  // debug phase-trace instance (hy_debug_set_join_trace)
      wide ? launch(hyk::join_partition<H, P, true, 6>) : launch(hyk::join_partition<H, P, true, hyk::JP_PER>);
    else
      wide ? launch(hyk::join_partition<H, P, false, 6>) : launch(hyk::join_partition<H, P, false, hyk::JP_PER>);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  uint32_t flags[4] = {0, 0, 0, 0};
  uint64_t total = 0;
  HY_HIP(hipMemcpyAsync(flags, c.misc, 16, hipMemcpyDeviceToHost, s));
  HY_HIP(hipMemcpyAsync(&total, c.totals + 1, 8, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  if (flags[1]) return fail(HY_ERR_KERNEL, "join look-back did not complete");
  if (result) {
    result->total_pairs = total;
    result->capacity_required = total;
  }
  if (flags[2] || total > out_capacity)
    return fail(HY_ERR_CAPACITY, "join output needs " + std::to_string(total) + " pairs");
  return HY_OK;
}

SideSizes sizes_of(const SidePlan& p) {
  SideSizes z;
  z.rows = p.n_rows;
  z.tiles1 = p.n_tiles1;
  z.n_chunks = p.chunks.size();
  z.n_referenced = p.referenced.size();
  return z;
}

template <typename H>
size_t join_bytes(const SidePlan& bp, const SidePlan& pp, uint32_t bits) {
  const auto w = digit_plan(bits, 0);
  Carver cv{nullptr, 0};
  SideBufs<H> a, b;
  carve_side<H, uint32_t>(cv, sizes_of(bp), bits, w, 1, true, a);
  carve_side<H, uint32_t>(cv, sizes_of(pp), bits, w, 1, true, b);
  uint64_t ha, hb, t;
  pass_sizes(sizes_of(bp), w, 1, &ha, &t);
  pass_sizes(sizes_of(pp), w, 1, &hb, &t);
  Common c;
  carve_common(cv, std::max({ha, hb, (uint64_t(1) << bits) + 1}), bits, &c);
  return cv.used + 256;
}

template <typename H, typename P>
hy_status upload_side(const SidePlan& p, const SideBufs<H, P>& b, hipStream_t s) {
  auto upload = [&](auto* dst, const auto& v) -> hy_status {
    if (!v.empty()) HY_HIP(hipMemcpyAsync(dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, s));
    return HY_OK;
  };
  if (upload(b.chunks, p.chunks) || upload(b.tile_begin, p.tile_begin) || upload(b.row_begin, p.row_begin) ||
      upload(b.referenced, p.referenced) || upload(b.ref_row_begin, p.ref_row_begin))
    return HY_ERR_DEVICE;
  return HY_OK;
}

template <typename TB, typename TP, typename H>
hy_status join_typed(const SidePlan& bp, const SidePlan& pp, const hy_join_params* prm, hy_row_id* out_build,
                     hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                     uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                     hipStream_t s) {
  const uint32_t bits = prm->radix_bits;
  if (workspace_bytes < join_bytes<H>(bp, pp, bits)) return fail(HY_ERR_WORKSPACE, "join workspace too small");
  const auto w = digit_plan(bits, 0);
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  SideBufs<H> bb, pb;
  carve_side<H, uint32_t>(cv, sizes_of(bp), bits, w, 1, true, bb);
  carve_side<H, uint32_t>(cv, sizes_of(pp), bits, w, 1, true, pb);
  uint64_t ha, hb2, t;
  pass_sizes(sizes_of(bp), w, 1, &ha, &t);
  pass_sizes(sizes_of(pp), w, 1, &hb2, &t);
  Common c{};
  carve_common(cv, std::max({ha, hb2, (uint64_t(1) << bits) + 1}), bits, &c);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "join workspace too small");
  if (upload_side(bp, bb, s) || upload_side(pp, pb, s)) return HY_ERR_DEVICE;
  const bool keep_nulls = prm->mode == HY_JOIN_LEFT || prm->mode == HY_JOIN_RIGHT;

  hyk::Rec<H>* recs[2] = {nullptr, nullptr};
  uint32_t* bounds[2] = {nullptr, nullptr};
  for (int side = 0; side < 2; ++side) {
    const SidePlan& p = side == 0 ? bp : pp;
    SideBufs<H>& b = side == 0 ? bb : pb;
    const char* tag = side == 0 ? "build" : "probe";
    hy_status st = side == 0
                       ? pass0_side<TB, H, uint32_t>(tag, p, b, bits, w.empty() ? 0 : w[0], prm->seed, false,
                                                     p.ref_base, c, s, b.recA)
                       : pass0_side<TP, H, uint32_t>(tag, p, b, bits, w.empty() ? 0 : w[0], prm->seed, keep_nulls,
                                                     p.ref_base, c, s, b.recA);
    if (st != HY_OK) return st;
    st = local_passes<H, uint32_t>(tag, b, w, 1, bits, prm->seed, b.recA, b.recB, b.segA, b.segB,
                                   w.empty() ? 1 : (1ull << w[0]), b.total, p.n_rows, c, s, &recs[side], &bounds[side]);
    if (st != HY_OK) return st;
  }
  const hyk::RowMap bmap = bp.fuse ? make_map(bb.ref_row_begin, bp.ref_row_begin) : make_map(bb.row_begin, bp.row_begin);
  const hyk::RowMap pmap = pp.fuse ? make_map(pb.ref_row_begin, pp.ref_row_begin) : make_map(pb.row_begin, pp.row_begin);
  return run_join_partitions<H, uint32_t>(bounds[0], bounds[1], 1u << bits, recs[0], recs[1], bmap, pmap, prm->mode,
                                          out_build, out_probe, out_capacity, partition_begin, partition_counts,
                                          result, c, s, bp.n_rows + pp.n_rows);
}

// ---------------------------------------------------------------------------------------------------------------
// Distributed JoinHash: exchange records are Rec<H, hy_row_id> (16 bytes: key, global RowID).
// ---------------------------------------------------------------------------------------------------------------
uint32_t ceil_log2(uint32_t n) {
  uint32_t b = 0;
  while ((1u << b) < n) ++b;
  return b;
}

template <typename H>
size_t exchange_partition_bytes(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w) {
  Carver cv{nullptr, 0};
  SideBufs<H, hy_row_id> b;
  SideSizes z = sizes_of(p);
  carve_side<H, hy_row_id>(cv, z, bits, std::vector<uint32_t>(w.begin(), w.begin() + 1), 1, false, b);
  Common c;
  carve_common(cv, std::max<uint64_t>((1ull << w[0]) * std::max<uint64_t>(1, p.n_tiles1), 2), bits, &c);
  return cv.used + 256;
}

// Receiver geometry of one side: runs (bucket j, sender s) of the received buffer, listed j-major.
struct RecvPlan {
  uint64_t rows = 0, tiles = 0;
  std::vector<uint32_t> seg_begin, seg_end, seg_stride, seg_toff;
  std::vector<uint64_t> seg_tile_begin, seg_hbase, group_hbase;
  std::vector<uint32_t> group_tiles, group_out;
  uint64_t hist_words = 1;
};

RecvPlan recv_plan(const uint64_t* counts, uint32_t n_senders, uint32_t nb, uint32_t digits) {
  RecvPlan r;
  std::vector<uint64_t> sender_base(n_senders + 1, 0);
  for (uint32_t s = 0; s < n_senders; ++s) {
    uint64_t n = 0;
    for (uint32_t j = 0; j < nb; ++j) n += counts[uint64_t(s) * nb + j];
    sender_base[s + 1] = sender_base[s] + n;
  }
  r.rows = sender_base[n_senders];
  const uint32_t nseg = nb * n_senders;
  r.seg_begin.resize(nseg);
  r.seg_end.resize(nseg);
  r.seg_stride.resize(nseg);
  r.seg_toff.resize(nseg);
  r.seg_hbase.resize(nseg);
  r.seg_tile_begin.resize(nseg + 1);
  r.group_hbase.resize(nb);
  r.group_tiles.resize(nb);
  r.group_out.resize(nb);
  std::vector<uint64_t> run_in_sender(n_senders, 0);
  uint64_t tiles = 0, hbase = 0, out = 0;
  for (uint32_t j = 0; j < nb; ++j) {
    uint32_t gt = 0;
    r.group_out[j] = static_cast<uint32_t>(out);
    for (uint32_t s = 0; s < n_senders; ++s) {
      const uint64_t cnt = counts[uint64_t(s) * nb + j];
      const uint32_t q = j * n_senders + s;
      const uint64_t b0 = sender_base[s] + run_in_sender[s];
      run_in_sender[s] += cnt;
      r.seg_begin[q] = static_cast<uint32_t>(b0);
      r.seg_end[q] = static_cast<uint32_t>(b0 + cnt);
      const uint32_t t = static_cast<uint32_t>((cnt + span2() - 1) / span2());
      r.seg_tile_begin[q] = tiles;
      r.seg_toff[q] = gt;
      tiles += t;
      gt += t;
      out += cnt;
    }
    r.group_tiles[j] = gt;
    r.group_hbase[j] = hbase;
    for (uint32_t s = 0; s < n_senders; ++s) {
      r.seg_hbase[j * n_senders + s] = hbase;
      r.seg_stride[j * n_senders + s] = gt;
    }
    hbase += uint64_t(gt) * digits;
  }
  r.seg_tile_begin[nseg] = tiles;
  r.tiles = tiles;
  r.hist_words = std::max<uint64_t>(1, hbase);
  return r;
}

// Receiver device buffers of one side.
template <typename H>
struct RecvBufs {
  SideBufs<H, hy_row_id> b;
  uint32_t *seg_begin, *seg_end, *seg_stride, *seg_toff, *group_tiles, *group_out, *owner;
  uint64_t *seg_tile_begin, *seg_hbase, *group_hbase;
};

template <typename H>
void carve_recv(Carver& cv, const RecvPlan& r, uint32_t bits, const std::vector<uint32_t>& w, uint32_t nb,
                uint32_t n_senders, RecvBufs<H>& rb) {
  SideSizes z;
  z.rows = r.rows;
  std::vector<uint32_t> tail(w.begin() + 1, w.end());
  if (tail.empty()) tail.push_back(0);
  carve_side<H, hy_row_id>(cv, z, bits, tail, uint64_t(nb) * n_senders, true, rb.b);
  const uint32_t nseg = std::max<uint32_t>(1, nb * n_senders);
  rb.seg_begin = cv.take<uint32_t>(nseg);
  rb.seg_end = cv.take<uint32_t>(nseg);
  rb.seg_stride = cv.take<uint32_t>(nseg);
  rb.seg_toff = cv.take<uint32_t>(nseg);
  rb.seg_tile_begin = cv.take<uint64_t>(nseg + 1);
  rb.seg_hbase = cv.take<uint64_t>(nseg);
  rb.group_hbase = cv.take<uint64_t>(std::max<uint32_t>(1, nb));
  rb.group_tiles = cv.take<uint32_t>(std::max<uint32_t>(1, nb));
  rb.group_out = cv.take<uint32_t>(std::max<uint32_t>(1, nb));
  rb.owner = cv.take<uint32_t>(std::max<uint64_t>(1, r.tiles));
}

template <typename H>
hy_status recv_side(const char* tag, const RecvPlan& r, RecvBufs<H>& rb, const std::vector<uint32_t>& w, uint32_t bits,
                    uint32_t nb, uint32_t n_senders, uint32_t seed, const hyk::Rec<H, hy_row_id>* in,
                    const Common& c, hipStream_t s, hyk::Rec<H, hy_row_id>** recs, uint32_t** bounds) {
  auto up = [&](auto* dst, const auto& v) -> hy_status {
    if (!v.empty()) HY_HIP(hipMemcpyAsync(dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, s));
    return HY_OK;
  };
  if (up(rb.seg_begin, r.seg_begin) || up(rb.seg_end, r.seg_end) || up(rb.seg_stride, r.seg_stride) ||
      up(rb.seg_toff, r.seg_toff) || up(rb.seg_tile_begin, r.seg_tile_begin) || up(rb.seg_hbase, r.seg_hbase) ||
      up(rb.group_hbase, r.group_hbase) || up(rb.group_tiles, r.group_tiles) || up(rb.group_out, r.group_out))
    return HY_ERR_DEVICE;
  HY_HIP(hipMemcpyAsync(rb.b.total, &r.rows, 8, hipMemcpyHostToDevice, s));
  const uint32_t nseg = nb * n_senders;
  if (r.tiles) {
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3(grid_for(nseg, 256)), dim3(256), 0, s, rb.seg_tile_begin, nseg,
                       rb.owner);
    HY_HIP(hipGetLastError());
  }
  const uint32_t w1 = w.size() > 1 ? w[1] : 0;  // one digit only: a stable merge of the senders' runs
  const uint32_t shift = bits - w[0] - w1;
  hyk::Segs sg{rb.seg_begin, rb.seg_tile_begin, rb.owner,    nseg,   rb.seg_end,
               rb.seg_hbase, rb.seg_stride,     rb.seg_toff, sub2()};
  hyk::Groups gr{rb.group_hbase, rb.group_tiles, rb.group_out};
  // the merge pass must not write through a stale histogram entry: hist words are exactly the groups' tiles x digits
  hy_status st = record_pass<H, hy_row_id>(tag, rb.b, sg, gr, nb, r.tiles, bits, shift, w1, seed, in, rb.b.recA,
                                           rb.b.total, rb.b.segA, c, s, r.rows);
  if (st != HY_OK) return st;
  return local_passes<H, hy_row_id>(tag, rb.b, w, 2, bits, seed, rb.b.recA, rb.b.recB, rb.b.segA, rb.b.segB,
                                    uint64_t(nb) << w1, rb.b.total, r.rows, c, s, recs, bounds);
}

template <typename H>
size_t exchange_join_bytes(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits, const std::vector<uint32_t>& w,
                           uint32_t nb, uint32_t n_senders) {
  Carver cv{nullptr, 0};
  RecvBufs<H> a, b;
  carve_recv<H>(cv, rbp, bits, w, nb, n_senders, a);
  carve_recv<H>(cv, rpp, bits, w, nb, n_senders, b);
  Common c;
  const uint64_t max_scan = std::max({rbp.hist_words * 2, rpp.hist_words * 2, (uint64_t(1) << bits) + 1,
                                      (rbp.rows + rpp.rows) / span2() * 256 + uint64_t(nb) * n_senders * 256});
  carve_common(cv, max_scan, bits, &c);
  return cv.used + 256;
}

int type_bytes(int32_t t) { return (t == HY_TYPE_INT32 || t == HY_TYPE_FLOAT) ? 4 : (t == HY_TYPE_INT64 || t == HY_TYPE_DOUBLE) ? 8 : 0; }

template <typename F>
hy_status dispatch_type(int32_t t, F&& f) {
  switch (t) {
    case HY_TYPE_INT32:
      return f(int32_t{});
    case HY_TYPE_INT64:
      return f(int64_t{});
    case HY_TYPE_FLOAT:
      return f(float{});
    case HY_TYPE_DOUBLE:
      return f(double{});
  }
  return fail(HY_ERR_UNSUPPORTED, "join column type");
}

hy_status prepare(const hy_join_side* build, const hy_join_side* probe, const hy_join_params* params, SidePlan& bp,
                  SidePlan& pp) {
  if (!params) return fail(HY_ERR_INVALID_ARGUMENT, "params");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (!(params->mode == HY_JOIN_INNER || params->mode == HY_JOIN_LEFT || params->mode == HY_JOIN_RIGHT ||
        params->mode == HY_JOIN_SEMI || params->mode == HY_JOIN_ANTI))
    return fail(HY_ERR_UNSUPPORTED, "join mode");
  hy_status st = plan_side(build, bp);
  if (st != HY_OK) return st;
  st = plan_side(probe, pp);
  if (st != HY_OK) return st;
  // fuse the dereference when the side is a reference table (one PosList per chunk shared by the join column)
  bp.fuse = (!bp.referenced.empty() && build->fuse_dereference) ? 1 : 0;
  pp.fuse = (!pp.referenced.empty() && probe->fuse_dereference) ? 1 : 0;
  if (!type_bytes(build->value_type) || !type_bytes(probe->value_type) || !type_bytes(params->hashed_type))
    return fail(HY_ERR_UNSUPPORTED, "join column type");
  return HY_OK;
}

}  // namespace

extern "C" {

hy_status hy_join_hash_workspace_size(const hy_join_side* build, const hy_join_side* probe,
                                      const hy_join_params* params, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "bytes");
  SidePlan bp, pp;
  hy_status st = prepare(build, probe, params, bp, pp);
  if (st != HY_OK) return st;
  *bytes = type_bytes(params->hashed_type) == 4 ? join_bytes<int32_t>(bp, pp, params->radix_bits)
                                                : join_bytes<int64_t>(bp, pp, params->radix_bits);
  return HY_OK;
}

hy_status hy_join_hash(const hy_join_side* build, const hy_join_side* probe, const hy_join_params* params,
                       hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                       uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                       hy_stream_t stream) {
  SidePlan bp, pp;
  hy_status st = prepare(build, probe, params, bp, pp);
  if (st != HY_OK) return st;
  if (!partition_begin || !partition_counts) return fail(HY_ERR_INVALID_ARGUMENT, "partition arrays");
  hipStream_t s = S(stream);
  return dispatch_type(params->hashed_type, [&](auto htag) -> hy_status {
    using H = decltype(htag);
    return dispatch_type(build->value_type, [&](auto btag) -> hy_status {
      using TB = decltype(btag);
      return dispatch_type(probe->value_type, [&](auto ptag) -> hy_status {
        using TP = decltype(ptag);
        // only hashed types reachable through JoinHashTraits are instantiated
        constexpr bool ok_b = sizeof(H) >= sizeof(TB) || std::is_floating_point_v<H>;
        constexpr bool ok_p = sizeof(H) >= sizeof(TP) || std::is_floating_point_v<H>;
        constexpr bool ok_f = !(std::is_floating_point_v<TB> && !std::is_floating_point_v<H>) &&
                              !(std::is_floating_point_v<TP> && !std::is_floating_point_v<H>);
        if constexpr (ok_b && ok_p && ok_f) {
          return join_typed<TB, TP, H>(bp, pp, params, out_build, out_probe, out_capacity, partition_begin,
                                       partition_counts, result, workspace, workspace_bytes, s);
        } else {
          return fail(HY_ERR_UNSUPPORTED, "hashed type not reachable from column types");
        }
      });
    });
  });
}

hy_status hy_join_exchange_partition_workspace_size(const hy_join_side* side, const hy_join_params* params,
                                                    uint32_t n_ranks, size_t* bytes) {
  if (!bytes || !params || n_ranks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  SidePlan p;
  hy_status st = plan_side(side, p);
  if (st != HY_OK) return st;
  const auto w = digit_plan(params->radix_bits, ceil_log2(n_ranks));
  if (w.empty() || (1u << w[0]) < n_ranks) return fail(HY_ERR_UNSUPPORTED, "radix bits too few for the ranks");
  *bytes = type_bytes(params->hashed_type) == 4 ? exchange_partition_bytes<int32_t>(p, params->radix_bits, w)
                                                : exchange_partition_bytes<int64_t>(p, params->radix_bits, w);
  return HY_OK;
}

hy_status hy_join_exchange_partition(const hy_join_side* side, const hy_join_params* params, int32_t keep_nulls,
                                     uint32_t n_ranks, void* out_records, uint64_t* bucket_counts, void* workspace,
                                     size_t workspace_bytes, hy_stream_t stream) {
  if (!params || !bucket_counts || n_ranks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  SidePlan p;
  hy_status st = plan_side(side, p);
  if (st != HY_OK) return st;
  p.fuse = (!p.referenced.empty() && side->fuse_dereference) ? 1 : 0;
  const uint32_t bits = params->radix_bits;
  const auto w = digit_plan(bits, ceil_log2(n_ranks));
  if (w.empty() || (1u << w[0]) < n_ranks) return fail(HY_ERR_UNSUPPORTED, "radix bits too few for the ranks");
  if (p.n_rows && !out_records) return fail(HY_ERR_INVALID_ARGUMENT, "out_records");
  hipStream_t s = S(stream);
  const uint32_t T = 1u << w[0];
  return dispatch_type(params->hashed_type, [&](auto htag) -> hy_status {
    using H = decltype(htag);
    return dispatch_type(side->value_type, [&](auto ttag) -> hy_status {
      using T_ = decltype(ttag);
      constexpr bool ok = (sizeof(H) >= sizeof(T_) || std::is_floating_point_v<H>) &&
                          !(std::is_floating_point_v<T_> && !std::is_floating_point_v<H>);
      if constexpr (ok) {
        if (workspace_bytes < exchange_partition_bytes<H>(p, bits, w)) return fail(HY_ERR_WORKSPACE, "workspace");
        Carver cv{static_cast<char*>(workspace), workspace_bytes};
        SideBufs<H, hy_row_id> b;
        carve_side<H, hy_row_id>(cv, sizes_of(p), bits, std::vector<uint32_t>(w.begin(), w.begin() + 1), 1, false, b);
        Common c{};
        carve_common(cv, std::max<uint64_t>(uint64_t(T) * std::max<uint64_t>(1, p.n_tiles1), 2), bits, &c);
        if (!cv.ok) return fail(HY_ERR_WORKSPACE, "workspace");
        if (upload_side(p, b, s)) return HY_ERR_DEVICE;
        hy_status st2 = pass0_side<T_, H, hy_row_id>("exchange", p, b, bits, w[0], params->seed, keep_nulls != 0,
                                                     p.ref_base, c, s,
                                                     static_cast<hyk::Rec<H, hy_row_id>*>(out_records));
        if (st2 != HY_OK) return st2;
        std::vector<uint32_t> bounds(T + 1);
        HY_HIP(hipMemcpyAsync(bounds.data(), b.segA, 4 * (T + 1), hipMemcpyDeviceToHost, s));
        HY_HIP(hipStreamSynchronize(s));
        for (uint32_t i = 0; i < T; ++i) bucket_counts[i] = bounds[i + 1] - bounds[i];
        return HY_OK;
      } else {
        return fail(HY_ERR_UNSUPPORTED, "hashed type not reachable from the column type");
      }
    });
  });
}

hy_status hy_join_exchange_join_workspace_size(const uint64_t* build_counts, const uint64_t* probe_counts,
                                               uint32_t n_senders, uint32_t n_buckets, const hy_join_params* params,
                                               size_t* bytes) {
  if (!bytes || !params || !build_counts || !probe_counts || n_senders == 0)
    return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  const uint32_t bits = params->radix_bits;
  const auto w = digit_plan(bits, ceil_log2(n_senders));
  if (w.empty()) return fail(HY_ERR_UNSUPPORTED, "radix_bits 0");
  const uint32_t digits = 1u << (w.size() > 1 ? w[1] : 0);
  const RecvPlan rb = recv_plan(build_counts, n_senders, n_buckets, digits);
  const RecvPlan rp = recv_plan(probe_counts, n_senders, n_buckets, digits);
  *bytes = type_bytes(params->hashed_type) == 4 ? exchange_join_bytes<int32_t>(rb, rp, bits, w, n_buckets, n_senders)
                                                : exchange_join_bytes<int64_t>(rb, rp, bits, w, n_buckets, n_senders);
  return HY_OK;
}

hy_status hy_join_exchange_join(const void* build_records, const uint64_t* build_counts, const void* probe_records,
                                const uint64_t* probe_counts, uint32_t n_senders, uint32_t first_bucket,
                                uint32_t n_buckets, const hy_join_params* params, hy_row_id* out_build,
                                hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                                uint32_t* partition_counts, hy_join_result* result, void* workspace,
                                size_t workspace_bytes, hy_stream_t stream) {
  if (!params || !build_counts || !probe_counts || n_senders == 0 || !partition_begin || !partition_counts)
    return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (!(params->mode == HY_JOIN_INNER || params->mode == HY_JOIN_LEFT || params->mode == HY_JOIN_RIGHT ||
        params->mode == HY_JOIN_SEMI || params->mode == HY_JOIN_ANTI))
    return fail(HY_ERR_UNSUPPORTED, "join mode");
  const uint32_t bits = params->radix_bits;
  const auto w = digit_plan(bits, ceil_log2(n_senders));
  if (w.empty() || first_bucket + n_buckets > (1u << w[0])) return fail(HY_ERR_INVALID_ARGUMENT, "bucket range");
  const uint32_t digits = 1u << (w.size() > 1 ? w[1] : 0);
  const RecvPlan rbp = recv_plan(build_counts, n_senders, n_buckets, digits);
  const RecvPlan rpp = recv_plan(probe_counts, n_senders, n_buckets, digits);
  if (rbp.rows >= 0xFFFFFFFFull || rpp.rows >= 0xFFFFFFFFull)
    return fail(HY_ERR_UNSUPPORTED, "received side exceeds 2^32-1 rows");
  hipStream_t s = S(stream);
  return dispatch_type(params->hashed_type, [&](auto htag) -> hy_status {
    using H = decltype(htag);
    if (workspace_bytes < exchange_join_bytes<H>(rbp, rpp, bits, w, n_buckets, n_senders))
      return fail(HY_ERR_WORKSPACE, "exchange join workspace too small");
    Carver cv{static_cast<char*>(workspace), workspace_bytes};
    RecvBufs<H> rb, rp;
    carve_recv<H>(cv, rbp, bits, w, n_buckets, n_senders, rb);
    carve_recv<H>(cv, rpp, bits, w, n_buckets, n_senders, rp);
    Common c{};
    const uint64_t max_scan =
        std::max({rbp.hist_words * 2, rpp.hist_words * 2, (uint64_t(1) << bits) + 1,
                  (rbp.rows + rpp.rows) / span2() * 256 + uint64_t(n_buckets) * n_senders * 256});
    carve_common(cv, max_scan, bits, &c);
    if (!cv.ok) return fail(HY_ERR_WORKSPACE, "exchange join workspace too small");
    using R = hyk::Rec<H, hy_row_id>;
    R* recs[2] = {nullptr, nullptr};
    uint32_t* bounds[2] = {nullptr, nullptr};
    hy_status st = recv_side<H>("build", rbp, rb, w, bits, n_buckets, n_senders, params->seed,
                                static_cast<const R*>(build_records), c, s, &recs[0], &bounds[0]);
    if (st != HY_OK) return st;
    st = recv_side<H>("probe", rpp, rp, w, bits, n_buckets, n_senders, params->seed,
                      static_cast<const R*>(probe_records), c, s, &recs[1], &bounds[1]);
    if (st != HY_OK) return st;
    const uint32_t n_parts = n_buckets << (bits - w[0]);
    return run_join_partitions<H, hy_row_id>(bounds[0], bounds[1], n_parts, recs[0], recs[1], hyk::RowMap{},
                                             hyk::RowMap{}, params->mode, out_build, out_probe, out_capacity,
                                             partition_begin, partition_counts, result, c, s, rbp.rows + rpp.rows);
  });
}

uint32_t hy_join_exchange_bucket_bits(uint32_t radix_bits, uint32_t n_ranks) {
  const auto w = digit_plan(radix_bits, ceil_log2(std::max<uint32_t>(1, n_ranks)));
  return w.empty() ? 0u : w[0];
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
