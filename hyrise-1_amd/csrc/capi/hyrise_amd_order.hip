// Reference-input TableScan over a PosList that references several chunks: the reference splits the PosList by
// referenced chunk (split_pos_list_by_chunk_id, chunk_offset_mapping.cpp:5-21) into a std::unordered_map and scans the
// groups in that map's iteration order, each group's positions ascending (base_single_column_table_scan_impl.cpp:36-60).
// The device scans ALL positions in one launch (hy_reference_scan: ascending positions of the matches); this
// translation unit reorders those matches into the reference's group order with one stable radix sort of 64-bit keys
// (group rank << 32 | position) - rocPRIM's onesweep sort behind hipcub, its own TU because of its compile time.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <string>

#include "hyrise_amd.h"
#include "capi_common.hpp"

using namespace hyc;

namespace {

__global__ void order_keys_kernel(const hy_row_id* __restrict__ pos_list, const uint32_t* __restrict__ positions,
                                  uint64_t n, const uint32_t* __restrict__ chunk_rank, uint32_t n_chunks,
                                  uint64_t* __restrict__ keys) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t p = positions[i];
    const uint32_t c = pos_list[p].chunk_id;
    const uint64_t rank = c < n_chunks ? chunk_rank[c] : 0xFFFFFFFFull;
    keys[i] = (rank << 32) | p;
  }
}

__global__ void order_positions_kernel(const uint64_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = static_cast<uint32_t>(keys[i]);
}

uint32_t rank_bits(uint32_t n_ranks) {
  uint32_t b = 1;
  while (b < 32 && (uint64_t(1) << b) <= n_ranks) ++b;
  return b;
}

size_t sort_temp_bytes(uint64_t n, uint32_t n_ranks) {
  size_t t = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, t, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                                    static_cast<int>(n), 32, 32 + static_cast<int>(rank_bits(n_ranks)));
  return t;
}

}  // namespace

extern "C" {

hy_status hy_reference_scan_order_workspace_size(uint64_t n, uint32_t n_ranks, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (n >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 matches");
  Carver cv{nullptr, 0};
  cv.take<uint64_t>(n + 1);
  cv.take<uint64_t>(n + 1);
  cv.take<char>(sort_temp_bytes(n, n_ranks) + 16);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_reference_scan_order(const hy_row_id* pos_list, const uint32_t* positions, uint64_t n,
                                  const uint32_t* chunk_rank, uint32_t n_chunks, uint32_t n_ranks,
                                  uint32_t* out_positions, void* workspace, size_t workspace_bytes,
                                  hy_stream_t stream) {
  if (n == 0) return HY_OK;
  if (!pos_list || !positions || !chunk_rank || !out_positions) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  size_t need = 0;
  hy_status st = hy_reference_scan_order_workspace_size(n, n_ranks, &need);
  if (st != HY_OK) return st;
  if (workspace_bytes < need) return fail(HY_ERR_WORKSPACE, "reference scan order workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  uint64_t* keys_in = cv.take<uint64_t>(n + 1);
  uint64_t* keys_out = cv.take<uint64_t>(n + 1);
  size_t temp = sort_temp_bytes(n, n_ranks);
  char* tmp = cv.take<char>(temp + 16);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "reference scan order workspace too small");
  hipLaunchKernelGGL(order_keys_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, pos_list, positions, n, chunk_rank,
                     n_chunks, keys_in);
  HY_HIP(hipGetLastError());
  HY_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, temp, keys_in, keys_out, static_cast<int>(n), 32,
                                           32 + static_cast<int>(rank_bits(n_ranks)), s));
  hipLaunchKernelGGL(order_positions_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, keys_out, n, out_positions);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

}  // extern "C"
