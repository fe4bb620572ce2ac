// MVCC visibility filter (reference Validate::_on_execute, src/lib/operators/validate.cpp:14-95): a row is visible to
// transaction `our_tid` with snapshot commit id `snapshot` iff
//     snapshot < end_cid && ((snapshot >= begin_cid) != (row_tid == our_tid))        (validate.cpp:14-26)
// i.e. an own uncommitted insert or a past committed insert that is not deleted as of the snapshot.
//
// Data-table input: one thread per row of every chunk (tiles never straddle chunks) writes a flag and the row's RowID
// at its global index; one order-preserving DeviceSelect::Flagged yields the visible rows chunk-major. Reference input:
// the PosList's RowIDs are flagged through the referenced chunks' MVCC vectors and compacted the same way. The MVCC
// vectors are 12 B per row read once; the flag/item pass adds 9 B per row.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "hyrise_amd.h"
#include "capi_common.hpp"

using namespace hyc;

namespace {

constexpr int VAL_THREADS = 256;

__device__ __forceinline__ bool row_visible(const hy_mvcc_chunk& m, uint32_t off, uint32_t our_tid,
                                            uint32_t snapshot) {
  const uint32_t tid = m.tids[off];
  const uint32_t begin = m.begin_cids[off];
  const uint32_t end = m.end_cids[off];
  return snapshot < end && ((snapshot >= begin) != (tid == our_tid));
}

__global__ __launch_bounds__(VAL_THREADS) void validate_rows_kernel(
    const hy_mvcc_chunk* __restrict__ chunks, const uint32_t* __restrict__ chunk_ids,
    const uint32_t* __restrict__ tile_chunk, const uint64_t* __restrict__ chunk_tile_begin,
    const uint64_t* __restrict__ chunk_row_begin, uint64_t n_tiles, uint32_t our_tid, uint32_t snapshot,
    hy_row_id* __restrict__ items, uint8_t* __restrict__ flags, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_count;
  const uint64_t tile = blockIdx.x;
  if (tile >= n_tiles) return;
  const uint32_t c = tile_chunk[tile];
  const hy_mvcc_chunk m = chunks[c];
  const uint32_t off = static_cast<uint32_t>(tile - chunk_tile_begin[c]) * VAL_THREADS + threadIdx.x;
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  if (off < m.size) {
    const bool v = row_visible(m, off, our_tid, snapshot);
    const uint64_t g = chunk_row_begin[c] + off;
    flags[g] = v;
    items[g] = hy_row_id{chunk_ids[c], off};
    if (v) atomicAdd(&s_count, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_count) atomicAdd(&counts[c], s_count);
}

__global__ __launch_bounds__(VAL_THREADS) void validate_pos_list_kernel(const hy_row_id* __restrict__ pos_list,
                                                                        uint64_t n,
                                                                        const hy_mvcc_chunk* __restrict__ chunks,
                                                                        uint32_t n_chunks, uint32_t our_tid,
                                                                        uint32_t snapshot,
                                                                        uint8_t* __restrict__ flags) {
  const uint64_t i = blockIdx.x * static_cast<uint64_t>(VAL_THREADS) + threadIdx.x;
  if (i >= n) return;
  const hy_row_id r = pos_list[i];
  bool v = false;
  if (r.chunk_offset != 0xFFFFFFFFu && r.chunk_id < n_chunks) {
    const hy_mvcc_chunk& m = chunks[r.chunk_id];
    v = r.chunk_offset < m.size && row_visible(m, r.chunk_offset, our_tid, snapshot);
  }
  flags[i] = v;
}

size_t select_bytes(uint64_t n) {
  size_t t = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, t, static_cast<const hy_row_id*>(nullptr),
                                      static_cast<const uint8_t*>(nullptr), static_cast<hy_row_id*>(nullptr),
                                      static_cast<uint64_t*>(nullptr), static_cast<int>(n));
  return t + 16;
}

struct ValWs {
  hy_mvcc_chunk* chunks;
  uint32_t* chunk_ids;
  uint32_t* tile_chunk;
  uint64_t* tile_begin;
  uint64_t* row_begin;
  hy_row_id* items;
  uint8_t* flags;
  char* temp;
  size_t temp_bytes;
};

// n_rows: rows of all chunks (data input) or the PosList length; n_chunks: chunks / referenced chunks
void carve(Carver& cv, uint64_t n_rows, uint32_t n_chunks, ValWs* w) {
  const uint64_t tiles = n_rows / VAL_THREADS + n_chunks + 1;
  w->chunks = cv.take<hy_mvcc_chunk>(std::max<uint32_t>(n_chunks, 1));
  w->chunk_ids = cv.take<uint32_t>(std::max<uint32_t>(n_chunks, 1));
  w->tile_chunk = cv.take<uint32_t>(tiles);
  w->tile_begin = cv.take<uint64_t>(n_chunks + 1);
  w->row_begin = cv.take<uint64_t>(n_chunks + 1);
  w->items = cv.take<hy_row_id>(n_rows + 1);
  w->flags = cv.take<uint8_t>(n_rows + 16);
  w->temp_bytes = select_bytes(n_rows);
  w->temp = cv.take<char>(w->temp_bytes);
}

hy_status check_chunks(const hy_mvcc_chunk* chunks, uint32_t n) {
  if (n && !chunks) return fail(HY_ERR_INVALID_ARGUMENT, "null mvcc chunks");
  for (uint32_t c = 0; c < n; ++c)
    if (chunks[c].size && (!chunks[c].tids || !chunks[c].begin_cids || !chunks[c].end_cids))
      return fail(HY_ERR_INVALID_ARGUMENT, "Trying to use Validate on a table that has no MVCC columns");
  return HY_OK;
}

}  // namespace

extern "C" {

hy_status hy_validate_workspace_size(uint64_t n_rows, uint32_t n_chunks, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null bytes");
  if (n_rows >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 rows");
  Carver cv{nullptr, 0};
  ValWs w;
  carve(cv, n_rows, n_chunks, &w);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_validate(const hy_mvcc_chunk* chunks, uint32_t n_chunks, const uint32_t* chunk_ids, uint32_t our_tid,
                      uint32_t snapshot_commit_id, hy_row_id* out_rows, uint32_t* counts, uint64_t* n_out,
                      void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  hy_status st = check_chunks(chunks, n_chunks);
  if (st != HY_OK) return st;
  if (!n_out || (n_chunks && (!counts || !chunk_ids || !out_rows))) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(n_out, 0, 8, s));
  if (n_chunks) HY_HIP(hipMemsetAsync(counts, 0, 4ull * n_chunks, s));
  uint64_t rows = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) rows += chunks[c].size;
  if (rows == 0) return HY_OK;
  if (rows >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 rows");
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  ValWs w;
  carve(cv, rows, n_chunks, &w);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "validate workspace too small");
  std::vector<uint32_t> h_tc;
  std::vector<uint64_t> h_tb(n_chunks + 1), h_rb(n_chunks + 1);
  uint64_t r = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    h_tb[c] = h_tc.size();
    h_rb[c] = r;
    const uint64_t k = (chunks[c].size + VAL_THREADS - 1) / VAL_THREADS;
    h_tc.insert(h_tc.end(), k, c);
    r += chunks[c].size;
  }
  h_tb[n_chunks] = h_tc.size();
  h_rb[n_chunks] = r;
  const uint64_t tiles = h_tc.size();
  HY_STAGE(w.chunks, chunks, sizeof(hy_mvcc_chunk) * n_chunks, s);
  HY_STAGE(w.chunk_ids, chunk_ids, 4ull * n_chunks, s);
  HY_STAGE(w.tile_chunk, h_tc.data(), 4 * tiles, s);
  HY_STAGE(w.tile_begin, h_tb.data(), 8ull * (n_chunks + 1), s);
  HY_STAGE(w.row_begin, h_rb.data(), 8ull * (n_chunks + 1), s);
  hipLaunchKernelGGL(validate_rows_kernel, dim3(static_cast<uint32_t>(tiles)), dim3(VAL_THREADS), 0, s, w.chunks,
                     w.chunk_ids, w.tile_chunk, w.tile_begin, w.row_begin, tiles, our_tid, snapshot_commit_id, w.items,
                     w.flags, counts);
  HY_HIP(hipGetLastError());
  HY_HIP(hipcub::DeviceSelect::Flagged(w.temp, w.temp_bytes, w.items, w.flags, out_rows, n_out, static_cast<int>(rows),
                                       s));
  return HY_OK;
}

hy_status hy_validate_pos_list(const hy_row_id* pos_list, uint64_t pos_list_size,
                               const hy_mvcc_chunk* referenced_chunks, uint32_t n_referenced, uint32_t our_tid,
                               uint32_t snapshot_commit_id, hy_row_id* out_rows, uint64_t* n_out, void* workspace,
                               size_t workspace_bytes, hy_stream_t stream) {
  hy_status st = check_chunks(referenced_chunks, n_referenced);
  if (st != HY_OK) return st;
  if (!n_out) return fail(HY_ERR_INVALID_ARGUMENT, "null n_out");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(n_out, 0, 8, s));
  if (pos_list_size == 0) return HY_OK;
  if (!pos_list || !out_rows) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (pos_list_size >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 rows");
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  ValWs w;
  carve(cv, pos_list_size, n_referenced, &w);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "validate workspace too small");
  if (n_referenced) HY_STAGE(w.chunks, referenced_chunks, sizeof(hy_mvcc_chunk) * n_referenced, s);
  const uint32_t blocks = static_cast<uint32_t>((pos_list_size + VAL_THREADS - 1) / VAL_THREADS);
  hipLaunchKernelGGL(validate_pos_list_kernel, dim3(blocks), dim3(VAL_THREADS), 0, s, pos_list, pos_list_size, w.chunks,
                     n_referenced, our_tid, snapshot_commit_id, w.flags);
  HY_HIP(hipGetLastError());
  HY_HIP(hipcub::DeviceSelect::Flagged(w.temp, w.temp_bytes, pos_list, w.flags, out_rows, n_out,
                                       static_cast<int>(pos_list_size), s));
  return HY_OK;
}

}  // extern "C"
