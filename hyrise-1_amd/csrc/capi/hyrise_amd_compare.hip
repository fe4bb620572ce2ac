// Column-vs-column TableScan (reference ColumnComparisonTableScanImpl::scan_chunk,
// src/lib/operators/table_scan/column_comparison_table_scan_impl.cpp:23-84, and BaseTableScanImpl::_binary_scan,
// base_table_scan_impl.hpp:64-76): row i of chunk c matches iff neither side is NULL and `left OP right` holds under
// C++'s usual arithmetic conversions of the two column types (int vs float compares as float, int vs long as long).
//
// One launch evaluates every row of every chunk (one thread per row, tiles never straddle chunks) and writes a flag
// plus the row's output item (its RowID or its chunk offset) at the row's global index; one order-preserving
// compaction (hipcub DeviceSelect::Flagged) then yields the matches chunk-major, offsets ascending - the PosLists
// the reference's per-chunk jobs build. Per-chunk counts come from one atomic add per tile. Both inputs read 1x;
// this is not a headline kernel, the extra flag/item pass (9-12 B per row) keeps it to two launches.
// String columns (both sides HY_TYPE_STRING; STRING chunks or DICT chunks with packed dictionaries) compare as the
// reference's std::string operators do (kernels/common.hpp string_compare).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "hyrise_amd.h"
#include "capi_common.hpp"
#include "../kernels/common.hpp"

using namespace hyc;

namespace {

constexpr int CMP_THREADS = 256;

struct CmpSide {
  const hy_join_chunk* chunks;        // device copy, one per chunk
  const hy_column_chunk* referenced;  // device copy (reference sides)
  uint32_t n_referenced;
  uint32_t referenced_chunk_base;
};

struct CmpDesc {
  CmpSide left, right;
  const uint32_t* tile_chunk;        // n_tiles
  const uint64_t* chunk_tile_begin;  // n_chunks + 1
  const uint64_t* chunk_row_begin;   // n_chunks + 1
  uint64_t n_tiles;
  int32_t op;
};

// Value of row `off` of a data column chunk; returns true for NULL (value chunk null flag / dictionary null id).
// Strings (T = hyk::DevString): the dictionary / value chunk's packed string array.
template <typename T>
__device__ __forceinline__ bool column_value(const hy_column_chunk& col, uint32_t off, T* v) {
  if (col.kind == HY_COL_DICT) {
    const uint32_t vid = col.vid_width == 1   ? static_cast<const uint8_t*>(col.data)[off]
                         : col.vid_width == 2 ? static_cast<const uint16_t*>(col.data)[off]
                                              : static_cast<const uint32_t*>(col.data)[off];
    if (vid >= col.dictionary_size) return true;
    if constexpr (std::is_same_v<T, hyk::DevString>)
      *v = hyk::packed_string(col.dictionary, col.dictionary_size, vid);
    else
      *v = static_cast<const T*>(col.dictionary)[vid];
    return false;
  }
  if (col.nulls != nullptr && col.nulls[off]) return true;
  if constexpr (std::is_same_v<T, hyk::DevString>)
    *v = hyk::packed_string(col.data, col.size, off);
  else
    *v = static_cast<const T*>(col.data)[off];
  return false;
}

// Row `off` of chunk ch of one side: data chunk, or PosList entry dereferenced (NULL RowID -> NULL).
template <typename T>
__device__ __forceinline__ bool side_value(const CmpSide& s, const hy_join_chunk& ch, uint32_t off, T* v) {
  if (ch.pos_list == nullptr) return column_value<T>(ch.column, off, v);
  const hy_row_id rid = ch.pos_list[off];
  if (rid.chunk_offset == 0xFFFFFFFFu) return true;
  const uint32_t r = rid.chunk_id - s.referenced_chunk_base;
  if (r >= s.n_referenced) return true;
  return column_value<T>(s.referenced[r], rid.chunk_offset, v);
}

template <typename L, typename R, bool ROWS>
__global__ __launch_bounds__(CMP_THREADS) void compare_flags_kernel(CmpDesc d, void* __restrict__ items,
                                                                    uint8_t* __restrict__ flags,
                                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_count;
  const uint64_t tile = blockIdx.x;
  if (tile >= d.n_tiles) return;
  const uint32_t c = d.tile_chunk[tile];
  const hy_join_chunk lc = d.left.chunks[c];
  const hy_join_chunk rc = d.right.chunks[c];
  const uint32_t off = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * CMP_THREADS + threadIdx.x;
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  if (off < lc.size) {
    L lv{};
    R rv{};
    const bool ln = side_value<L>(d.left, lc, off, &lv);
    const bool rn = side_value<R>(d.right, rc, off, &rv);
    bool m = !ln && !rn;
    if constexpr (std::is_same_v<L, hyk::DevString>) {
      m = m && hyk::cmp_result(d.op, hyk::string_compare(lv, rv));  // std::string operators
    } else {
      using C = decltype(L{} + R{});  // the comparator's operand type (usual arithmetic conversions)
      m = m && hyk::cmp_op<C>(d.op, static_cast<C>(lv), static_cast<C>(rv));
    }
    const uint64_t g = d.chunk_row_begin[c] + off;
    flags[g] = m;
    if constexpr (ROWS)
      static_cast<hy_row_id*>(items)[g] = hy_row_id{lc.chunk_id, off};
    else
      static_cast<uint32_t*>(items)[g] = off;
    if (m) atomicAdd(&s_count, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_count) atomicAdd(&counts[c], s_count);
}

int type_size(int32_t t) {
  return t == HY_TYPE_INT32 || t == HY_TYPE_FLOAT ? 4 : (t == HY_TYPE_INT64 || t == HY_TYPE_DOUBLE ? 8 : 0);
}

struct Geometry {
  uint64_t rows = 0, tiles = 0;
};

hy_status check_sides(const hy_join_side* l, const hy_join_side* r, Geometry* g) {
  if (!l || !r) return fail(HY_ERR_INVALID_ARGUMENT, "null side");
  if (l->n_chunks != r->n_chunks) return fail(HY_ERR_INVALID_ARGUMENT, "sides have different chunk counts");
  if ((l->n_chunks && (!l->chunks || !r->chunks))) return fail(HY_ERR_INVALID_ARGUMENT, "null chunks");
  const bool ls = l->value_type == HY_TYPE_STRING, rs = r->value_type == HY_TYPE_STRING;
  if (ls != rs) return fail(HY_ERR_INVALID_ARGUMENT, "string column compared with a numeric column");
  if (!ls && (!type_size(l->value_type) || !type_size(r->value_type)))
    return fail(HY_ERR_UNSUPPORTED, "column comparison value type");
  auto kind_ok = [&](const hy_column_chunk& x) {
    return x.size == 0 || x.kind == HY_COL_DICT || x.kind == (ls ? HY_COL_STRING : HY_COL_VALUE);
  };
  for (uint32_t i = 0; i < l->n_referenced; ++i)
    if (!kind_ok(l->referenced[i])) return fail(HY_ERR_UNSUPPORTED, "column comparison chunk kind");
  for (uint32_t i = 0; i < r->n_referenced; ++i)
    if (!kind_ok(r->referenced[i])) return fail(HY_ERR_UNSUPPORTED, "column comparison chunk kind");
  for (uint32_t c = 0; c < l->n_chunks; ++c) {
    const hy_join_chunk& a = l->chunks[c];
    const hy_join_chunk& b = r->chunks[c];
    if ((!a.pos_list && !kind_ok(a.column)) || (!b.pos_list && !kind_ok(b.column)))
      return fail(HY_ERR_UNSUPPORTED, "column comparison chunk kind");
    if (a.size != b.size) return fail(HY_ERR_INVALID_ARGUMENT, "chunk sizes differ between the columns");
    if ((a.pos_list == nullptr) != (b.pos_list == nullptr))
      return fail(HY_ERR_INVALID_ARGUMENT, "Invalid column combination detected!");  // data vs reference column
    g->rows += a.size;
    g->tiles += (a.size + CMP_THREADS - 1) / CMP_THREADS;
  }
  if (g->rows >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 rows");
  return HY_OK;
}

size_t select_temp_bytes(uint64_t rows, bool out_rows) {
  size_t t = 0;
  if (out_rows)
    (void)hipcub::DeviceSelect::Flagged(nullptr, t, static_cast<const hy_row_id*>(nullptr),
                                        static_cast<const uint8_t*>(nullptr), static_cast<hy_row_id*>(nullptr),
                                        static_cast<uint64_t*>(nullptr), static_cast<int>(rows));
  else
    (void)hipcub::DeviceSelect::Flagged(nullptr, t, static_cast<const uint32_t*>(nullptr),
                                        static_cast<const uint8_t*>(nullptr), static_cast<uint32_t*>(nullptr),
                                        static_cast<uint64_t*>(nullptr), static_cast<int>(rows));
  return t;
}

void carve(Carver& cv, const hy_join_side* l, const hy_join_side* r, const Geometry& g, bool out_rows,
           CmpDesc* d, void** items, uint8_t** flags, char** temp, size_t* temp_bytes, hy_join_chunk** lch,
           hy_join_chunk** rch, hy_column_chunk** lref, hy_column_chunk** rref, uint32_t** tile_chunk,
           uint64_t** tile_begin, uint64_t** row_begin) {
  const uint32_t n = l->n_chunks;
  *lch = cv.take<hy_join_chunk>(std::max<uint32_t>(n, 1));
  *rch = cv.take<hy_join_chunk>(std::max<uint32_t>(n, 1));
  *lref = cv.take<hy_column_chunk>(std::max<uint32_t>(l->n_referenced, 1));
  *rref = cv.take<hy_column_chunk>(std::max<uint32_t>(r->n_referenced, 1));
  *tile_chunk = cv.take<uint32_t>(g.tiles + 1);
  *tile_begin = cv.take<uint64_t>(n + 1);
  *row_begin = cv.take<uint64_t>(n + 1);
  *items = out_rows ? static_cast<void*>(cv.take<hy_row_id>(g.rows + 1)) : static_cast<void*>(cv.take<uint32_t>(g.rows + 1));
  *flags = cv.take<uint8_t>(g.rows + 16);
  *temp_bytes = select_temp_bytes(g.rows, out_rows) + 16;
  *temp = cv.take<char>(*temp_bytes);
  (void)d;
}

}  // namespace

extern "C" {

hy_status hy_column_compare_scan_workspace_size(const hy_join_side* left, const hy_join_side* right, int32_t out_rows,
                                                size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null bytes");
  Geometry g;
  hy_status st = check_sides(left, right, &g);
  if (st != HY_OK) return st;
  Carver cv{nullptr, 0};
  void* items;
  uint8_t* flags;
  char* temp;
  size_t tb;
  hy_join_chunk *lch, *rch;
  hy_column_chunk *lref, *rref;
  uint32_t* tc;
  uint64_t *tbg, *rbg;
  carve(cv, left, right, g, out_rows != 0, nullptr, &items, &flags, &temp, &tb, &lch, &rch, &lref, &rref, &tc, &tbg,
        &rbg);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_column_compare_scan(const hy_join_side* left, const hy_join_side* right, int32_t op,
                                 hy_row_id* out_rows, uint32_t* out_offsets, uint32_t* counts, uint64_t* n_out,
                                 void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  Geometry g;
  hy_status st = check_sides(left, right, &g);
  if (st != HY_OK) return st;
  if (op < HY_OP_EQ || op > HY_OP_GE) return fail(HY_ERR_INVALID_ARGUMENT, "column comparison op");
  if ((out_rows == nullptr) == (out_offsets == nullptr))
    return fail(HY_ERR_INVALID_ARGUMENT, "exactly one of out_rows / out_offsets");
  if (!n_out || (left->n_chunks && !counts)) return fail(HY_ERR_INVALID_ARGUMENT, "null counts");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(n_out, 0, 8, s));
  const uint32_t n = left->n_chunks;
  if (n) HY_HIP(hipMemsetAsync(counts, 0, 4ull * n, s));
  if (g.rows == 0) return HY_OK;
  const bool rows = out_rows != nullptr;

  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  CmpDesc d{};
  void* items;
  uint8_t* flags;
  char* temp;
  size_t tb;
  hy_join_chunk *lch, *rch;
  hy_column_chunk *lref, *rref;
  uint32_t* tc;
  uint64_t *tbg, *rbg;
  carve(cv, left, right, g, rows, &d, &items, &flags, &temp, &tb, &lch, &rch, &lref, &rref, &tc, &tbg, &rbg);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "column comparison workspace too small");

  std::vector<uint32_t> h_tc(g.tiles);
  std::vector<uint64_t> h_tbg(n + 1), h_rbg(n + 1);
  uint64_t t = 0, r = 0;
  for (uint32_t c = 0; c < n; ++c) {
    h_tbg[c] = t;
    h_rbg[c] = r;
    const uint64_t k = (left->chunks[c].size + CMP_THREADS - 1) / CMP_THREADS;
    for (uint64_t i = 0; i < k; ++i) h_tc[t + i] = c;
    t += k;
    r += left->chunks[c].size;
  }
  h_tbg[n] = t;
  h_rbg[n] = r;
  HY_STAGE(lch, left->chunks, sizeof(hy_join_chunk) * n, s);
  HY_STAGE(rch, right->chunks, sizeof(hy_join_chunk) * n, s);
  if (left->n_referenced) HY_STAGE(lref, left->referenced, sizeof(hy_column_chunk) * left->n_referenced, s);
  if (right->n_referenced) HY_STAGE(rref, right->referenced, sizeof(hy_column_chunk) * right->n_referenced, s);
  HY_STAGE(tc, h_tc.data(), 4 * g.tiles, s);
  HY_STAGE(tbg, h_tbg.data(), 8 * (n + 1), s);
  HY_STAGE(rbg, h_rbg.data(), 8 * (n + 1), s);
  d.left = CmpSide{lch, lref, left->n_referenced, left->referenced_chunk_base};
  d.right = CmpSide{rch, rref, right->n_referenced, right->referenced_chunk_base};
  d.tile_chunk = tc;
  d.chunk_tile_begin = tbg;
  d.chunk_row_begin = rbg;
  d.n_tiles = g.tiles;
  d.op = op;

  auto launch = [&](auto ltag, auto rtag) -> hy_status {
    using L = decltype(ltag);
    using R = decltype(rtag);
    if (rows)
      hipLaunchKernelGGL((compare_flags_kernel<L, R, true>), dim3(static_cast<uint32_t>(g.tiles)), dim3(CMP_THREADS), 0,
                         s, d, items, flags, counts);
    else
      hipLaunchKernelGGL((compare_flags_kernel<L, R, false>), dim3(static_cast<uint32_t>(g.tiles)),
                         dim3(CMP_THREADS), 0, s, d, items, flags, counts);
    HY_HIP(hipGetLastError());
    return HY_OK;
  };
  auto with_right = [&](auto ltag) -> hy_status {
    switch (right->value_type) {
      case HY_TYPE_INT32:
        return launch(ltag, int32_t{});
      case HY_TYPE_INT64:
        return launch(ltag, int64_t{});
      case HY_TYPE_FLOAT:
        return launch(ltag, float{});
      default:
        return launch(ltag, double{});
    }
  };
  switch (left->value_type) {
    case HY_TYPE_STRING:
      st = launch(hyk::DevString{}, hyk::DevString{});
      break;
    case HY_TYPE_INT32:
      st = with_right(int32_t{});
      break;
    case HY_TYPE_INT64:
      st = with_right(int64_t{});
      break;
    case HY_TYPE_FLOAT:
      st = with_right(float{});
      break;
    default:
      st = with_right(double{});
      break;
  }
  if (st != HY_OK) return st;
  if (rows)
    HY_HIP(hipcub::DeviceSelect::Flagged(temp, tb, static_cast<const hy_row_id*>(items), flags, out_rows, n_out,
                                         static_cast<int>(g.rows), s));
  else
    HY_HIP(hipcub::DeviceSelect::Flagged(temp, tb, static_cast<const uint32_t*>(items), flags, out_offsets, n_out,
                                         static_cast<int>(g.rows), s));
  // the staged descriptors live in the pinned ring; the workspace is the caller's: nothing to wait for here
  return HY_OK;
}

}  // extern "C"
