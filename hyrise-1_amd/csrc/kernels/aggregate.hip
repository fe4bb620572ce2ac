// Aggregate kernels for gfx950: GROUP BY + MIN / MAX / SUM / AVG / COUNT / COUNT(*) / COUNT(DISTINCT).
//
// The reference (src/lib/operators/aggregate.cpp) first maps every group-by value to a first-seen id per column
// (:291-394), then, chunk by chunk and aggregate by aggregate, upserts results[key] in a std::unordered_map and folds
// the row's value in (_aggregate_column, :133-249, traits aggregate_traits.hpp:15-74). Its output order is the
// unordered_map's, its group values are read back at each group's LAST row (:543-566, _write_groupby_output).
//
// Here one pass over the input rows produces, per group, a record of 64-bit words:
//   [0, n_gb)     key words: the group-by values' bits (0 when NULL), floats with -0.0 folded into +0.0
//   n_gb          NULL mask of the key columns
//   n_gb + 1      first row (smallest input row index of the group)  -> reproduces the reference's insertion order
//   n_gb + 2      last row  (largest input row index)                -> the row the reference reads group values at
//   n_gb + 3      rows (COUNT(*))
//   then per aggregate, at its first word w:
//     COUNT(col) / COUNT(DISTINCT col):  w = count
//     SUM/AVG of int32/int64:            w = non-NULL count, w+1 = int64 sum (two's complement wrap, like the
//                                        reference's int64 accumulator)
//     SUM/AVG of float/double:           w = non-NULL count, w+1 = non-finite flags (1 +inf, 2 -inf, 4 NaN),
//                                        w+2.. = exact fixed-point sum: limb i holds a signed sum of 32-bit pieces of
//                                        weight 2^(32 i + emin) (float: 9 limbs, emin -149; double: 66, emin -1074).
//                                        Integer atomics make it exact and order-independent; the host rounds it
//                                        once to double (hy_agg_float_sum).
//     MIN / MAX:                         w = non-NULL count, w+1 = order-preserving bits of the extreme value
// Group records are combined with per-word operations (ADD / MIN / MAX / OR), so any split of the rows over
// workgroups gives the same result.
//
// Two kernels:
//   agg_dense_rows  every group-by column arrives as small integer codes (host-built code dictionaries), so the
//                   group is a mixed-radix index < 64. Each wave folds 64 rows per step with ballots (counts, first /
//                   last row) and 64-bit butterfly reductions (sums, min/max), one lane updates the workgroup's LDS
//                   records; a workgroup flushes its records to HBM with a handful of atomics at the end. This is the
//                   TPC-H Q1 shape (4 groups over 6e8 rows): HBM-bound on the column reads.
//   agg_hash_runs   general keys: a global open-addressing table of group records in HBM (linear probing, claim by
//                   CAS, record initialised before the slot is published), accumulators updated with global atomics,
//                   once per run of equal keys inside a wave. COUNT(DISTINCT) inserts (group slot, aggregate, value)
//                   into a second global set.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int AGG_MAX_COLUMNS = 16;
constexpr int AGG_MAX_GROUPBY = 8;
constexpr int AGG_MAX_AGGREGATES = 16;
constexpr int AGG_MAX_POS_GROUPS = 8;
constexpr int AGG_DENSE_MAX = 64;
constexpr int AGG_THREADS = 256;
constexpr int AGG_ITEMS = 16;                           // rows per lane per tile
constexpr int AGG_TILE = AGG_THREADS * AGG_ITEMS;       // 4096 rows
constexpr int AGG_WAVE_SPAN = WAVE * AGG_ITEMS;         // 1024 consecutive rows per wave
constexpr int AGG_DENSE_LDS_WORDS = 6144;               // 48 KiB of group records per workgroup

enum : int32_t { WOP_KEY = 0, WOP_ADD = 1, WOP_MIN = 2, WOP_MAX = 3, WOP_OR = 4 };
enum : int32_t { AGG_HDR_NULLS = 0, AGG_HDR_FIRST = 1, AGG_HDR_LAST = 2, AGG_HDR_ROWS = 3, AGG_HDR_WORDS = 4 };

constexpr int FLOAT_LIMBS = 9;
constexpr int FLOAT_EMIN = -149;
constexpr int DOUBLE_LIMBS = 66;
constexpr int DOUBLE_EMIN = -1074;

struct AggCol {
  const hy_column_chunk* chunks;  // device array: per input chunk (data input) or per referenced chunk
  int32_t type;                   // HY_TYPE_*
  int32_t pos_group;              // -1: read at (input chunk, offset); else through pos_lists[pos_group]
  uint32_t domain;                // dense grouping: codes in [0, domain), NULL -> domain
  uint32_t stride;                // dense grouping: weight of this column's code in the group index
  int32_t ukind;                  // HY_COL_* shared by every chunk of the column, -1 if mixed (host-computed)
  int32_t uwidth;                 // dictionary chunks: the vid width they all share (0 if mixed)
  int32_t unulls;                 // value chunks: some chunk has NULL flags
};

struct AggFn {
  int32_t function;  // HY_AGG_*
  int32_t column;    // index into cols, -1 for COUNT(*)
  uint32_t word;     // first word of this aggregate in a group record
  int32_t limbs;     // float/double SUM/AVG: limbs of the fixed-point accumulator, else 0
};

struct AggDesc {
  AggCol cols[AGG_MAX_COLUMNS];
  AggFn fns[AGG_MAX_AGGREGATES];
  int32_t gb[AGG_MAX_GROUPBY];       // group-by entries (indexes into cols)
  uint32_t n_cols, n_fns, n_gb, n_pos_groups;
  const hy_row_id* const* pos_lists; // device: pos_lists[g * n_chunks + c]
  const uint32_t* chunk_size;        // device: rows per input chunk
  const uint64_t* chunk_row_begin;   // device: n_chunks + 1
  const uint64_t* chunk_tile_begin;  // device: n_chunks + 1
  const uint32_t* tile_chunk;        // device: chunk of each tile
  uint32_t n_chunks;
  uint64_t n_tiles;
  uint32_t words;                    // words per group record
  const int32_t* word_op;            // device: WOP_* per record word
  uint32_t* error;                   // bit 0: table full / livelock guard, bit 1: dense code out of range
  // fused TableScan (hy_agg_input.filter, data input only): a row takes part only if the predicate column's chunk c
  // (filter[c]: op + search_vid of the host's dictionary rewrite, or a value compare with filter_cbits) matches
  const hy_scan_chunk* filter;
  uint64_t filter_cbits;
  int32_t filter_type;
};

// Item k < R of a lane in one aggregation step is row first + k * STRIDE of its chunk: STRIDE = WAVE for the FQ-style
// mapping (first = base + lane), STRIDE = 1 for a lane's R consecutive rows (first = base + lane * R; agg_dense_lanes
// over a data input reads them with one vector load per column).
typedef uint32_t hy_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t hy_u32x4 __attribute__((ext_vector_type(4)));
template <int R>
__device__ __forceinline__ void vec_load_ids(const void* data, uint32_t width, uint32_t first, uint32_t (&v)[R]) {
  static_assert(R == 4, "one dword / dwordx2 / dwordx4 per lane");
  const uintptr_t p = reinterpret_cast<uintptr_t>(data);
  if (width == 1) {
    const uint32_t w = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(p + first);
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = (w >> (8 * k)) & 0xFFu;
  } else if (width == 2) {
    const hy_u32x2 w = *reinterpret_cast<const __attribute__((address_space(1))) hy_u32x2*>(p + 2ull * first);
    v[0] = w.x & 0xFFFFu;
    v[1] = w.x >> 16;
    v[2] = w.y & 0xFFFFu;
    v[3] = w.y >> 16;
  } else {
    const hy_u32x4 w = *reinterpret_cast<const __attribute__((address_space(1))) hy_u32x4*>(p + 4ull * first);
    v[0] = w.x;
    v[1] = w.y;
    v[2] = w.z;
    v[3] = w.w;
  }
}
// The same rows one element at a time (a chunk's last, partial step), indexes clamped to the chunk.
template <int R>
__device__ __forceinline__ void elem_load_ids(const void* data, uint32_t width, uint32_t first, uint32_t size,
                                              uint32_t (&v)[R]) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(data);
  if (width == 1) {
#pragma unroll
    for (int k = 0; k < R; ++k)
      v[k] = *reinterpret_cast<const __attribute__((address_space(1))) uint8_t*>(p + min(first + k, size - 1));
  } else if (width == 2) {
#pragma unroll
    for (int k = 0; k < R; ++k)
      v[k] = *reinterpret_cast<const __attribute__((address_space(1))) uint16_t*>(p + 2ull * min(first + k, size - 1));
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k)
      v[k] = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(p + 4ull * min(first + k, size - 1));
  }
}

// A dictionary predicate (op, search_vid) of the host's rewrite as an id range: a non-NULL id matches iff
// ((id - lo) < span) != neg - EQ [s, s+1), LT [0, s), LE [0, s+1), NE / GE / GT their complements, ALL / IS NOT NULL
// everything, NONE nothing. One subtract, compare and xor per row instead of a switch on the op.
struct IdRange {
  uint32_t lo, span, neg, dsize;
  bool range;  // false: an op without a range form (VID_SET, ...)
};
__device__ __forceinline__ IdRange id_range(int32_t op, uint32_t svid, uint32_t dsize) {
  IdRange r{0u, 0u, 0u, dsize, true};
  switch (op) {
    case HY_OP_EQ: r.lo = svid; r.span = 1; break;
    case HY_OP_NE: r.lo = svid; r.span = 1; r.neg = 1; break;
    case HY_OP_LT: r.span = svid; break;
    case HY_OP_LE: r.span = svid + 1; break;
    case HY_OP_GT: r.span = svid + 1; r.neg = 1; break;
    case HY_OP_GE: r.span = svid; r.neg = 1; break;
    case HY_OP_ALL:
    case HY_OP_IS_NOT_NULL: r.neg = 1; break;
    case HY_OP_NONE: break;
    default: r.range = false; break;
  }
  return r;
}
__device__ __forceinline__ bool id_in_range(const IdRange& r, uint32_t id) {
  return ((id - r.lo < r.span) != (r.neg != 0)) && id < r.dsize;
}

// Match mask of a lane's items (see above) of input chunk c under the fused scan predicate (reference
// SingleColumnTableScanImpl, single_column_table_scan_impl.cpp:38-205); rows past the chunk are 0. With STRIDE 1 a
// dictionary predicate over the lane's whole run reads its ids with one vector load (the host checked alignment).
template <int R, int STRIDE = WAVE>
__device__ __forceinline__ uint32_t agg_filter_mask(const AggDesc& d, uint32_t c, uint32_t first) {
  const hy_scan_chunk f = d.filter[c];
  const uint32_t n = f.column.size;
  if (f.op == HY_OP_NONE || n == 0) return 0u;
  uint32_t m = 0;
  if (f.column.kind == HY_COL_DICT) {
    const uint32_t w = static_cast<uint32_t>(f.column.vid_width);
    uint32_t vids[R];
    bool loaded = false;
    if constexpr (STRIDE == 1 && R == 4) {
      if (first + R <= n) {
        vec_load_ids<R>(f.column.data, w, first, vids);
        loaded = true;
      }
    }
    if (!loaded) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t i = min(first + k * STRIDE, n - 1);
        vids[k] = w == 1 ? static_cast<const uint8_t*>(f.column.data)[i]
                  : w == 2 ? static_cast<const uint16_t*>(f.column.data)[i]
                           : static_cast<const uint32_t*>(f.column.data)[i];
      }
    }
    const IdRange ir = id_range(f.op, f.search_vid, f.column.dictionary_size);
    if (ir.range) {
#pragma unroll
      for (int k = 0; k < R; ++k) m |= static_cast<uint32_t>(id_in_range(ir, vids[k])) << k;
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k)
        m |= static_cast<uint32_t>(vids[k] != f.column.dictionary_size && cmp_op<uint32_t>(f.op, vids[k], f.search_vid))
             << k;
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const uint32_t i = min(first + k * STRIDE, n - 1);
      const bool nul = f.column.nulls != nullptr && f.column.nulls[i];
      bool hit = false;
      switch (d.filter_type) {
        case HY_TYPE_INT32: {
          int32_t c0;
          __builtin_memcpy(&c0, &d.filter_cbits, 4);
          hit = cmp_op<int32_t>(f.op, static_cast<const int32_t*>(f.column.data)[i], c0);
          break;
        }
        case HY_TYPE_INT64: {
          int64_t c0;
          __builtin_memcpy(&c0, &d.filter_cbits, 8);
          hit = cmp_op<int64_t>(f.op, static_cast<const int64_t*>(f.column.data)[i], c0);
          break;
        }
        case HY_TYPE_FLOAT: {
          float c0;
          __builtin_memcpy(&c0, &d.filter_cbits, 4);
          hit = cmp_op<float>(f.op, static_cast<const float*>(f.column.data)[i], c0);
          break;
        }
        default: {
          double c0;
          __builtin_memcpy(&c0, &d.filter_cbits, 8);
          hit = cmp_op<double>(f.op, static_cast<const double*>(f.column.data)[i], c0);
        }
      }
      m |= static_cast<uint32_t>(hit && !nul) << k;
    }
  }
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (first + k * STRIDE >= n) m &= ~(1u << k);
  return m;
}

__host__ __device__ inline uint64_t word_init(int32_t op) { return op == WOP_MIN ? ~0ull : 0ull; }

// ------------------------------------------------------------------------------------------------------------
// Column reads
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool is_wide(int32_t type) { return type == HY_TYPE_INT64 || type == HY_TYPE_DOUBLE; }

// Raw bits of row `off` of a column chunk (zero-extended for 4-byte types); false for NULL. Dictionary NULL is
// value id == dictionary size (dictionary_encoder.hpp:87); a ValueColumn NULL is its null flag.
__device__ __forceinline__ bool load_bits(const hy_column_chunk& c, uint32_t off, bool wide, uint64_t* bits) {
  if (c.kind == HY_COL_DICT) {
    uint32_t vid;
    if (c.vid_width == 1)
      vid = static_cast<const uint8_t*>(c.data)[off];
    else if (c.vid_width == 2)
      vid = static_cast<const uint16_t*>(c.data)[off];
    else
      vid = static_cast<const uint32_t*>(c.data)[off];
    if (vid >= c.dictionary_size) {
      *bits = 0;
      return false;
    }
    *bits = wide ? static_cast<const uint64_t*>(c.dictionary)[vid] : static_cast<const uint32_t*>(c.dictionary)[vid];
    return true;
  }
  if (c.nulls != nullptr && c.nulls[off]) {
    *bits = 0;
    return false;
  }
  *bits = wide ? static_cast<const uint64_t*>(c.data)[off] : static_cast<const uint32_t*>(c.data)[off];
  return true;
}

// RowIDs of one input row in every PosList group (reference input); NULL RowIDs read as NULL values
// (reference_column_iterable.hpp:60-86).
struct RowRefs {
  hy_row_id rid[AGG_MAX_POS_GROUPS];
};

__device__ __forceinline__ void load_refs(const AggDesc& d, uint32_t c, uint32_t off, RowRefs* r) {
  for (uint32_t g = 0; g < d.n_pos_groups; ++g) r->rid[g] = d.pos_lists[static_cast<uint64_t>(g) * d.n_chunks + c][off];
}

__device__ __forceinline__ bool read_col(const AggDesc& d, const AggCol& col, uint32_t c, uint32_t off,
                                         const RowRefs& refs, uint64_t* bits) {
  const bool wide = is_wide(col.type);
  if (col.pos_group < 0) return load_bits(col.chunks[c], off, wide, bits);
  const hy_row_id rid = refs.rid[col.pos_group];
  if (rid.chunk_offset == 0xFFFFFFFFu) {
    *bits = 0;
    return false;
  }
  return load_bits(col.chunks[rid.chunk_id], rid.chunk_offset, wide, bits);
}

// Key word of a group-by value: raw bits, with -0.0 folded into +0.0 (they are one key of std::unordered_map<float>).
__device__ __forceinline__ uint64_t key_bits(uint64_t bits, int32_t type) {
  if (type == HY_TYPE_FLOAT && bits == 0x80000000ull) return 0;
  if (type == HY_TYPE_DOUBLE && bits == 0x8000000000000000ull) return 0;
  return bits;
}

// Order-preserving unsigned image of a value (MIN / MAX with unsigned 64-bit atomics).
__device__ __forceinline__ uint64_t ordered_bits(uint64_t bits, int32_t type) {
  switch (type) {
    case HY_TYPE_INT32:
      return static_cast<uint32_t>(bits) ^ 0x80000000u;
    case HY_TYPE_INT64:
      return bits ^ (1ull << 63);
    case HY_TYPE_FLOAT: {
      const uint32_t b = static_cast<uint32_t>(bits);
      return (b & 0x80000000u) ? static_cast<uint32_t>(~b) : (b | 0x80000000u);
    }
    default:
      return (bits >> 63) ? ~bits : (bits | (1ull << 63));
  }
}

__device__ __forceinline__ int64_t int_value(uint64_t bits, int32_t type) {
  return type == HY_TYPE_INT32 ? static_cast<int64_t>(static_cast<int32_t>(static_cast<uint32_t>(bits)))
                               : static_cast<int64_t>(bits);
}

// Exact fixed-point pieces of a float / double: value = sum_k part[k] * 2^(32 (i0 + k) + emin). Returns the number of
// pieces (0 for zero / non-finite; *special receives the non-finite flag).
__device__ __forceinline__ int float_parts(uint64_t bits, int32_t type, int* i0, int64_t part[3], uint32_t* special) {
  *special = 0;
  bool neg;
  uint32_t shift;
  unsigned __int128 c;
  if (type == HY_TYPE_FLOAT) {
    const uint32_t b = static_cast<uint32_t>(bits);
    const uint32_t e = (b >> 23) & 0xFFu;
    uint32_t m = b & 0x7FFFFFu;
    neg = (b >> 31) != 0;
    if (e == 0xFFu) {
      *special = m ? 4u : (neg ? 2u : 1u);
      return 0;
    }
    if (e == 0 && m == 0) return 0;
    if (e) m |= 0x800000u;
    shift = e ? e - 1 : 0;  // value = m * 2^(shift + FLOAT_EMIN)
    c = static_cast<unsigned __int128>(m) << (shift & 31u);
  } else {
    const uint64_t e = (bits >> 52) & 0x7FFull;
    uint64_t m = bits & 0xFFFFFFFFFFFFFull;
    neg = (bits >> 63) != 0;
    if (e == 0x7FFull) {
      *special = m ? 4u : (neg ? 2u : 1u);
      return 0;
    }
    if (e == 0 && m == 0) return 0;
    if (e) m |= 1ull << 52;
    shift = e ? static_cast<uint32_t>(e) - 1 : 0;  // value = m * 2^(shift + DOUBLE_EMIN)
    c = static_cast<unsigned __int128>(m) << (shift & 31u);
  }
  *i0 = static_cast<int>(shift >> 5);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int64_t p = static_cast<int64_t>(static_cast<uint32_t>(c >> (32 * k)));
    part[k] = neg ? -p : p;
  }
  return type == HY_TYPE_FLOAT ? 2 : 3;
}

// ------------------------------------------------------------------------------------------------------------
// Wave reductions (64 lanes, 64-bit)
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, WAVE);
  return v;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = __shfl_xor(v, d, WAVE);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = __shfl_xor(v, d, WAVE);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, WAVE));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, WAVE));
  return v;
}

// Applies one word operation atomically (LDS or global, by address space of p).
__device__ __forceinline__ void word_apply(unsigned long long* p, int32_t op, uint64_t v) {
  switch (op) {
    case WOP_ADD:
      if (v) atomicAdd(p, static_cast<unsigned long long>(v));
      break;
    case WOP_MIN:
      if (v != ~0ull) atomicMin(p, static_cast<unsigned long long>(v));
      break;
    case WOP_MAX:
      if (v) atomicMax(p, static_cast<unsigned long long>(v));
      break;
    case WOP_OR:
      if (v) atomicOr(p, static_cast<unsigned long long>(v));
      break;
    default:
      break;
  }
}

__device__ __forceinline__ uint32_t agg_tile_chunk(const AggDesc& d, uint64_t tile) { return d.tile_chunk[tile]; }

// ------------------------------------------------------------------------------------------------------------
// Dense grouping
// ------------------------------------------------------------------------------------------------------------
__global__ void agg_init_records(unsigned long long* __restrict__ rec, uint64_t n_records, uint32_t words,
                                 const int32_t* __restrict__ word_op) {
  const uint64_t n = n_records * words;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    rec[i] = word_init(word_op[i % words]);
}

__global__ __launch_bounds__(AGG_THREADS) void agg_dense_rows(AggDesc d, uint32_t n_groups,
                                                             unsigned long long* __restrict__ records) {
  __shared__ unsigned long long s_rec[AGG_DENSE_LDS_WORDS];
  const uint32_t words = d.words;
  const uint32_t n_words = n_groups * words;
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) s_rec[i] = word_init(d.word_op[i % words]);
  __syncthreads();
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t H = d.n_gb;  // header starts after the key words

  for (uint64_t tile = blockIdx.x; tile < d.n_tiles; tile += gridDim.x) {
    const uint32_t c = agg_tile_chunk(d, tile);
    const uint32_t size = d.chunk_size[c];
    const uint32_t base = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE + w * AGG_WAVE_SPAN;
    const uint64_t row0 = d.chunk_row_begin[c];
    for (int k = 0; k < AGG_ITEMS; ++k) {
      const uint32_t off0 = base + k * WAVE;
      if (off0 >= size) break;  // wave-uniform
      const uint32_t off = off0 + lane;
      const bool active = off < size;
      RowRefs refs;
      if (active) load_refs(d, c, off, &refs);
      // group index
      uint32_t g = 0;
      if (active) {
        for (uint32_t j = 0; j < d.n_gb; ++j) {
          const AggCol& col = d.cols[d.gb[j]];
          uint64_t bits;
          uint32_t code = col.domain;
          if (read_col(d, col, c, off, refs, &bits)) {
            code = static_cast<uint32_t>(bits);
            if (code >= col.domain) {
              atomicOr(d.error, 2u);
              code = col.domain;
            }
          }
          g += code * col.stride;
        }
      }
      uint64_t present = wave_or64(active ? (1ull << g) : 0ull);
      // values of every aggregate's column for this row
      uint64_t vbits[AGG_MAX_AGGREGATES];
      uint32_t valid = 0;
      for (uint32_t f = 0; f < d.n_fns; ++f) {
        vbits[f] = 0;
        const AggFn fn = d.fns[f];
        if (active && fn.column >= 0 && read_col(d, d.cols[fn.column], c, off, refs, &vbits[f])) valid |= 1u << f;
      }
      while (present) {
        const uint32_t gg = static_cast<uint32_t>(__builtin_ctzll(present));
        present &= present - 1;
        const bool mine = active && g == gg;
        const uint64_t m = __ballot(mine);
        unsigned long long* rec = s_rec + gg * words;
        if (lane == 0) {
          atomicAdd(rec + H + AGG_HDR_ROWS, static_cast<unsigned long long>(__popcll(m)));
          atomicMin(rec + H + AGG_HDR_FIRST, static_cast<unsigned long long>(row0 + off0 + __builtin_ctzll(m)));
          atomicMax(rec + H + AGG_HDR_LAST, static_cast<unsigned long long>(row0 + off0 + 63 - __builtin_clzll(m)));
        }
        for (uint32_t f = 0; f < d.n_fns; ++f) {
          const AggFn fn = d.fns[f];
          if (fn.column < 0) continue;  // COUNT(*) = rows
          const bool in = mine && ((valid >> f) & 1u);
          const uint64_t cnt = __popcll(__ballot(in));
          if (lane == 0 && cnt) atomicAdd(rec + fn.word, static_cast<unsigned long long>(cnt));
          if (cnt == 0 || fn.function == HY_AGG_COUNT) continue;
          const int32_t type = d.cols[fn.column].type;
          if (fn.function == HY_AGG_MIN || fn.function == HY_AGG_MAX) {
            const bool is_min = fn.function == HY_AGG_MIN;
            const uint64_t ob = in ? ordered_bits(vbits[f], type) : (is_min ? ~0ull : 0ull);
            const uint64_t r = is_min ? wave_min64(ob) : wave_max64(ob);
            if (lane == 0) {
              if (is_min)
                atomicMin(rec + fn.word + 1, static_cast<unsigned long long>(r));
              else
                atomicMax(rec + fn.word + 1, static_cast<unsigned long long>(r));
            }
          } else if (fn.limbs == 0) {  // SUM / AVG of integers
            const uint64_t s = wave_sum64(in ? static_cast<uint64_t>(int_value(vbits[f], type)) : 0ull);
            if (lane == 0 && s) atomicAdd(rec + fn.word + 1, static_cast<unsigned long long>(s));
          } else {  // SUM / AVG of floats: exact limbs
            int i0 = 0;
            int64_t part[3] = {0, 0, 0};
            uint32_t special = 0;
            const int np = in ? float_parts(vbits[f], type, &i0, part, &special) : 0;
            const uint64_t sp = wave_or64(special);
            if (lane == 0 && sp) atomicOr(rec + fn.word + 1, static_cast<unsigned long long>(sp));
            const int lo = wave_min_i(np ? i0 : 0x7FFFFFFF);
            const int hi = wave_max_i(np ? i0 + np - 1 : -1);
            for (int l = lo; l <= hi; ++l) {
              const int k = l - i0;
              const int64_t v = (np && k >= 0 && k < np) ? part[k] : 0;
              const uint64_t s = wave_sum64(static_cast<uint64_t>(v));
              if (lane == 0 && s) atomicAdd(rec + fn.word + 2 + l, static_cast<unsigned long long>(s));
            }
          }
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) {
    const int32_t op = d.word_op[i % words];
    word_apply(records + i, op, s_rec[i]);
  }
}

// ------------------------------------------------------------------------------------------------------------
// agg_dense_span: the dense path restructured for memory-level parallelism (TPC-H 1 shape). A wave owns a span of
// AGG_WAVE_SPAN = 1024 rows; lane l holds rows span + 64 k + l for k < 16 (coalesced per k). Every column is read
// for all 16 rows in phases (RowIDs, chunk descriptors, values, dictionary entries), so 16 independent loads per lane
// are in flight at each step instead of one dependent chain per row. Per group present in the span, each lane first
// folds its 16 rows in registers (counts, sums, min/max, limb pieces) and the wave then reduces once - 16x fewer
// cross-lane reductions than per-64-row ballots. Requires: at most one PosList group and every used column with one
// encoding (kind / vid width) across its chunks (AggCol::ukind); the host falls back to agg_dense_rows otherwise.
// Results are the same exact sums as agg_dense_rows (the same decoded values; integer-valued float rows are folded
// into the limbs as normalised pieces by span_fold_int_words, so individual limb words may differ).
// ------------------------------------------------------------------------------------------------------------
// A float / double that is an integer of small magnitude (|v| <= 2^24, resp. 2^31): its int64 value. Such rows of a
// float SUM are summed exactly in one int64 word (no overflow below 2^32 rows).
__device__ __forceinline__ bool small_integer(uint64_t bits, int32_t type, int64_t* iv) {
  if (type == HY_TYPE_FLOAT) {
    float f;
    const uint32_t b = static_cast<uint32_t>(bits);
    __builtin_memcpy(&f, &b, 4);
    if (!(fabsf(f) <= 16777216.0f) || f != truncf(f)) return false;
    *iv = static_cast<int64_t>(f);
    return true;
  }
  double x;
  __builtin_memcpy(&x, &bits, 8);
  if (!(fabs(x) <= 2147483648.0) || x != trunc(x)) return false;
  *iv = static_cast<int64_t>(x);
  return true;
}

// Adds the exact int64 word of every float SUM / AVG (integer-valued rows) into its limbs and clears it: value I has
// weight 2^0 = 2^(32 i + o + emin) with i = (-emin) / 32, o = (-emin) % 32. One thread per (group, aggregate).
__device__ __forceinline__ void span_fold_int_words(const AggDesc& d, uint32_t n_groups, unsigned long long* rec) {
  for (uint32_t t = threadIdx.x; t < n_groups * d.n_fns; t += AGG_THREADS) {
    const uint32_t gg = t / d.n_fns;
    const AggFn fn = d.fns[t % d.n_fns];
    if (fn.column < 0 || fn.limbs == 0) continue;
    unsigned long long* r = rec + gg * d.words;
    const int64_t I = static_cast<int64_t>(r[fn.word + 2 + fn.limbs]);
    if (I == 0) continue;
    r[fn.word + 2 + fn.limbs] = 0;
    const int p = fn.limbs == FLOAT_LIMBS ? -FLOAT_EMIN : -DOUBLE_EMIN;
    const unsigned __int128 u = static_cast<unsigned __int128>(I < 0 ? 0ull - static_cast<uint64_t>(I)
                                                                        : static_cast<uint64_t>(I))
                                << (p & 31);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int64_t piece = static_cast<int64_t>(static_cast<uint32_t>(u >> (32 * k)));
      const int l = (p >> 5) + k;
      if (piece && l < fn.limbs) r[fn.word + 2 + l] += static_cast<uint64_t>(I < 0 ? -piece : piece);
    }
  }
}

constexpr int SPAN_K = 4;  // rows per lane per step: a wave span is AGG_ITEMS / SPAN_K steps (register budget)

// Loads the values of column col for the 16 rows of this lane; returns the non-NULL mask (bit k).
__device__ __forceinline__ uint32_t span_load(const AggDesc& d, const AggCol& col, uint32_t c, uint32_t base,
                                              uint32_t act, const hy_row_id (&rid)[SPAN_K], uint64_t (&b)[SPAN_K]) {
  const bool wide = is_wide(col.type);
  const int lane = __lane_id();
  uint32_t ok = act;
  uint32_t off[SPAN_K];
  uint32_t cc = c;  // chunk whose descriptor serves every row of the step when `uniform`
  bool uniform = true;
  if (col.pos_group < 0) {
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) off[k] = base + k * WAVE + lane;
  } else {
    // scan outputs reference one chunk per PosList: then the descriptor is wave-uniform (scalar loads, no per-row
    // descriptor round trip); otherwise rows are read one by one through their own chunk's descriptor
    cc = __builtin_amdgcn_readfirstlane(rid[0].chunk_id);
    bool same = true;
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) {
      off[k] = rid[k].chunk_offset;
      if ((act >> k) & 1u) same = same && rid[k].chunk_id == cc && rid[k].chunk_offset != 0xFFFFFFFFu;
    }
    uniform = __ballot(!same) == 0ull;
  }
  if (!uniform) {
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) {
      b[k] = 0;
      if (!((ok >> k) & 1u)) continue;
      if (rid[k].chunk_offset == 0xFFFFFFFFu || !load_bits(col.chunks[rid[k].chunk_id], off[k], wide, &b[k]))
        ok &= ~(1u << k);
    }
    return ok;
  }
  const hy_column_chunk& ch = col.chunks[cc];
  if (col.ukind == HY_COL_DICT) {
    const void* data = ch.data;
    const void* dict = ch.dictionary;
    const uint32_t dsz = ch.dictionary_size;
    uint32_t vid[SPAN_K];
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) {
      vid[k] = 0xFFFFFFFFu;
      if ((ok >> k) & 1u) {
        if (col.uwidth == 1)
          vid[k] = static_cast<const uint8_t*>(data)[off[k]];
        else if (col.uwidth == 2)
          vid[k] = static_cast<const uint16_t*>(data)[off[k]];
        else
          vid[k] = static_cast<const uint32_t*>(data)[off[k]];
      }
    }
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) {
      b[k] = 0;
      if (((ok >> k) & 1u) && vid[k] < dsz)
        b[k] = wide ? static_cast<const uint64_t*>(dict)[vid[k]] : static_cast<const uint32_t*>(dict)[vid[k]];
      else
        ok &= ~(1u << k);
    }
  } else {
    const void* data = ch.data;
    const uint8_t* nul = col.unulls ? ch.nulls : nullptr;
    uint8_t nf[SPAN_K];
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) {
      b[k] = 0;
      nf[k] = 0;
      if ((ok >> k) & 1u) {
        b[k] = wide ? static_cast<const uint64_t*>(data)[off[k]] : static_cast<const uint32_t*>(data)[off[k]];
        if (nul != nullptr) nf[k] = nul[off[k]];
      }
    }
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k)
      if (nf[k]) {
        ok &= ~(1u << k);
        b[k] = 0;
      }
  }
  return ok;
}

__global__ __launch_bounds__(AGG_THREADS) void agg_dense_span(AggDesc d, uint32_t n_groups,
                                                             unsigned long long* __restrict__ records) {
  extern __shared__ unsigned long long s_recd[];
  const uint32_t words = d.words;
  const uint32_t n_words = n_groups * words;
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) s_recd[i] = word_init(d.word_op[i % words]);
  __syncthreads();
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t H = d.n_gb;

  for (uint64_t tile = blockIdx.x; tile < d.n_tiles; tile += gridDim.x) {
    const uint32_t c = agg_tile_chunk(d, tile);
    const uint32_t size = d.chunk_size[c];
    const uint32_t span = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE + w * AGG_WAVE_SPAN;
    const uint64_t row0 = d.chunk_row_begin[c];
    for (int h = 0; h < AGG_ITEMS / SPAN_K; ++h) {
    const uint32_t base = span + h * SPAN_K * WAVE;
    if (base >= size) break;  // wave-uniform
    uint32_t act = 0;
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k)
      if (base + k * WAVE + lane < size) act |= 1u << k;
    hy_row_id rid[SPAN_K];
    if (d.n_pos_groups) {
      const hy_row_id* pl = d.pos_lists[c];
#pragma unroll
      for (int k = 0; k < SPAN_K; ++k)
        rid[k] = ((act >> k) & 1u) ? pl[base + k * WAVE + lane] : hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu};
    }
    // group index of every row
    uint8_t g[SPAN_K];
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k) g[k] = 0;
    for (uint32_t j = 0; j < d.n_gb; ++j) {
      const AggCol& col = d.cols[d.gb[j]];
      uint64_t b[SPAN_K];
      const uint32_t ok = span_load(d, col, c, base, act, rid, b);
      bool bad = false;
#pragma unroll
      for (int k = 0; k < SPAN_K; ++k) {
        uint32_t code = col.domain;
        if ((ok >> k) & 1u) {
          code = static_cast<uint32_t>(b[k]);
          if (code >= col.domain) {
            bad = true;
            code = col.domain;
          }
        }
        g[k] = static_cast<uint8_t>(g[k] + code * col.stride);
      }
      if (bad) atomicOr(d.error, 2u);
    }
    uint64_t mine_groups = 0;
#pragma unroll
    for (int k = 0; k < SPAN_K; ++k)
      if ((act >> k) & 1u) mine_groups |= 1ull << g[k];
    const uint64_t span_groups = wave_or64(mine_groups);
    // header words: rows, first row, last row
    for (uint64_t pg = span_groups; pg;) {
      const uint32_t gg = static_cast<uint32_t>(__builtin_ctzll(pg));
      pg &= pg - 1;
      uint32_t cnt = 0;
      uint64_t first = ~0ull, last = 0;
#pragma unroll
      for (int k = 0; k < SPAN_K; ++k) {
        if (((act >> k) & 1u) && g[k] == gg) {
          const uint64_t row = row0 + base + k * WAVE + lane;
          ++cnt;
          first = row < first ? row : first;
          last = row > last ? row : last;
        }
      }
      const uint32_t rows = wave_sum(cnt);
      first = wave_min64(first);
      last = wave_max64(last);
      if (lane == 0) {
        unsigned long long* rec = s_recd + gg * words;
        atomicAdd(rec + H + AGG_HDR_ROWS, static_cast<unsigned long long>(rows));
        atomicMin(rec + H + AGG_HDR_FIRST, static_cast<unsigned long long>(first));
        atomicMax(rec + H + AGG_HDR_LAST, static_cast<unsigned long long>(last));
      }
    }
    // aggregates
    for (uint32_t f = 0; f < d.n_fns; ++f) {
      const AggFn fn = d.fns[f];
      if (fn.column < 0) continue;  // COUNT(*) = rows
      const AggCol& col = d.cols[fn.column];
      uint64_t b[SPAN_K];
      const uint32_t ok = span_load(d, col, c, base, act, rid, b);
      const int32_t type = col.type;
      for (uint64_t pg = span_groups; pg;) {
        const uint32_t gg = static_cast<uint32_t>(__builtin_ctzll(pg));
        pg &= pg - 1;
        uint32_t inm = 0;
#pragma unroll
        for (int k = 0; k < SPAN_K; ++k)
          if (((ok >> k) & 1u) && g[k] == gg) inm |= 1u << k;
        const uint32_t cnt = wave_sum(static_cast<uint32_t>(__popc(inm)));
        unsigned long long* rec = s_recd + gg * words;
        if (lane == 0 && cnt) atomicAdd(rec + fn.word, static_cast<unsigned long long>(cnt));
        if (cnt == 0 || fn.function == HY_AGG_COUNT) continue;
        if (fn.function == HY_AGG_MIN || fn.function == HY_AGG_MAX) {
          const bool is_min = fn.function == HY_AGG_MIN;
          uint64_t r = is_min ? ~0ull : 0ull;
#pragma unroll
          for (int k = 0; k < SPAN_K; ++k) {
            if ((inm >> k) & 1u) {
              const uint64_t ob = ordered_bits(b[k], type);
              r = is_min ? (ob < r ? ob : r) : (ob > r ? ob : r);
            }
          }
          r = is_min ? wave_min64(r) : wave_max64(r);
          if (lane == 0) {
            if (is_min)
              atomicMin(rec + fn.word + 1, static_cast<unsigned long long>(r));
            else
              atomicMax(rec + fn.word + 1, static_cast<unsigned long long>(r));
          }
        } else if (fn.limbs == 0) {  // SUM / AVG of integers (two's complement wrap, like agg_dense_rows)
          uint64_t s = 0;
#pragma unroll
          for (int k = 0; k < SPAN_K; ++k)
            if ((inm >> k) & 1u) s += static_cast<uint64_t>(int_value(b[k], type));
          s = wave_sum64(s);
          if (lane == 0 && s) atomicAdd(rec + fn.word + 1, static_cast<unsigned long long>(s));
        } else {  // SUM / AVG of floats: exact limbs; each row's pieces are split once, then summed per limb
          // integer-valued rows (TPC-H quantities, cents) skip the limbs: an exact int64 word, folded into the
          // limbs when the workgroup flushes (span_fold_int_words); only the other rows are split into pieces
          {
            uint64_t isum = 0;
            uint32_t frac = 0;
#pragma unroll
            for (int k = 0; k < SPAN_K; ++k) {
              if ((inm >> k) & 1u) {
                int64_t iv;
                if (small_integer(b[k], type, &iv))
                  isum += static_cast<uint64_t>(iv);
                else
                  frac |= 1u << k;
              }
            }
            isum = wave_sum64(isum);
            if (lane == 0 && isum) atomicAdd(rec + fn.word + 2 + fn.limbs, static_cast<unsigned long long>(isum));
            if (__ballot(frac != 0) == 0ull) continue;
            inm = frac;
          }
          uint32_t special = 0;
          int lo = 0x7FFFFFFF, hi = -1;
          int i0s[SPAN_K];
          int64_t pc[SPAN_K][3];
#pragma unroll
          for (int k = 0; k < SPAN_K; ++k) {
            i0s[k] = -4;  // no piece of this row matches any limb
            pc[k][0] = pc[k][1] = pc[k][2] = 0;
            if ((inm >> k) & 1u) {
              int i0 = 0;
              uint32_t sp = 0;
              const int np = float_parts(b[k], type, &i0, pc[k], &sp);
              special |= sp;
              if (np) {
                i0s[k] = i0;
                lo = min(lo, i0);
                hi = max(hi, i0 + np - 1);
              } else {
                pc[k][0] = pc[k][1] = pc[k][2] = 0;
              }
            }
          }
          const uint64_t spw = wave_or64(special);
          if (lane == 0 && spw) atomicOr(rec + fn.word + 1, static_cast<unsigned long long>(spw));
          lo = wave_min_i(lo);
          hi = wave_max_i(hi);
          for (int l = lo; l <= hi; ++l) {
            int64_t s = 0;
#pragma unroll
            for (int k = 0; k < SPAN_K; ++k) {
              const int q = l - i0s[k];
              s += q == 0 ? pc[k][0] : (q == 1 ? pc[k][1] : (q == 2 ? pc[k][2] : 0));
            }
            const uint64_t ws = wave_sum64(static_cast<uint64_t>(s));
            if (lane == 0 && ws) atomicAdd(rec + fn.word + 2 + l, static_cast<unsigned long long>(ws));
          }
        }
      }
    }
    }  // steps of the span
  }
  __syncthreads();
  span_fold_int_words(d, n_groups, s_recd);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) {
    const int32_t op = d.word_op[i % words];
    word_apply(records + i, op, s_recd[i]);
  }
}

// Dense records -> compact group records with their key words (code per group-by column, NULL code = domain).
__global__ void agg_dense_compact(AggDesc d, uint32_t n_groups, const unsigned long long* __restrict__ records,
                                  unsigned long long* __restrict__ out, uint64_t capacity,
                                  unsigned long long* __restrict__ n_out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const unsigned long long* rec = records + static_cast<uint64_t>(g) * d.words;
  if (rec[d.n_gb + AGG_HDR_ROWS] == 0) return;
  const uint64_t idx = atomicAdd(n_out, 1ull);
  if (idx >= capacity) return;
  unsigned long long* o = out + idx * d.words;
  for (uint32_t i = 0; i < d.words; ++i) o[i] = rec[i];
  uint64_t nulls = 0;
  for (uint32_t j = 0; j < d.n_gb; ++j) {
    const AggCol& col = d.cols[d.gb[j]];
    const uint32_t code = (g / col.stride) % (col.domain + 1);
    o[j] = code == col.domain ? 0ull : code;
    if (code == col.domain) nulls |= 1ull << j;
  }
  o[d.n_gb + AGG_HDR_NULLS] = nulls;
}

// ------------------------------------------------------------------------------------------------------------
// Hash grouping
// ------------------------------------------------------------------------------------------------------------
constexpr uint32_t HSLOT_EMPTY = 0, HSLOT_LOCKED = 1, HSLOT_READY = 2;

struct AggTable {
  uint32_t* state;                 // cap
  unsigned long long* records;     // cap * words
  uint64_t cap;                    // power of two
  // COUNT(DISTINCT) set: keys (slot << 8 | aggregate, value bits)
  uint32_t* dstate;
  unsigned long long* dkeys;       // dcap * 2
  uint64_t dcap;
};

constexpr uint64_t LOCK_SPIN_LIMIT = 1ull << 22;  // waits on a slot being initialised (not probe steps)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Group table visibility (MI355X_MICROARCH.md, inter-workgroup visibility: the "8-B agent atomics on both sides"
// form). Every table word another workgroup reads in this launch is written and read with 8-B relaxed agent-scope
// atomics (sc1 stores / loads, coherent per location across XCDs), the claimer drains its stores (s_waitcnt
// vmcnt(0)) before it publishes the slot as READY, and readers load the keys only after they saw READY. No release /
// acquire fences: at agent scope those are an L2 writeback / L1 invalidate (microseconds each), once per group.
__device__ __forceinline__ uint64_t table_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void table_store(unsigned long long* p, uint64_t v) {
  __hip_atomic_store(p, static_cast<unsigned long long>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The records one wave claims in one probe round, staged for the wave's cooperative initialisation.
struct ClaimStage {
  uint64_t slot[WAVE];
  uint64_t key[WAVE][AGG_MAX_GROUPBY + 1];
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every lane of the wave calls this together; a lane with `want` gets the slot of the group with its key words,
// inserted if new, ~0 on failure (other lanes: ~0). The probe loop runs in wave-uniform rounds: the slots the wave's
// lanes claim in a round are initialised by the whole wave - consecutive lanes store consecutive words of the claimed
// records, so a 19-word record leaves as ~3 line writes instead of 19 separate 8-byte write-throughs - drained, and
// published before the next round. No claim outlives its round, so a lane that meets a slot locked by its own wave
// only waits for that round's publish.
__device__ __forceinline__ uint64_t group_slot_wave(const AggDesc& d, const AggTable& t, const uint64_t* key,
                                                    uint32_t nk, bool want, ClaimStage& cs) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < nk; ++i) h = mix64(h ^ key[i]);
  uint64_t s = h & (t.cap - 1);
  // a READY slot's state word carries a tag of the key's hash (>= HSLOT_READY): other keys are skipped without
  // loading their key words
  const uint32_t tag = static_cast<uint32_t>(h >> 32) | HSLOT_READY;
  const uint32_t W = d.words;
  const int lane = __lane_id();
  uint64_t result = ~0ull, probes = 0, spins = 0;
  bool active = want;
  while (__ballot(active)) {
    bool claimed = false;
    if (active) {
      if (probes >= t.cap || spins >= LOCK_SPIN_LIMIT) {
        atomicOr(d.error, 1u);
        active = false;
      } else {
        const uint32_t st = __hip_atomic_load(&t.state[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st == HSLOT_EMPTY) {
          // (no insert counter: the compaction counts the groups, and past the load limit the host reports
          // HY_ERR_GROUP_BOUND. A counter per insert - even 64 sharded ones - serialises ~10^4 atomics per word at
          // the L2: TPC-H 3 SF100, 1.1 M groups, 2 ms.) A lost race re-reads the same slot next round.
          uint32_t expected = HSLOT_EMPTY;
          claimed = __hip_atomic_compare_exchange_strong(&t.state[s], &expected, HSLOT_LOCKED, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (st == HSLOT_LOCKED) {
          ++spins;
        } else {
          bool match = false;
          if (st == tag) {
            const unsigned long long* rec = t.records + s * W;
            uint64_t diff = 0;  // every key word loaded at once (no short-circuit chain of dependent loads)
            for (uint32_t i = 0; i < nk; ++i) diff |= table_load(rec + i) ^ key[i];
            match = diff == 0;
          }
          if (match) {
            result = s;
            active = false;
          } else {
            s = (s + 1) & (t.cap - 1);
            ++probes;
          }
        }
      }
    }
    const uint64_t cm = __ballot(claimed);
    if (cm == 0) {
      if (__ballot(active)) __builtin_amdgcn_s_sleep(1);  // only locked slots left to wait for
      continue;
    }
    if (claimed) {
      const uint32_t r = static_cast<uint32_t>(__popcll(cm & lanemask_lt()));
      cs.slot[r] = s;
      for (uint32_t i = 0; i < nk; ++i) cs.key[r][i] = key[i];
    }
    wave_lds_sync();
    const uint32_t n = static_cast<uint32_t>(__popcll(cm));
    for (uint32_t e = lane; e < n * W; e += WAVE) {
      const uint32_t q = e / W, w = e - q * W;
      table_store(t.records + cs.slot[q] * W + w, w < nk ? cs.key[q][w] : word_init(d.word_op[w]));
    }
    drain_stores();
    wave_lds_sync();  // (the stage is rewritten next round)
    if (claimed) {
      __hip_atomic_store(&t.state[s], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      result = s;
      active = false;
    }
  }
  return result;
}

// true if (tag, value) was not in the distinct set yet
__device__ __forceinline__ bool distinct_insert(const AggDesc& d, const AggTable& t, uint64_t tag, uint64_t value) {
  uint64_t s = mix64(tag * 0x9E3779B97F4A7C15ull ^ mix64(value)) & (t.dcap - 1);
  uint64_t probes = 0, spins = 0;
  while (probes < t.dcap && spins < LOCK_SPIN_LIMIT) {
    const uint32_t st = __hip_atomic_load(&t.dstate[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st == HSLOT_EMPTY) {
      uint32_t expected = HSLOT_EMPTY;
      if (__hip_atomic_compare_exchange_strong(&t.dstate[s], &expected, HSLOT_LOCKED, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        table_store(t.dkeys + 2 * s, tag);
        table_store(t.dkeys + 2 * s + 1, value);
        drain_stores();
        __hip_atomic_store(&t.dstate[s], HSLOT_READY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
      }
      continue;
    }
    if (st == HSLOT_LOCKED) {
      ++spins;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (table_load(t.dkeys + 2 * s) == tag && table_load(t.dkeys + 2 * s + 1) == value) return false;
    s = (s + 1) & (t.dcap - 1);
    ++probes;
  }
  atomicOr(d.error, 1u);
  return false;
}

// Flat row mapping (kernels whose tiles run over the input's global row numbers, so that many small chunks, e.g. a
// join output's radix partitions, do not leave most lanes of a chunk-aligned tile idle): chunk of global row r, the
// last chunk whose first row is <= r (empty chunks are skipped by construction).
__device__ __forceinline__ uint32_t row_chunk(const AggDesc& d, uint64_t r) {
  uint32_t lo = 0, hi = d.n_chunks;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (d.chunk_row_begin[mid] <= r) lo = mid;
    else hi = mid;
  }
  return lo;
}
// The same for a row after the row whose chunk is c (rows only move forward within a lane).
__device__ __forceinline__ uint32_t advance_chunk(const AggDesc& d, uint32_t c, uint64_t r) {
  while (d.chunk_row_begin[c + 1] <= r) ++c;
  return c;
}

// The chunks a tile's rows fall into, as first-row offsets from the tile's first row in LDS: a row's chunk is then a
// binary search in LDS instead of a chain of dependent global loads (row_chunk's search, then advance_chunk's walk
// over the ~46-row partitions of a join output: ~9 dependent loads per row, TPC-H 3's projection / aggregate inputs).
// A tile spanning more than CW_MAX chunks (empty chunks) falls back to row_chunk per row.
constexpr uint32_t CW_MAX = 2048;
struct ChunkWin {
  uint32_t c0, n;    // first chunk, chunks
  uint64_t base0;    // first row of chunk c0
};
struct ChunkWinLds {
  uint32_t begin[CW_MAX];  // begin[i] = first row of chunk c0 + i - tile_row0 (0 for i = 0)
  uint32_t c[2];
  uint64_t base0;
};
// Every thread of the workgroup calls it (two barriers); rows [tile_row0, tile_end) with tile_end <= total rows.
__device__ __forceinline__ ChunkWin chunk_window(const AggDesc& d, uint64_t tile_row0, uint64_t tile_end,
                                                 ChunkWinLds& s) {
  if (threadIdx.x == 0) {
    const uint32_t c0 = tile_end > tile_row0 ? row_chunk(d, tile_row0) : 0u;
    s.c[0] = c0;
    s.c[1] = tile_end > tile_row0 ? row_chunk(d, tile_end - 1) : c0;
    s.base0 = d.chunk_row_begin[c0];
  }
  __syncthreads();
  ChunkWin w{s.c[0], s.c[1] - s.c[0] + 1, s.base0};
  if (w.n <= CW_MAX)
    for (uint32_t i = threadIdx.x; i < w.n; i += blockDim.x)
      s.begin[i] = i == 0 ? 0u : static_cast<uint32_t>(d.chunk_row_begin[w.c0 + i] - tile_row0);
  __syncthreads();
  return w;
}
// Chunk and chunk offset of `row` of the tile (the last chunk whose first row is <= row, as row_chunk).
__device__ __forceinline__ uint32_t win_chunk(const AggDesc& d, const ChunkWin& w, const ChunkWinLds& s,
                                              uint64_t tile_row0, uint64_t row, uint32_t* off) {
  if (w.n > CW_MAX) {
    const uint32_t c = row_chunk(d, row);
    *off = static_cast<uint32_t>(row - d.chunk_row_begin[c]);
    return c;
  }
  const uint32_t r = static_cast<uint32_t>(row - tile_row0);
  uint32_t lo = 0, hi = w.n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s.begin[mid] <= r) lo = mid;
    else hi = mid;
  }
  *off = lo ? r - s.begin[lo] : static_cast<uint32_t>(row - w.base0);
  return w.c0 + lo;
}

// Inclusive scan inside runs of lanes: lane i combines lanes [start, i] of its run.
template <typename T, typename Op>
__device__ __forceinline__ T run_scan(T v, int start, Op op) {
  const int lane = __lane_id();
#pragma unroll
  for (int dd = 1; dd < WAVE; dd <<= 1) {
    const T o = __shfl_up(v, dd, WAVE);
    if (lane - dd >= start) v = op(v, o);
  }
  return v;
}

// Hash grouping. The 64 lanes of a wave hold 64 consecutive input rows; lanes whose group-by keys equal their left
// neighbour's form a run (rows of one group arriving together, e.g. the lines of one order after a join on the order
// key). Every run is folded inside the wave (segmented shuffle scans) and applied to its group record once, by the
// run's last lane: one table lookup and one set of atomics per run instead of per row. Float SUM/AVG runs whose values
// share a limb window are folded exactly in that window (integer limb parts); other runs add per row. The record
// words are combined by ADD / MIN / MAX / OR, so the result is the same for any order and any run split.
// Rows per lane of a flat tile: enough tiles to give every CU several workgroups, at most AGG_ITEMS.
inline uint32_t flat_items(uint64_t rows) {
  const uint64_t want_tiles = 256ull * 8;
  const uint64_t items = (rows + uint64_t(AGG_THREADS) * want_tiles - 1) / (uint64_t(AGG_THREADS) * want_tiles);
  return static_cast<uint32_t>(items < 1 ? 1 : (items > AGG_ITEMS ? AGG_ITEMS : items));
}

__global__ __launch_bounds__(AGG_THREADS) void agg_hash_runs(AggDesc d, AggTable t, uint64_t total_rows,
                                                             uint32_t items) {
  __shared__ ClaimStage s_claim[AGG_THREADS / WAVE];
  __shared__ ChunkWinLds s_win;
  const int lane = __lane_id();
  const uint64_t tile_row0 = static_cast<uint64_t>(blockIdx.x) * AGG_THREADS * items;
  const uint32_t H = d.n_gb;
  uint32_t c = 0;
  const ChunkWin win =
      chunk_window(d, tile_row0, min(total_rows, tile_row0 + static_cast<uint64_t>(AGG_THREADS) * items), s_win);
  for (uint32_t k = 0; k < items; ++k) {
    const uint64_t wave_row0 = tile_row0 + static_cast<uint64_t>(k) * AGG_THREADS + (threadIdx.x & ~(WAVE - 1u));
    if (wave_row0 >= total_rows) break;  // wave-uniform
    const uint64_t row = wave_row0 + lane;
    const bool valid = row < total_rows;
    uint32_t off = 0;
    RowRefs refs;
    uint64_t key[AGG_MAX_GROUPBY + 1];
    for (uint32_t j = 0; j <= H; ++j) key[j] = 0;
    if (valid) {
      c = win_chunk(d, win, s_win, tile_row0, row, &off);
      if (d.n_pos_groups) load_refs(d, c, off, &refs);
      uint64_t nulls = 0;
      for (uint32_t j = 0; j < H; ++j) {
        const AggCol& col = d.cols[d.gb[j]];
        uint64_t bits;
        if (read_col(d, col, c, off, refs, &bits)) key[j] = key_bits(bits, col.type);
        else nulls |= 1ull << j;
      }
      key[H] = nulls;
    }
    // runs: a lane starts a run unless it is valid and its keys equal the previous lane's (invalid lanes, a suffix
    // of the wave, are runs of their own and do nothing)
    bool same = valid && lane > 0;
    for (uint32_t j = 0; j <= H; ++j) {
      const uint64_t prev = __shfl_up(key[j], 1, WAVE);
      same = same && prev == key[j];
    }
    const uint64_t heads = __ballot(!same);
    const uint64_t upto = (2ull << lane) - 1;  // lanes [0, lane] (all lanes for lane 63)
    const int start = 63 - __builtin_clzll(heads & upto);
    const uint64_t after = heads & ~upto;
    const int end = after ? __builtin_ctzll(after) - 1 : WAVE - 1;
    const uint64_t run_mask = (end == WAVE - 1 ? ~0ull : ((2ull << end) - 1)) & ~((1ull << start) - 1);
    const bool tail = valid && end == lane;
    uint64_t s = group_slot_wave(d, t, key, H + 1, tail, s_claim[threadIdx.x / WAVE]);
    s = __shfl(s, end, WAVE);  // the run's slot, in every lane of the run
    unsigned long long* rec = (valid && s != ~0ull) ? t.records + s * d.words : nullptr;
    if (tail && rec) {
      atomicAdd(rec + H + AGG_HDR_ROWS, static_cast<unsigned long long>(end - start + 1));
      atomicMin(rec + H + AGG_HDR_FIRST, static_cast<unsigned long long>(row - (lane - start)));
      atomicMax(rec + H + AGG_HDR_LAST, static_cast<unsigned long long>(row));
    }
    for (uint32_t f = 0; f < d.n_fns; ++f) {
      const AggFn fn = d.fns[f];
      if (fn.column < 0) continue;
      const int32_t type = d.cols[fn.column].type;
      uint64_t bits = 0;
      const bool ok = rec != nullptr && read_col(d, d.cols[fn.column], c, off, refs, &bits);
      const uint32_t cnt = __popcll(__ballot(ok) & run_mask);
      if (fn.function == HY_AGG_COUNT_DISTINCT) {
        if (ok && distinct_insert(d, t, (s << 8) | f, key_bits(bits, type))) atomicAdd(rec + fn.word, 1ull);
        continue;
      }
      if (tail && rec && cnt) atomicAdd(rec + fn.word, static_cast<unsigned long long>(cnt));
      if (fn.function == HY_AGG_COUNT) continue;
      if (fn.function == HY_AGG_MIN || fn.function == HY_AGG_MAX) {
        const bool mx = fn.function == HY_AGG_MAX;
        uint64_t v = ok ? ordered_bits(bits, type) : (mx ? 0ull : ~0ull);
        v = mx ? run_scan(v, start, [](uint64_t a, uint64_t b) { return a > b ? a : b; })
               : run_scan(v, start, [](uint64_t a, uint64_t b) { return a < b ? a : b; });
        if (tail && rec && cnt) {
          if (mx) atomicMax(rec + fn.word + 1, static_cast<unsigned long long>(v));
          else atomicMin(rec + fn.word + 1, static_cast<unsigned long long>(v));
        }
        continue;
      }
      if (fn.limbs == 0) {  // SUM / AVG of integers
        uint64_t v = ok ? static_cast<uint64_t>(int_value(bits, type)) : 0ull;
        v = run_scan(v, start, [](uint64_t a, uint64_t b) { return a + b; });
        if (tail && rec && v) atomicAdd(rec + fn.word + 1, static_cast<unsigned long long>(v));
        continue;
      }
      // SUM / AVG of floats
      int i0 = 0;
      int64_t part[3] = {0, 0, 0};
      uint32_t special = 0;
      const int np = ok ? float_parts(bits, type, &i0, part, &special) : 0;
      const uint64_t sp = run_scan(static_cast<uint64_t>(special), start, [](uint64_t a, uint64_t b) { return a | b; });
      if (tail && rec && sp) atomicOr(rec + fn.word + 1, static_cast<unsigned long long>(sp));
      const bool has = np > 0;
      int lo = run_scan(has ? i0 : 0x7FFFFFFF, start, [](int a, int b) { return a < b ? a : b; });
      int hi = run_scan(has ? i0 : -1, start, [](int a, int b) { return a > b ? a : b; });
      lo = __shfl(lo, end, WAVE);
      hi = __shfl(hi, end, WAVE);
      if (hi - lo <= 1) {  // the run's parts fit limbs [lo, lo + np]: fold them exactly, one atomic per limb
        const int rel = has ? i0 - lo : 0;
        const int W = type == HY_TYPE_FLOAT ? 3 : 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q >= W) break;
          int64_t v = 0;
          if (has) v = rel == 0 ? (q < 3 ? part[q] : 0) : (q >= 1 ? part[q - 1] : 0);
          v = static_cast<int64_t>(
              run_scan(static_cast<uint64_t>(v), start, [](uint64_t a, uint64_t b) { return a + b; }));
          if (tail && rec && v && lo + q < fn.limbs)
            atomicAdd(rec + fn.word + 2 + lo + q, static_cast<unsigned long long>(v));
        }
      } else if (has) {
        for (int q = 0; q < np; ++q)
          if (part[q]) atomicAdd(rec + fn.word + 2 + i0 + q, static_cast<unsigned long long>(part[q]));
      }
    }
  }
}

// The table's occupied slots into `out`. A workgroup takes HC_ITEMS consecutive 256-slot rows of the table at a time:
// its threads count their occupied slots, one block scan gives every thread its offset and ONE atomic on the output
// counter reserves the workgroup's range. (One atomic per occupied slot - or per wave - on the single counter is
// serialised at the L2: Q3 SF100, 1.6 ms either way.)
constexpr int HC_ITEMS = 16;
__global__ __launch_bounds__(256) void agg_hash_compact(AggDesc d, AggTable t, unsigned long long* __restrict__ out,
                                                        uint64_t capacity, unsigned long long* __restrict__ n_out) {
  __shared__ uint32_t s_scan[256 / WAVE + 1];
  __shared__ unsigned long long s_base;
  __shared__ uint16_t s_src[256 * HC_ITEMS];  // the row's occupied slots (offsets in the row), in output order
  constexpr uint64_t PER = 256ull * HC_ITEMS;
  for (uint64_t b0 = blockIdx.x * PER; b0 < t.cap; b0 += static_cast<uint64_t>(gridDim.x) * PER) {
    uint32_t occ = 0;  // bit i: slot b0 + i * 256 + threadIdx.x holds a group
#pragma unroll
    for (int i = 0; i < HC_ITEMS; ++i) {
      const uint64_t sl = b0 + static_cast<uint64_t>(i) * 256 + threadIdx.x;
      if (sl < t.cap && t.state[sl] >= HSLOT_READY) occ |= 1u << i;  // READY slots hold a hash tag >= HSLOT_READY
    }
    uint32_t total;
    const uint32_t pos = block_exclusive_sum<256>(static_cast<uint32_t>(__popc(occ)), s_scan, &total);
    if (threadIdx.x == 0) s_base = total ? atomicAdd(n_out, static_cast<unsigned long long>(total)) : 0ull;
    __syncthreads();
    // the row's records copied word by word by the whole workgroup: consecutive lanes read and write consecutive
    // words (one lane copying a whole record wrote 8-byte pieces 19 words apart: ~5x the output bytes in partial
    // line writes at TPC-H 3)
    uint32_t r = pos;
    while (occ) {
      const int i = __builtin_ctz(occ);
      occ &= occ - 1;
      s_src[r++] = static_cast<uint16_t>(i * 256 + threadIdx.x);
    }
    __syncthreads();
    const uint64_t base = s_base;
    const uint32_t W = d.words;
    for (uint32_t e = threadIdx.x; e < total * W; e += 256) {
      const uint32_t rr = e / W, w = e - rr * W;
      if (base + rr < capacity) out[(base + rr) * W + w] = t.records[(b0 + s_src[rr]) * W + w];
    }
    __syncthreads();  // s_base and s_src read by every thread before the next row's
  }
}

}  // namespace hyk
