// TableScan kernels for gfx950.
//
// One launch scans every chunk of one column class (dictionary u8/u16/u32 attribute vectors, or value columns of
// one type) and writes, per chunk, the ascending list of matching chunk offsets — the PosList that
// BaseTableScanImpl::_unary_scan_with_value builds per chunk (reference
// src/lib/operators/table_scan/base_table_scan_impl.hpp:33-63).
//
// Layout: a tile is 4096 consecutive rows of one chunk; thread t of the 256-thread workgroup owns rows
// [16t, 16t+16) and reads them with 16-byte vector loads (1 B/row for u8 vids -> one dwordx4 per lane).
// Matches are compacted order-preservingly: per-thread popcount -> workgroup exclusive sum -> decoupled look-back
// across the tiles of the same chunk -> offsets staged in LDS -> coalesced stores.
// The roofline is HBM: vid_width bytes read per row + 4 bytes written per match.
//
// Compressed chunks are scanned in their compressed form:
//   FrameOfReference (MODE_FOR): the 1/2/4-byte offsets stream through the same tiles; a thread's 16 rows share one
//     2048-row block, whose minimum is added back before the compare (frame_of_reference_column.cpp:25-37) -
//     offset bytes per row instead of the value's 4 / 8.
//   RunLength: one predicate evaluation per run, then the matching runs' row ranges are expanded straight into the
//     output (rle_* kernels below) - the rows themselves are never read.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.hpp"

namespace hyk {

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ROWS_PER_THREAD = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ROWS_PER_THREAD;  // 4096

struct ScanLaunchDesc {
  const hy_scan_chunk* chunks;       // device copy of this class's chunk descriptors
  const uint64_t* chunk_tile_begin;  // n_chunks + 1 prefix of tile counts
  const uint32_t* tile_chunk;        // n_tiles: chunk of each tile (fill_tile_owner)
  const uint32_t* chunk_index;       // original chunk index (for counts[])
  const uint32_t* chunk_ids;         // chunk id written into RowID outputs
  uint64_t n_rows;
  uint32_t n_chunks;
  uint64_t n_tiles;
  uint64_t* status;                  // n_tiles look-back words (zeroed)
  uint32_t* ticket;                  // zeroed
  uint32_t* error;                   // zeroed before the first launch of a call
  uint32_t* masks;                   // two-pass scans: the count pass's match masks, mask_words(SEG) x 256 per segment
};

// 32-bit words a lane's SEG 16-bit tile masks take (two tiles per word)
__host__ __device__ constexpr int mask_words(int seg) { return (seg + 1) / 2; }

template <typename T>
struct ScanConst {
  T value;
};

// Loads 16 consecutive elements of E bytes starting at element `first` (16-byte aligned), elements past `n`
// are returned as garbage and masked by the caller.
template <typename E>
__device__ __forceinline__ void load16(const E* __restrict__ base, uint32_t first, E (&out)[16]) {
  constexpr int VECS = sizeof(E);  // 16 elements * sizeof(E) bytes / 16 bytes per vector
  const u32x4* p = reinterpret_cast<const u32x4*>(base + first);
  u32x4 tmp[VECS];
#pragma unroll
  for (int i = 0; i < VECS; ++i) tmp[i] = __builtin_nontemporal_load(p + i);
  __builtin_memcpy(out, tmp, sizeof(tmp));
}

// Tiles per workgroup ("segment"): 128 bytes of loads in flight per lane whatever the element width.
template <typename E>
__host__ __device__ constexpr int seg_tiles() {
  return sizeof(E) >= 8 ? 1 : static_cast<int>(8 / sizeof(E));
}

enum { MODE_VALUE = 0, MODE_DICT = 1, MODE_FOR = 2 };

// Match mask of the 16 rows [row0, row0 + 16) of chunk ch (bit i = row row0 + i matches). E: the element read from
// memory (value / value id / frame-of-reference offset); V: the value type compared (E except for MODE_FOR).
template <typename E, int MODE, typename V>
__device__ __forceinline__ uint32_t match_mask(const hy_scan_chunk& ch, uint32_t row0, const E (&v)[16],
                                               const u32x4& nulls, const ScanConst<V>& constant) {
  constexpr bool IS_DICT = MODE == MODE_DICT;
  const uint32_t n = ch.column.size;
  if (row0 >= n || ch.op == HY_OP_NONE) return 0u;
  uint32_t mask = 0;
  const uint32_t valid = (n - row0) >= 16 ? 0xFFFFu : ((1u << (n - row0)) - 1u);
  const int op = ch.op;
  if constexpr (IS_DICT) {
    const E null_vid = static_cast<E>(ch.column.dictionary_size);
    if (op == HY_OP_VID_SET) {  // like_table_scan_impl.cpp:62-83: dictionary_matches[vid], NULL rows skipped
      const uint32_t* __restrict__ set = ch.vid_set;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t vid = static_cast<uint32_t>(v[i]);
        const bool m = v[i] != null_vid && ((set[vid >> 5] >> (vid & 31)) & 1u);
        mask |= static_cast<uint32_t>(m) << i;
      }
      return mask & valid;
    }
    // comparisons, ALL / NONE and IS [NOT] NULL (is_null_table_scan_impl.cpp:55-61: the iterator's is_null() is
    // vid == null id) as one id range
    const DictPred pr = dict_pred(op, static_cast<E>(ch.search_vid), null_vid);
#pragma unroll
    for (int i = 0; i < 16; ++i) mask |= static_cast<uint32_t>(dict_match(pr, v[i])) << i;
  } else {
    uint8_t nl[16];
    __builtin_memcpy(nl, &nulls, 16);
    if (op == HY_OP_IS_NULL) {  // is_null_table_scan_impl.cpp:35-53 (a column without null flags matches none)
#pragma unroll
      for (int i = 0; i < 16; ++i) mask |= static_cast<uint32_t>(nl[i] != 0) << i;
      return mask & valid;
    }
    if constexpr (MODE == MODE_FOR) {
      const V base = static_cast<const V*>(ch.column.dictionary)[row0 >> 11];  // the 16 rows share one block
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const V x = static_cast<V>(base + static_cast<V>(v[i]));
        const bool m = (nl[i] == 0) & cmp_op<V>(op, x, constant.value);
        mask |= static_cast<uint32_t>(m) << i;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool m = (nl[i] == 0) & cmp_op<E>(op, v[i], constant.value);
        mask |= static_cast<uint32_t>(m) << i;
      }
    }
  }
  return mask & valid;
}

// E = element type read from memory (vid type for DICT, value type for VALUE, offset type for FOR); MODE selects the
// semantics, V the compared value type. OUT_ROWID: write reference RowIDs {chunk_id, offset} (8 B) instead of chunk
// offsets (4 B).
// SEG: tiles per workgroup (seg_tiles<E>; the host may pick fewer for 1-byte elements: more, shorter workgroups).
// 1-byte ids with at most 4 tiles per workgroup run at 8 waves per SIMD (<= 64 VGPRs: 76 otherwise, 6 waves).

// The per-lane 16-bit match masks of one segment (SEG consecutive tiles from tile_row0 of chunk ch): all SEG loads
// per lane issued up front, then the compares.
template <typename E, int MODE, typename V, int SEG>
__device__ __forceinline__ void segment_masks(const hy_scan_chunk& ch, uint32_t tile_row0, const ScanConst<V>& constant,
                                              uint32_t (&masks)[SEG]) {
  const uint32_t n = ch.column.size;
  E v[SEG][16];
  u32x4 nl[SEG];
#pragma unroll
  for (int t = 0; t < SEG; ++t) {
    const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    nl[t] = u32x4{0u, 0u, 0u, 0u};
    if (r0 < n && ch.op != HY_OP_NONE) {
      load16(reinterpret_cast<const E*>(ch.column.data), r0, v[t]);
      if (MODE != MODE_DICT && ch.column.nulls != nullptr) nl[t] = *reinterpret_cast<const u32x4*>(ch.column.nulls + r0);
    }
  }
#pragma unroll
  for (int t = 0; t < SEG; ++t)
    masks[t] = match_mask<E, MODE, V>(ch, tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD, v[t], nl[t],
                                      constant);
}

// A segment's matches, tile by tile, compacted through LDS into coalesced stores from output position `run` on.
template <bool OUT_ROWID, int SEG>
__device__ __forceinline__ void segment_store(const uint32_t (&masks)[SEG], uint32_t tile_row0, uint32_t n, uint64_t run,
                                              uint32_t cid, void* __restrict__ out_any, uint32_t* s_stage,
                                              uint32_t* s_scratch) {
#pragma unroll
  for (int t = 0; t < SEG; ++t) {
    if (tile_row0 + t * SCAN_TILE >= n) break;  // uniform
    const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    uint32_t tile_total;
    uint32_t pos = block_exclusive_sum<SCAN_THREADS>(__popc(masks[t]), s_scratch, &tile_total);
    // stage matching offsets in LDS in order, then store them coalesced
    uint32_t m = masks[t];
    while (m) {
      const int i = __builtin_ctz(m);
      m &= m - 1;
      s_stage[pos++] = r0 + i;
    }
    __syncthreads();
    if constexpr (OUT_ROWID) {
      hy_row_id* out = static_cast<hy_row_id*>(out_any) + run;
      // streaming stores: the RowIDs are read by a later operator, not by this kernel (8 B {chunk_id, offset} each),
      // two per 16-byte store from a 16-byte boundary on (tools/scan_probe.hip, profiles/r05_scan_probe.jsonl: the
      // 221 MB RowID write of config 2 takes 0.052 ms this way against 0.063 ms with one 8-byte store per RowID)
      uint64_t* out64 = reinterpret_cast<uint64_t*>(out);
      const uint32_t lead = (reinterpret_cast<uintptr_t>(out64) & 15u) ? 1u : 0u;  // (RowIDs are 8-byte aligned)
      if (lead && threadIdx.x == 0 && tile_total)
        __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[0]) << 32), out64);
      const uint32_t body = tile_total > lead ? tile_total - lead : 0u;
      u64x2* out128 = reinterpret_cast<u64x2*>(out64 + lead);
      for (uint32_t p = threadIdx.x; p < body / 2; p += SCAN_THREADS) {
        const uint32_t i = lead + 2 * p;
        u64x2 v;
        v.x = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[i]) << 32);
        v.y = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[i + 1]) << 32);
        __builtin_nontemporal_store(v, out128 + p);
      }
      if ((body & 1u) && threadIdx.x == SCAN_THREADS - 1)
        __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[tile_total - 1]) << 32),
                                    out64 + tile_total - 1);
    } else {
      uint32_t* out = static_cast<uint32_t*>(out_any) + run;
      for (uint32_t i = threadIdx.x; i < tile_total; i += SCAN_THREADS) out[i] = s_stage[i];
    }
    run += tile_total;
    __syncthreads();  // s_stage is refilled by the next tile
  }
}

// One pass: a segment's count is chained to its predecessors in the chunk by a decoupled look-back. For chunks of any
// number of segments (the two-pass kernels below take chunks of at most SCAN_TWO_PASS_SEGS segments).
template <typename E, int MODE, bool OUT_ROWID, typename V = E, int SEG = seg_tiles<E>()>
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(sizeof(E) == 1 && SEG <= 4 ? 8 : 1)))
void scan_kernel(ScanLaunchDesc d, ScanConst<V> constant, void* __restrict__ out_any, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_stage[SCAN_TILE];
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  __shared__ uint64_t s_tile;
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_prefix;

  if (threadIdx.x == 0) {
    const uint64_t tile = atomicAdd(d.ticket, 1u);
    s_tile = tile;
    s_chunk = tile < d.n_tiles ? d.tile_chunk[tile] : 0u;
  }
  __syncthreads();
  const uint64_t tile = s_tile;
  if (tile >= d.n_tiles) return;
  const uint32_t c = s_chunk;
  const hy_scan_chunk ch = d.chunks[c];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  // (for this kernel d.chunk_tile_begin / d.tile_chunk / d.n_tiles / d.status count segments of SEG tiles)
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - first_tile) * (SEG * SCAN_TILE);

  // One workgroup = one segment of SEG consecutive tiles of this chunk: the per-lane 16-bit match masks stay in
  // registers, the segment's count is chained to its predecessors by one decoupled look-back, and the tiles' offsets
  // are then compacted tile by tile through LDS into coalesced stores.
  uint32_t masks[SEG];
  segment_masks<E, MODE, V, SEG>(ch, tile_row0, constant, masks);
  uint32_t mine = 0;
#pragma unroll
  for (int t = 0; t < SEG; ++t) mine += __popc(masks[t]);
  uint32_t seg_total;
  block_exclusive_sum<SCAN_THREADS>(mine, s_scratch, &seg_total);

  // Decoupled look-back across the segments of this chunk (wave 0, 64 predecessors per poll).
  if (threadIdx.x < WAVE) {
    uint64_t prefix = 0;
    if (tile == first_tile) {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, seg_total);
    } else {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_AGG, seg_total);
      prefix = lb_lookback_wave(d.status, first_tile, tile, d.error);
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, prefix + seg_total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      const uint64_t last_tile = d.chunk_tile_begin[c + 1] - 1;
      if (tile == last_tile) counts[d.chunk_index[c]] = static_cast<uint32_t>(prefix + seg_total);
    }
  }
  __syncthreads();
  segment_store<OUT_ROWID, SEG>(masks, tile_row0, ch.column.size, ch.out_begin + s_prefix,
                                OUT_ROWID ? d.chunk_ids[c] : 0u, out_any, s_stage, s_scratch);
}

// Two passes (round 6): scan_count_kernel evaluates the predicate over every segment, writes the lanes' match masks
// (2 bytes per 16 rows: 1/8 of the u8 ids) and the segment's count (d.status, one 32-bit count per segment);
// scan_write_kernel then reads only the masks - not the column - takes its output position from the counts of the
// segments before it in its chunk (at most SCAN_TWO_PASS_SEGS - 1, summed by one wave) and stores the RowIDs. No ticket,
// no look-back: every workgroup stores as soon as its masks are back. The look-back's chain of cross-XCD flag
// hand-offs cost more than the second pass (config 2: one pass 0.101 ms; count 0.016 + write 0.064 ms re-reading the
// ids, tools/scan_probe.hip and profiles/r06_scan_*).
constexpr uint32_t SCAN_TWO_PASS_SEGS = 64;

template <typename E, int MODE, typename V = E, int SEG = seg_tiles<E>()>
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(sizeof(E) == 1 && SEG <= 4 ? 8 : 1)))
void scan_count_kernel(ScanLaunchDesc d, ScanConst<V> constant) {
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  const uint64_t tile = blockIdx.x;
  const uint32_t c = d.tile_chunk[tile];
  const hy_scan_chunk ch = d.chunks[c];
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * (SEG * SCAN_TILE);
  uint32_t masks[SEG];
  segment_masks<E, MODE, V, SEG>(ch, tile_row0, constant, masks);
  uint32_t mine = 0;
#pragma unroll
  for (int t = 0; t < SEG; ++t) mine += __popc(masks[t]);
  constexpr int MW = mask_words(SEG);
  uint32_t* mw = d.masks + tile * (MW * SCAN_THREADS) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < MW; ++k)
    __builtin_nontemporal_store(masks[2 * k] | (2 * k + 1 < SEG ? masks[2 * k + 1] << 16 : 0u), mw + k * SCAN_THREADS);
  // one wave sum per wave, one LDS word each, one store
  mine = wave_inclusive_sum(mine);
  if (__lane_id() == WAVE - 1) s_scratch[threadIdx.x / WAVE] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t total = 0;
#pragma unroll
    for (int w = 0; w < SCAN_THREADS / WAVE; ++w) total += s_scratch[w];
    reinterpret_cast<uint32_t*>(d.status)[tile] = total;
  }
}

template <bool OUT_ROWID, int SEG>
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(SEG <= 4 ? 8 : 1)))
void scan_write_kernel(ScanLaunchDesc d, void* __restrict__ out_any, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_stage[SCAN_TILE];
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  __shared__ uint32_t s_prefix;
  const uint64_t tile = blockIdx.x;
  const uint32_t c = d.tile_chunk[tile];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - first_tile) * (SEG * SCAN_TILE);
  constexpr int MW = mask_words(SEG);
  uint32_t masks[SEG];
  {
    const uint32_t* mw = d.masks + tile * (MW * SCAN_THREADS) + threadIdx.x;
    uint32_t w[MW];
#pragma unroll
    for (int k = 0; k < MW; ++k) w[k] = __builtin_nontemporal_load(mw + k * SCAN_THREADS);
#pragma unroll
    for (int t = 0; t < SEG; ++t) masks[t] = (w[t / 2] >> (16 * (t & 1))) & 0xFFFFu;
  }
  if (threadIdx.x < WAVE) {
    const uint32_t* seg_count = reinterpret_cast<const uint32_t*>(d.status);
    const uint64_t before = tile - first_tile;  // < SCAN_TWO_PASS_SEGS (the host's condition for this kernel)
    uint32_t p = threadIdx.x < before ? seg_count[first_tile + threadIdx.x] : 0u;
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if (threadIdx.x == 0) {
      s_prefix = p;
      if (tile + 1 == d.chunk_tile_begin[c + 1]) counts[d.chunk_index[c]] = p + seg_count[tile];
    }
  }
  __syncthreads();
  const hy_scan_chunk& ch = d.chunks[c];
  segment_store<OUT_ROWID, SEG>(masks, tile_row0, ch.column.size, ch.out_begin + s_prefix,
                                OUT_ROWID ? d.chunk_ids[c] : 0u, out_any, s_stage, s_scratch);
}

// ------------------------------------------------------------------------------------------------------------
// Reference-column scan: for each PosList position, gather the referenced value through the referenced chunk's
// descriptor and compare; emit matching positions in PosList order.
// ------------------------------------------------------------------------------------------------------------
struct RefScanDesc {
  const hy_row_id* pos_list;
  uint64_t n;
  const hy_scan_chunk* chunks;  // referenced chunks, indexed by chunk id
  uint32_t n_chunks;
  uint64_t n_tiles;
  uint64_t* status;
  uint32_t* ticket;
  uint32_t* error;
};

template <typename T>
__device__ __forceinline__ bool ref_match(const hy_scan_chunk& ch, uint32_t off, T constant) {
  if (ch.op == HY_OP_NONE) return false;
  if (ch.column.kind == HY_COL_DICT) {
    uint32_t vid;
    if (ch.column.vid_width == 1)
      vid = reinterpret_cast<const uint8_t*>(ch.column.data)[off];
    else if (ch.column.vid_width == 2)
      vid = reinterpret_cast<const uint16_t*>(ch.column.data)[off];
    else
      vid = reinterpret_cast<const uint32_t*>(ch.column.data)[off];
    if (ch.op == HY_OP_IS_NULL) return vid == ch.column.dictionary_size;
    if (vid == ch.column.dictionary_size) return false;
    if (ch.op == HY_OP_VID_SET) return (ch.vid_set[vid >> 5] >> (vid & 31)) & 1u;
    return cmp_op<uint32_t>(ch.op, vid, ch.search_vid);
  }
  if (ch.column.kind == HY_COL_RLE) {  // the row's run: the first with end_position >= off (run_length_column.cpp:24-36)
    const uint32_t* ends = static_cast<const uint32_t*>(ch.column.dictionary);
    uint32_t lo = 0, hi = ch.column.dictionary_size - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ends[mid] < off)
        lo = mid + 1;
      else
        hi = mid;
    }
    const bool run_null = ch.column.nulls != nullptr && ch.column.nulls[lo];
    if (ch.op == HY_OP_IS_NULL) return run_null;
    if (run_null) return false;
    return cmp_op<T>(ch.op, reinterpret_cast<const T*>(ch.column.data)[lo], constant);
  }
  const bool is_null = ch.column.nulls != nullptr && ch.column.nulls[off];
  if (ch.op == HY_OP_IS_NULL) return is_null;
  if (is_null) return false;
  if (ch.column.kind == HY_COL_FOR) {
    const uint32_t o = ch.column.vid_width == 1   ? reinterpret_cast<const uint8_t*>(ch.column.data)[off]
                       : ch.column.vid_width == 2 ? reinterpret_cast<const uint16_t*>(ch.column.data)[off]
                                                  : reinterpret_cast<const uint32_t*>(ch.column.data)[off];
    if constexpr (std::is_integral_v<T>)
      return cmp_op<T>(ch.op, static_cast<T>(static_cast<const T*>(ch.column.dictionary)[off >> 11] + static_cast<T>(o)),
                       constant);
    else
      return false;  // FrameOfReference holds int32 / int64 only
  }
  const T v = reinterpret_cast<const T*>(ch.column.data)[off];
  return cmp_op<T>(ch.op, v, constant);
}

// NULL_ROWS: select the NULL RowIDs of the PosList instead (hy_pos_list_null_positions).
template <typename T, bool NULL_ROWS = false>
__global__ __launch_bounds__(SCAN_THREADS) void ref_scan_kernel(RefScanDesc d, ScanConst<T> constant,
                                                               uint32_t* __restrict__ out_positions,
                                                               uint64_t* __restrict__ count) {
  __shared__ uint32_t s_stage[SCAN_TILE];
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  __shared__ uint64_t s_tile;
  __shared__ uint64_t s_prefix;
  if (threadIdx.x == 0) s_tile = atomicAdd(d.ticket, 1u);
  __syncthreads();
  const uint64_t tile = s_tile;
  if (tile >= d.n_tiles) return;
  const uint64_t row0 = tile * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;

  uint32_t mask = 0;
#pragma unroll 4
  for (int i = 0; i < SCAN_ROWS_PER_THREAD; ++i) {
    const uint64_t r = row0 + i;
    if (r < d.n) {
      const hy_row_id rid = d.pos_list[r];
      if constexpr (NULL_ROWS) {
        if (rid.chunk_offset == 0xFFFFFFFFu) mask |= 1u << i;  // RowID::is_null (types.hpp)
      } else if (rid.chunk_offset != 0xFFFFFFFFu && rid.chunk_id < d.n_chunks) {
        const hy_scan_chunk& ch = d.chunks[rid.chunk_id];
        if (ref_match<T>(ch, rid.chunk_offset, constant.value)) mask |= 1u << i;
      }
    }
  }

  uint32_t tile_total;
  const uint32_t local = block_exclusive_sum<SCAN_THREADS>(__popc(mask), s_scratch, &tile_total);
  if (threadIdx.x < WAVE) {
    uint64_t prefix = 0;
    if (tile == 0) {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, tile_total);
    } else {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_AGG, tile_total);
      prefix = lb_lookback_wave(d.status, 0, tile, d.error);
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, prefix + tile_total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == d.n_tiles - 1) *count = prefix + tile_total;
    }
  }
  uint32_t pos = local;
  uint32_t m = mask;
  while (m) {
    const int i = __builtin_ctz(m);
    m &= m - 1;
    s_stage[pos++] = static_cast<uint32_t>(row0 + i);
  }
  __syncthreads();
  uint32_t* out = out_positions + s_prefix;
  for (uint32_t i = threadIdx.x; i < tile_total; i += SCAN_THREADS) out[i] = s_stage[i];
}

// ------------------------------------------------------------------------------------------------------------
// RunLength chunks scanned per run. Runs of all RLE chunks of one call are numbered globally (run g of chunk k =
// run g - run_begin[k] of that chunk); a run matches as a whole (one value, one NULL flag), so the scan's output is
// the concatenation of the matching runs' row ranges, in order.
// ------------------------------------------------------------------------------------------------------------
struct RleDesc {
  const hy_scan_chunk* chunks;
  const uint64_t* run_begin;  // n_chunks + 1
  const uint32_t* run_chunk;  // n_runs
  uint64_t n_runs;
  uint32_t n_chunks;
};

__device__ __forceinline__ uint32_t rle_run_start(const hy_scan_chunk& ch, uint32_t r) {
  return r == 0 ? 0u : static_cast<const uint32_t*>(ch.column.dictionary)[r - 1] + 1u;
}

// match_len[g] = rows of run g if it matches, else 0 (match_len[n_runs] = 0 so that an exclusive scan of n_runs + 1
// entries also yields the total)
template <typename T>
__global__ __launch_bounds__(SCAN_THREADS) void rle_match_kernel(RleDesc d, ScanConst<T> constant,
                                                                uint32_t* __restrict__ match_len) {
  for (uint64_t g = blockIdx.x * (uint64_t)SCAN_THREADS + threadIdx.x; g <= d.n_runs;
       g += (uint64_t)gridDim.x * SCAN_THREADS) {
    if (g == d.n_runs) {
      match_len[g] = 0;
      continue;
    }
    const uint32_t k = d.run_chunk[g];
    const hy_scan_chunk& ch = d.chunks[k];
    const uint32_t r = static_cast<uint32_t>(g - d.run_begin[k]);
    const uint32_t end = static_cast<const uint32_t*>(ch.column.dictionary)[r];
    const uint32_t len = end - rle_run_start(ch, r) + 1u;
    const bool null_run = ch.column.nulls != nullptr && ch.column.nulls[r];
    bool m;
    if (ch.op == HY_OP_NONE)
      m = false;
    else if (ch.op == HY_OP_IS_NULL)
      m = null_run;
    else
      m = !null_run && cmp_op<T>(ch.op, static_cast<const T*>(ch.column.data)[r], constant.value);
    match_len[g] = m ? len : 0u;
  }
}

__global__ void rle_counts_kernel(RleDesc d, const uint64_t* __restrict__ prefix,
                                  const uint32_t* __restrict__ chunk_index, uint32_t* __restrict__ counts) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < d.n_chunks; k += gridDim.x * blockDim.x)
    counts[chunk_index[k]] = static_cast<uint32_t>(prefix[d.run_begin[k + 1]] - prefix[d.run_begin[k]]);
}

// Output j (of `total` matching rows): its run is the last g with prefix[g] <= j (a run with rows left, since empty
// runs repeat the prefix); coalesced stores, one binary search per output over the L2-resident prefix.
template <bool OUT_ROWID>
__global__ __launch_bounds__(SCAN_THREADS) void rle_expand_kernel(RleDesc d, const uint64_t* __restrict__ prefix,
                                                                 uint64_t total, const uint32_t* __restrict__ chunk_ids,
                                                                 void* __restrict__ out_any) {
  for (uint64_t j = blockIdx.x * (uint64_t)SCAN_THREADS + threadIdx.x; j < total;
       j += (uint64_t)gridDim.x * SCAN_THREADS) {
    uint64_t lo = 0, hi = d.n_runs;  // prefix[lo] <= j < prefix[hi]
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (prefix[mid] <= j)
        lo = mid;
      else
        hi = mid;
    }
    const uint64_t g = lo;
    const uint32_t k = d.run_chunk[g];
    const hy_scan_chunk& ch = d.chunks[k];
    const uint32_t r = static_cast<uint32_t>(g - d.run_begin[k]);
    const uint32_t offset = rle_run_start(ch, r) + static_cast<uint32_t>(j - prefix[g]);
    const uint64_t slot = ch.out_begin + (j - prefix[d.run_begin[k]]);
    if constexpr (OUT_ROWID)
      static_cast<hy_row_id*>(out_any)[slot] = hy_row_id{chunk_ids[k], offset};
    else
      static_cast<uint32_t*>(out_any)[slot] = offset;
  }
}

__global__ void gather_row_ids_kernel(const hy_row_id* __restrict__ pos_list, const uint32_t* __restrict__ positions,
                                      uint64_t n, hy_row_id* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = pos_list[positions[i]];
}

__global__ void first_seen_kernel(const hy_row_id* __restrict__ pos_list, uint64_t n, uint32_t n_chunks,
                                  unsigned long long* __restrict__ first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const hy_row_id r = pos_list[i];
    if (r.chunk_offset != 0xFFFFFFFFu && r.chunk_id < n_chunks) atomicMin(&first[r.chunk_id], (unsigned long long)i);
  }
}

__global__ void expand_row_ids_kernel(uint32_t chunk_id, const uint32_t* __restrict__ offsets, uint64_t n,
                                      hy_row_id* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = hy_row_id{chunk_id, offsets[i]};
}

// Matches per chunk of a dictionary predicate, counted only (no output): workgroup c counts chunk c (its rows' value
// ids in 16-element vector loads, as scan_kernel reads them). The row count a consumer needs before a deferred scan
// runs inside its join (the reference's swap rule compares the inputs' row counts, join_hash.cpp:55-76).
template <typename E>
__global__ __launch_bounds__(256) void scan_count_kernel(const hy_scan_chunk* __restrict__ chunks,
                                                         uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const hy_scan_chunk ch = chunks[blockIdx.x];
  const E* base = static_cast<const E*>(ch.column.data);
  const u32x4 no_nulls{0u, 0u, 0u, 0u};
  const ScanConst<E> unused{};
  uint32_t n = 0;
  for (uint32_t row0 = threadIdx.x * 16u; row0 < ch.column.size; row0 += 256u * 16u) {
    E v[16];
    load16(base, row0, v);
    n += static_cast<uint32_t>(__popc(match_mask<E, MODE_DICT, E>(ch, row0, v, no_nulls, unused)));
  }
  if (n) atomicAdd(&s_n, n);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = s_n;
}

// Every chunk's offset list at once (a fused TableScan's output, hy_scan_join_hash's out_offsets / out_chunk_begin):
// workgroup c expands chunk c's range [chunk_begin[c], chunk_begin[c + 1]) with chunk id chunk_ids[c] (c when null).
__global__ __launch_bounds__(256) void expand_chunk_row_ids_kernel(const uint32_t* __restrict__ offsets,
                                                                   const uint64_t* __restrict__ chunk_begin,
                                                                   const uint32_t* __restrict__ chunk_ids,
                                                                   hy_row_id* __restrict__ out) {
  const uint32_t c = blockIdx.x;
  const uint64_t b = chunk_begin[c], e = chunk_begin[c + 1];
  const uint32_t id = chunk_ids ? chunk_ids[c] : c;
  for (uint64_t i = b + threadIdx.x; i < e; i += 256) out[i] = hy_row_id{id, offsets[i]};
}

}  // namespace hyk
