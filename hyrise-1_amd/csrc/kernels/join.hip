// JoinHash kernels for gfx950: radix partitioning + per-partition LDS hash build/probe.
//
// The reference (src/lib/operators/join_hash.cpp) materializes {RowID, murmur2(v, 17), v} per row
// (materialize_input, :203-285), partitions both sides by hash & (2^b - 1) with a stable, partition-major /
// chunk-minor scatter (partition_radix_parallel, :287-355), builds one std::unordered_map per partition (build,
// :127-185) and probes it partition by partition (probe / probe_semi_anti, :362-527). Its output order is therefore:
// partition ascending, then probe rows in (chunk, offset) order, then build matches in (chunk, offset) order.
//
// This file reproduces that order exactly with an MI355X-shaped pipeline:
//   pass 1  part1_hist / part1_scatter : read the join column straight from its chunks (value, dictionary, or
//           through a PosList), murmur2-hash, stable scatter of 8-byte {key, payload} records by the HIGH digit of
//           the partition id (up to 8 bits, 256 buckets). 4096-row tiles; a per-wave match-any ranking (LDS lane
//           masks) keeps the scatter stable; tiles are mapped to XCDs in contiguous ranges so neighbouring tiles'
//           shared output lines are completed in one L2.
//   pass 2  part2_hist / part2_scatter : inside every high-digit bucket, stable scatter by the LOW 8 bits. After
//           pass 2 every radix partition is contiguous and in row order (MSD, so partition bounds fall out of the
//           pass-2 histogram).
//   join    join_partition : one workgroup per partition. The build partition (~1-2k rows with the reference's
//           radix-bit formula) is hashed into LDS; probe records are matched from registers, counted, and written
//           once one atomic add on the running total has reserved the partition's output range (partitions are
//           located by their begin / count, so no workgroup waits on another).
// Roofline: HBM. Partition passes move 8 B/row per read or write; the join reads 8 B/row (6 B for int32 keys with
// b >= 16 radix bits, whose last pass keeps 16 hash bits instead of the key: HashSrc) and writes 16 B/pair.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int PART_THREADS = 256;
constexpr int PART_WAVES = PART_THREADS / WAVE;
constexpr int PART_ITEMS = 16;                              // items per lane per tile
constexpr int PART_TILE = PART_THREADS * PART_ITEMS;        // 4096 rows per tile
constexpr int WAVE_SPAN = WAVE * PART_ITEMS;                // 1024 consecutive rows per wave
// A partition workgroup handles one SPAN of `sub` consecutive tiles (a per-pass launch parameter), one after the
// other, carrying each digit's output position from tile to tile in a register; histograms and their scans are per
// span. Measured on MI355X (SF100 bench): with the XCD-aware tile map (xcd_tile) one tile per span is fastest - a
// workgroup working through several tiles in sequence keeps fewer loads in flight than several workgroups do - so
// the host default is sub = 1 (HY_PART_SUB1 / HY_PART_SUB2 override it).
constexpr int PART_SUB_MAX = 16;
constexpr uint32_t NULL_PAYLOAD = 0xFFFFFFFFu;

// Partition record: join key (hashed type) + payload. Single-GPU payload = 32-bit row index in the side's row space
// (8 B records for 4-byte keys); exchange records of the distributed join carry the row's global RowID (16 B).
template <typename H, typename P = uint32_t>
struct __attribute__((aligned(sizeof(H) == 8 || sizeof(P) == 8 ? 16 : 8))) Rec {
  H key;
  P payload;
};

// Column chunk of one join side as the device sees it.
struct SrcChunk {
  const void* data;
  const uint8_t* nulls;
  const void* dictionary;
  const hy_row_id* pos_list;  // reference chunk when != nullptr
  uint32_t single_chunk;      // reference chunk: the only referenced chunk (index into Side::referenced), or HY_MIXED_CHUNKS
  uint32_t chunk_id;          // chunk id written into RowID payloads (distributed join: global chunk id)
  uint32_t size;
  uint32_t dictionary_size;
  int32_t kind;
  int32_t vid_width;
  uint64_t row_begin;         // first row of this chunk in the side's row space
  uint32_t ref_offset;        // reference chunk: index in Side::referenced of its table's first chunk (several
                              // referenced tables are concatenated there)
};

// Maps a 32-bit global row index of some table to its RowID.
struct RowMap {
  const uint64_t* row_begin;  // n_chunks + 1
  uint32_t n_chunks;
  uint32_t uniform;           // chunk size if every chunk but the last has it, else 0
  uint64_t magic;             // floor(2^64 / uniform) + 1 (uniform >= 2)
};

// A join output RowID: a streaming store (the pairs are read by later operators, not by the join).
__device__ __forceinline__ void put_row(hy_row_id* p, hy_row_id v) {
  __builtin_nontemporal_store(static_cast<uint64_t>(v.chunk_id) | (static_cast<uint64_t>(v.chunk_offset) << 32),
                              reinterpret_cast<uint64_t*>(p));
}

__device__ __forceinline__ hy_row_id map_row(const RowMap& m, uint32_t idx) {
  if (idx == NULL_PAYLOAD) return hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu};
  if (m.uniform == 1) return hy_row_id{idx, 0u};
  if (m.uniform != 0) {
    const uint32_t q = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(idx), m.magic));
    return hy_row_id{q, idx - q * m.uniform};
  }
  uint32_t lo = 0, hi = m.n_chunks;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (m.row_begin[mid] <= idx)
      lo = mid;
    else
      hi = mid;
  }
  return hy_row_id{lo, static_cast<uint32_t>(idx - m.row_begin[lo])};
}

// RowID payloads (exchange records) already are the output RowIDs.
__device__ __forceinline__ hy_row_id map_row(const RowMap&, hy_row_id rid) { return rid; }

// Payload of row `off` of chunk c itself, and of a referenced row (fused dereference).
template <typename P>
__device__ __forceinline__ P own_payload(uint64_t row_begin, uint32_t chunk_id, uint32_t off) {
  if constexpr (std::is_same_v<P, hy_row_id>)
    return hy_row_id{chunk_id, off};
  else
    return static_cast<uint32_t>(row_begin + off);
}
template <typename P>
__device__ __forceinline__ P ref_payload(bool has, const hy_row_id& rid, uint64_t ref_row_begin) {
  if constexpr (std::is_same_v<P, hy_row_id>)
    return has ? rid : hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu};
  else
    return has ? static_cast<uint32_t>(ref_row_begin + rid.chunk_offset) : NULL_PAYLOAD;
}

// Which join side a partition kernel works for. Only the kernel's name carries it (its code is the same), so that a
// rocprofv3 kernel trace or counter pass attributes every partition launch to its side from the launch itself:
// hyk::part2_scatter<hyk::OnProbe, ...> is the probe side's.
struct OnBuild { static constexpr const char* name = "build"; };
struct OnProbe { static constexpr const char* name = "probe"; };
struct OnExchange { static constexpr const char* name = "exchange"; };  // a distributed join's pre-exchange pass

struct Side {
  const SrcChunk* chunks;
  uint32_t n_chunks;
  const uint64_t* chunk_tile_begin;  // n_chunks + 1 (pass-1 tiles)
  const uint32_t* tile_chunk;        // n_tiles: chunk of each pass-1 tile
  uint64_t n_tiles;
  const SrcChunk* referenced;        // referenced column chunks (reference sides)
  uint32_t n_referenced;
  const uint64_t* referenced_row_begin;  // for fused dereference payloads
  int32_t fuse_deref;                // payload = row in the referenced table instead of row in this table
  int32_t keep_nulls;
  uint32_t ref_base;                 // RowIDs in PosLists name referenced chunk ref_base + i for Side::referenced[i]
  uint32_t sub;                      // tiles per span
  // Fused TableScan (hy_scan_join_hash): the predicate column's chunk c is filter[c]; a row takes part only if it
  // matches. Matching chunk offsets are written chunk by chunk to scan_out (the scan's output, row order).
  const hy_scan_chunk* filter;       // device, n_chunks entries, or null
  uint64_t filter_const;             // type_cast<T>(constant) bits for VALUE predicate chunks
  int32_t filter_type;               // HY_TYPE_* of VALUE predicate chunks
  uint32_t* scan_out;
  // or (part1_spread only; null elsewhere) the scan's output as RowIDs {c, chunk offset} at the same positions
  hy_row_id* scan_rows;
  // Probe-side prefilter of a selective INNER / SEMI join (null: none) over the build keys: a probe row whose key is
  // certainly absent takes no part - it could produce no output, and dropping it keeps the stable order of the others
  // (the reference's output is unchanged). The fused scan's output still lists it. The filter words are either
  //  - a key-range bitmap (bloom_hdr set and the build keys' range fits range_words words): one bit per key value in
  //    [lo, hi], exact, and read almost in order when the probe keys are clustered (lineitem by l_orderkey), or
  //  - a blocked Bloom filter of bloom_mask + 1 words (one 32-bit word per key, two bits).
  const uint32_t* bloom;
  uint32_t bloom_mask;  // Bloom words - 1 (power of two)
  int32_t bloom_by_hash;  // the filter is keyed by murmur2(key, seed) (bloom_slot_hash; SoA joins) instead of the key
  uint32_t seed;
  const struct FilterHdr* bloom_hdr;  // integer keys of record joins: the build keys' range (filter_range), or null
  uint64_t range_words;               // words reserved for a key-range bitmap
};

// The build keys' range, set by filter_range: lo_c = max of ~ord_key (so that a zeroed header is an empty range),
// hi = max of ord_key.
struct FilterHdr {
  unsigned long long lo_c;
  unsigned long long hi;
};

// Keys as unsigned 64-bit values in the keys' order.
template <typename H>
__device__ __forceinline__ uint64_t ord_key(H k) {
  if constexpr (std::is_signed_v<H>) return static_cast<uint64_t>(static_cast<int64_t>(k)) ^ (1ull << 63);
  else return static_cast<uint64_t>(k);
}

// Words of the key-range bitmap for the header's range, or 0 when it does not fit range_words (or the build side
// is empty): then the filter is the Bloom filter.
__device__ __forceinline__ uint64_t range_bitmap_words(const FilterHdr* h, uint64_t range_words, uint64_t* lo) {
  const uint64_t l = ~h->lo_c, hi = h->hi;
  *lo = l;
  if (hi < l || ((hi - l) >> 5) >= range_words) return 0;
  return ((hi - l) >> 5) + 1;
}

// Bloom filter words: one 32-bit word per key selected by a hash independent of the partition and bucket hashes,
// two bits set in it.
template <typename H>
__device__ __forceinline__ uint2 bloom_slot(H key, uint32_t mask) {
  uint64_t b = 0;
  H k = key;
  if constexpr (std::is_floating_point_v<H>) {
    if (k == H(0)) k = H(0);  // -0.0 and 0.0 are equal keys
  }
  __builtin_memcpy(&b, &k, sizeof(H));
  const uint64_t h = (b ^ 0x9E3779B97F4A7C15ull) * 0xD6E8FEB86659FD93ull;
  const uint32_t hi = static_cast<uint32_t>(h >> 32);
  return make_uint2(static_cast<uint32_t>(h) & mask, (1u << (hi & 31u)) | (1u << ((hi >> 5) & 31u)));
}

// The same words and bits from the key's murmur2 hash (a join whose build records keep hashes instead of keys).
__device__ __forceinline__ uint2 bloom_slot_hash(uint32_t h, uint32_t mask) {
  const uint64_t x = (static_cast<uint64_t>(h) ^ 0x9E3779B97F4A7C15ull) * 0xD6E8FEB86659FD93ull;
  const uint32_t hi = static_cast<uint32_t>(x >> 32);
  return make_uint2(static_cast<uint32_t>(x) & mask, (1u << (hi & 31u)) | (1u << ((hi >> 5) & 31u)));
}

template <typename H>
__device__ __forceinline__ uint32_t bloom_filter_act(const Side& s, const H (&keys)[PART_ITEMS], uint32_t act) {
  if (s.bloom == nullptr) return act;
  if constexpr (std::is_integral_v<H>) {
    uint64_t lo;
    if (s.bloom_hdr != nullptr && range_bitmap_words(s.bloom_hdr, s.range_words, &lo) != 0) {  // (uniform)
      const uint64_t span = s.bloom_hdr->hi - lo;
      uint32_t words[PART_ITEMS];
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {  // all loads in flight before any test
        const uint64_t d = ord_key(keys[k]) - lo;
        words[k] = (((act >> k) & 1u) && d <= span) ? s.bloom[d >> 5] : 0u;
      }
      // (the bit recomputed from the key rather than held beside the word: part1_compact's prefiltered instance
      // 110 -> 92 VGPRs, 4 -> 5 waves per SIMD)
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k)
        if (((words[k] >> ((ord_key(keys[k]) - lo) & 31u)) & 1u) == 0u) act &= ~(1u << k);
      return act;
    }
  }
  uint32_t words[PART_ITEMS];
  uint32_t bits[PART_ITEMS];
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) {  // all loads in flight before any test
    const uint2 sl = s.bloom_by_hash ? bloom_slot_hash(murmur2<H>(keys[k], s.seed), s.bloom_mask)
                                     : bloom_slot<H>(keys[k], s.bloom_mask);
    bits[k] = sl.y;
    words[k] = ((act >> k) & 1u) ? s.bloom[sl.x] : sl.y;
  }
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k)
    if ((words[k] & bits[k]) != bits[k]) act &= ~(1u << k);
  return act;
}

// The prefilter of a record join, from the build side's records, in three launches: the keys' range (one atomic
// pair per workgroup into a zeroed header), the filter words zeroed (the bitmap's or the Bloom filter's), the keys'
// bits set.
template <typename H>
static __global__ __launch_bounds__(256) void filter_range(const Rec<H, uint32_t>* __restrict__ recs,
                                                           const uint64_t* __restrict__ n, FilterHdr* __restrict__ hdr) {
  __shared__ unsigned long long s_red[2][256 / WAVE];
  const uint64_t total = *n;
  unsigned long long lo_c = 0, hi = 0;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t u = ord_key(recs[i].key);
    lo_c = max(lo_c, static_cast<unsigned long long>(~u));
    hi = max(hi, static_cast<unsigned long long>(u));
  }
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1) {
    lo_c = max(lo_c, static_cast<unsigned long long>(__shfl_xor(lo_c, dd, WAVE)));
    hi = max(hi, static_cast<unsigned long long>(__shfl_xor(hi, dd, WAVE)));
  }
  if (__lane_id() == 0) {
    s_red[0][threadIdx.x / WAVE] = lo_c;
    s_red[1][threadIdx.x / WAVE] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 256 / WAVE; ++w) {
      lo_c = max(lo_c, s_red[0][w]);
      hi = max(hi, s_red[1][w]);
    }
    if (lo_c != 0) atomicMax(&hdr->lo_c, lo_c);  // (no keys: lo_c = hi = 0)
    if (hi != 0) atomicMax(&hdr->hi, hi);
  }
}

template <typename H>
static __global__ void filter_clear(const FilterHdr* __restrict__ hdr, uint32_t* __restrict__ words,
                                    uint64_t range_words, uint64_t bloom_words) {
  uint64_t lo;
  const uint64_t rw = std::is_integral_v<H> ? range_bitmap_words(hdr, range_words, &lo) : 0;
  const uint64_t nw = rw ? rw : bloom_words;
  uint4* w4 = reinterpret_cast<uint4*>(words);  // (16-byte aligned: the words follow a 64-byte header)
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < (nw + 3) / 4; i += stride)
    w4[i] = make_uint4(0u, 0u, 0u, 0u);
}

template <typename H>
static __global__ void filter_set(const Rec<H, uint32_t>* __restrict__ recs, const uint64_t* __restrict__ n,
                                  const FilterHdr* __restrict__ hdr, uint32_t* __restrict__ words,
                                  uint64_t range_words, uint32_t mask) {
  const uint64_t total = *n;
  uint64_t lo = 0;
  bool range = false;
  if constexpr (std::is_integral_v<H>) range = range_bitmap_words(hdr, range_words, &lo) != 0;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const H key = recs[i].key;
    if (range) {
      if constexpr (std::is_integral_v<H>) {
        const uint64_t d = ord_key(key) - lo;
        atomicOr(words + (d >> 5), 1u << (d & 31u));
      }
    } else {
      const uint2 sl = bloom_slot<H>(key, mask);
      atomicOr(words + sl.x, sl.y);
    }
  }
}

// The same filter words built without a global atomic per key (filter_set's 14.6 M memory-side atomics into a 75 MB
// bitmap took 0.54 ms in TPC-H 3's join 2): the filter is cut into regions of 2^shift words (<= FB_BINS regions, each
// small enough for LDS), and
//   filter_bucket_count   : counts every key's region (one LDS histogram per workgroup; workgroup-major columns of a
//                           region-major matrix, as the radix passes' histograms),
//   exclusive scan        : over regions x workgroups (length read on the device: the region count follows the
//                           build keys' range),
//   filter_bucket_scatter : writes each key's item - word within its region and its bit(s) - into its region's slice,
//   filter_bucket_set     : one workgroup per region ORs its items into an LDS copy of the region and writes the region
//                           out whole (this also clears the words no key sets: no filter_clear).
// An item: word in region (bits 0-15), first bit (16-20), second bit (21-25; the Bloom filter's pair, the bitmap repeats
// its single bit).
constexpr uint32_t FB_BINS = 4096;
constexpr uint32_t FB_SHIFT_MIN = 13;  // 8192-word regions at least
constexpr uint32_t FB_SHIFT_MAX = 14;  // 16384 words = 64 KB of LDS at most
constexpr uint32_t FB_THREADS = 1024;
constexpr int FB_UNROLL = 8;

struct FilterGeom {
  uint64_t words;   // filter words (bitmap or Bloom)
  uint64_t lo;      // bitmap: smallest key (ord_key)
  uint32_t shift;   // words per region = 1 << shift
  uint32_t bins;    // regions
  bool range;
};

template <typename H>
__device__ __forceinline__ FilterGeom filter_geom(const FilterHdr* hdr, uint64_t range_words, uint64_t bloom_words) {
  FilterGeom g{};
  uint64_t rw = 0;
  if constexpr (std::is_integral_v<H>) rw = range_bitmap_words(hdr, range_words, &g.lo);
  g.range = rw != 0;
  g.words = rw ? rw : bloom_words;
  g.shift = FB_SHIFT_MIN;
  while (((g.words + (1ull << g.shift) - 1) >> g.shift) > FB_BINS) ++g.shift;  // (host: shift <= FB_SHIFT_MAX)
  g.bins = static_cast<uint32_t>((g.words + (1ull << g.shift) - 1) >> g.shift);
  return g;
}

// (word, item) of a key
template <typename H>
__device__ __forceinline__ uint2 filter_item(const FilterGeom& g, H key, uint32_t mask) {
  uint64_t word;
  uint32_t b1, b2;
  if (g.range) {
    const uint64_t d = ord_key(key) - g.lo;
    word = d >> 5;
    b1 = b2 = static_cast<uint32_t>(d & 31u);
  } else {
    const uint2 sl = bloom_slot<H>(key, mask);
    word = sl.x;
    b1 = static_cast<uint32_t>(__builtin_ctz(sl.y));
    b2 = 31u - static_cast<uint32_t>(__builtin_clz(sl.y));
  }
  const uint32_t in_region = static_cast<uint32_t>(word & ((1ull << g.shift) - 1));
  return make_uint2(static_cast<uint32_t>(word >> g.shift), in_region | (b1 << 16) | (b2 << 21));
}

// Workgroup k takes the keys [k * per, (k + 1) * per) - the same ones in the count and the scatter.
__device__ __forceinline__ void fb_range(uint64_t total, uint64_t* b, uint64_t* e) {
  const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
  *b = min(total, per * blockIdx.x);
  *e = min(total, *b + per);
}

template <typename H>
static __global__ __launch_bounds__(FB_THREADS) void filter_bucket_count(const Rec<H, uint32_t>* __restrict__ recs,
                                                                        const uint64_t* __restrict__ n,
                                                                        const FilterHdr* __restrict__ hdr,
                                                                        uint64_t range_words, uint64_t bloom_words,
                                                                        uint32_t mask, uint32_t* __restrict__ hist,
                                                                        uint64_t* __restrict__ n_bins) {
  __shared__ uint32_t s_cnt[FB_BINS];
  const FilterGeom g = filter_geom<H>(hdr, range_words, bloom_words);
  for (uint32_t i = threadIdx.x; i < g.bins; i += FB_THREADS) s_cnt[i] = 0;
  __syncthreads();
  uint64_t b, e;
  fb_range(*n, &b, &e);
#pragma unroll 1
  for (uint64_t i0 = b + threadIdx.x; i0 < e; i0 += FB_THREADS * FB_UNROLL) {
    H k[FB_UNROLL];
#pragma unroll
    for (int u = 0; u < FB_UNROLL; ++u) k[u] = recs[min(i0 + u * FB_THREADS, e - 1)].key;  // all loads in flight
#pragma unroll
    for (int u = 0; u < FB_UNROLL; ++u)
      if (i0 + u * FB_THREADS < e) atomicAdd(&s_cnt[filter_item<H>(g, k[u], mask).x], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < g.bins; i += FB_THREADS) hist[static_cast<uint64_t>(i) * gridDim.x + blockIdx.x] = s_cnt[i];
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_bins = g.bins;
}

template <typename H>
static __global__ __launch_bounds__(FB_THREADS) void filter_bucket_scatter(const Rec<H, uint32_t>* __restrict__ recs,
                                                                          const uint64_t* __restrict__ n,
                                                                          const FilterHdr* __restrict__ hdr,
                                                                          uint64_t range_words, uint64_t bloom_words,
                                                                          uint32_t mask,
                                                                          const uint32_t* __restrict__ offsets,
                                                                          uint32_t* __restrict__ items) {
  __shared__ uint32_t s_cur[FB_BINS];
  const FilterGeom g = filter_geom<H>(hdr, range_words, bloom_words);
  for (uint32_t i = threadIdx.x; i < g.bins; i += FB_THREADS)
    s_cur[i] = offsets[static_cast<uint64_t>(i) * gridDim.x + blockIdx.x];
  __syncthreads();
  uint64_t b, e;
  fb_range(*n, &b, &e);
#pragma unroll 1
  for (uint64_t i0 = b + threadIdx.x; i0 < e; i0 += FB_THREADS * FB_UNROLL) {
    H k[FB_UNROLL];
#pragma unroll
    for (int u = 0; u < FB_UNROLL; ++u) k[u] = recs[min(i0 + u * FB_THREADS, e - 1)].key;
#pragma unroll
    for (int u = 0; u < FB_UNROLL; ++u)
      if (i0 + u * FB_THREADS < e) {
        const uint2 it = filter_item<H>(g, k[u], mask);
        items[atomicAdd(&s_cur[it.x], 1u)] = it.y;  // (order inside a region does not matter)
      }
  }
}

// Dynamic LDS: (1 << shift) words for the host's largest shift. n_blocks: the count / scatter grid.
template <typename H>
static __global__ __launch_bounds__(FB_THREADS) void filter_bucket_set(const FilterHdr* __restrict__ hdr,
                                                                      uint64_t range_words, uint64_t bloom_words,
                                                                      const uint32_t* __restrict__ offsets,
                                                                      const uint64_t* __restrict__ total,
                                                                      uint32_t n_blocks,
                                                                      const uint32_t* __restrict__ items,
                                                                      uint32_t* __restrict__ words) {
  extern __shared__ uint32_t s_words[];
  const FilterGeom g = filter_geom<H>(hdr, range_words, bloom_words);
  const uint32_t rw = 1u << g.shift;
#pragma unroll 1
  for (uint32_t r = blockIdx.x; r < g.bins; r += gridDim.x) {
    for (uint32_t i = threadIdx.x; i < rw; i += FB_THREADS) s_words[i] = 0;
    __syncthreads();
    const uint32_t b = offsets[static_cast<uint64_t>(r) * n_blocks];
    const uint32_t e = r + 1 < g.bins ? offsets[static_cast<uint64_t>(r + 1) * n_blocks] : static_cast<uint32_t>(*total);
#pragma unroll 1
    for (uint32_t i0 = b + threadIdx.x; i0 < e; i0 += FB_THREADS * FB_UNROLL) {
      uint32_t it[FB_UNROLL];
#pragma unroll
      for (int u = 0; u < FB_UNROLL; ++u) it[u] = items[min(i0 + u * FB_THREADS, e - 1)];
#pragma unroll
      for (int u = 0; u < FB_UNROLL; ++u)
        if (i0 + u * FB_THREADS < e)
          atomicOr(&s_words[it[u] & 0xFFFFu], (1u << ((it[u] >> 16) & 31u)) | (1u << ((it[u] >> 21) & 31u)));
    }
    __syncthreads();
    const uint64_t w0 = static_cast<uint64_t>(r) << g.shift;
    const uint32_t nw = static_cast<uint32_t>(min<uint64_t>(rw, g.words - w0));
    uint4* dst = reinterpret_cast<uint4*>(words + w0);  // (16-byte aligned: regions are >= 8192 words)
    const uint4* src = reinterpret_cast<const uint4*>(s_words);
    for (uint32_t i = threadIdx.x; i < nw / 4; i += FB_THREADS) dst[i] = src[i];
    for (uint32_t i = (nw & ~3u) + threadIdx.x; i < nw; i += FB_THREADS) words[w0 + i] = s_words[i];
    __syncthreads();  // the next region reuses s_words
  }
}

// NULL rows: a ValueColumn read directly yields its stored value (value_column_iterable), a dictionary column and
// any row reached through a ReferenceColumn yield T{} (dictionary_column_iterable.hpp:80,
// reference_column_iterable.hpp:60-86). The value only matters for outer joins, which keep NULL probe rows.
template <typename T>
__device__ __forceinline__ bool read_column_value(const SrcChunk& c, uint32_t off, T* v, bool stored_null_value) {
  if (c.kind == HY_COL_DICT) {
    uint32_t vid;
    if (c.vid_width == 1)
      vid = static_cast<const uint8_t*>(c.data)[off];
    else if (c.vid_width == 2)
      vid = static_cast<const uint16_t*>(c.data)[off];
    else
      vid = static_cast<const uint32_t*>(c.data)[off];
    if (vid >= c.dictionary_size) {
      *v = T{};
      return false;
    }
    *v = static_cast<const T*>(c.dictionary)[vid];
    return true;
  }
  if (c.nulls != nullptr && c.nulls[off]) {
    *v = stored_null_value ? static_cast<const T*>(c.data)[off] : T{};
    return false;
  }
  *v = static_cast<const T*>(c.data)[off];
  return true;
}

// Loads row `off` of chunk `c`: key (cast to the hashed type), payload, validity (NULLs are dropped unless
// keep_nulls, as materialize_input does at join_hash.cpp:253).
template <typename T, typename H, typename P>
__device__ __forceinline__ bool load_row(const Side& s, const SrcChunk& c, uint32_t off, H* key, P* payload) {
  T v;
  bool valid;
  if (c.pos_list != nullptr) {
    const hy_row_id rid = c.pos_list[off];
    if (rid.chunk_offset == 0xFFFFFFFFu) {
      v = T{};
      valid = false;
      *payload = s.fuse_deref ? ref_payload<P>(false, rid, 0) : own_payload<P>(c.row_begin, c.chunk_id, off);
    } else {
      const uint32_t rc = rid.chunk_id - s.ref_base + c.ref_offset;
      valid = read_column_value<T>(s.referenced[rc], rid.chunk_offset, &v, false);
      *payload = s.fuse_deref ? ref_payload<P>(true, rid, s.referenced_row_begin[rc])
                              : own_payload<P>(c.row_begin, c.chunk_id, off);
    }
  } else {
    // a filtered side stands for the scan's output, a reference table: its NULL rows read as T{} like any row reached
    // through a ReferenceColumn (they only matter to outer joins, which partition them by that value)
    valid = read_column_value<T>(c, off, &v, s.filter == nullptr);
    *payload = own_payload<P>(c.row_begin, c.chunk_id, off);
  }
  *key = static_cast<H>(v);
  return valid || s.keep_nulls;
}

// Loads the PART_ITEMS rows of this lane in a wave's span (row base + k * WAVE + lane for item k): keys (cast to the
// hashed type) and payloads; returns the mask of items that take part (valid rows, NULLs only when keep_nulls, as
// materialize_input does at join_hash.cpp:253). A reference chunk whose PosList references a single chunk (known
// from its producer, hy_join_chunk.single_chunk) reads that chunk's descriptor once with scalar loads instead of once
// per lane and row.
// Load paths a side can be specialised for (the host picks one per side; LP_ANY decides per chunk).
constexpr int LP_ANY = 0;    // any mix of value / dictionary / reference chunks, NULLs
constexpr int LP_VALUE = 1;  // every chunk a ValueColumn without NULLs
constexpr int LP_REF1 = 2;   // every chunk a PosList into one ValueColumn chunk without NULLs (single_chunk set)
constexpr int LP_REFM = 3;   // every chunk a PosList; every referenced chunk a non-empty ValueColumn without NULLs

template <typename T, typename H, typename P, int LP = LP_ANY>
__device__ __forceinline__ uint32_t load_items(const Side& s, const SrcChunk& ch, uint32_t base, H (&keys)[PART_ITEMS],
                                               P (&pays)[PART_ITEMS]) {
  uint32_t act = 0;
  // Row offsets are recomputed per tile: hoisting the 16 lane offsets out of a span's tile loop costs registers.
  uint32_t lane0 = __lane_id();
  asm volatile("" : "+v"(lane0));
  base += lane0;
  // Fast paths issue all PART_ITEMS loads of a phase before using any of them (the general per-item path below
  // serialises each item's dependent loads). Their loads are unconditional, from clamped addresses: a load under
  // `if (in range)` becomes its own exec-masked block with a full wait after it, i.e. PART_ITEMS serial round trips.
  // Items outside the chunk are masked out of `act`; their keys and payloads are never used.
  if (LP == LP_VALUE || (LP == LP_ANY && ch.pos_list == nullptr && ch.kind == HY_COL_VALUE && ch.nulls == nullptr)) {
    const T* data = static_cast<const T*>(ch.data);
    const uint32_t last = ch.size - 1;  // a tile exists only for a non-empty chunk
    T v[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) v[k] = data[min(base + k * WAVE, last)];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t off = base + k * WAVE;
      keys[k] = static_cast<H>(v[k]);
      pays[k] = own_payload<P>(ch.row_begin, ch.chunk_id, off);
      if (off < ch.size) act |= 1u << k;
    }
    return act;
  }
  if (LP == LP_REF1 || (LP == LP_ANY && ch.pos_list != nullptr && ch.single_chunk != HY_MIXED_CHUNKS)) {
    const SrcChunk rc = s.referenced[ch.single_chunk];
    const uint64_t rrow = s.fuse_deref ? s.referenced_row_begin[ch.single_chunk] : 0;
    const uint32_t last = ch.size - 1;
    hy_row_id rid[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) rid[k] = ch.pos_list[min(base + k * WAVE, last)];
    // LP_REF1 is chosen only for non-empty referenced chunks, so offset 0 is a valid stand-in for NULL rows.
    if (LP == LP_REF1 || (rc.kind == HY_COL_VALUE && rc.nulls == nullptr && rc.size > 0)) {
      const T* data = static_cast<const T*>(rc.data);
      T v[PART_ITEMS];
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) v[k] = data[rid[k].chunk_offset != 0xFFFFFFFFu ? rid[k].chunk_offset : 0u];
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {
        const uint32_t off = base + k * WAVE;
        const bool has = rid[k].chunk_offset != 0xFFFFFFFFu;
        pays[k] = s.fuse_deref ? ref_payload<P>(has, rid[k], rrow) : own_payload<P>(ch.row_begin, ch.chunk_id, off);
        keys[k] = static_cast<H>(v[k]);
        if (off < ch.size && (has || s.keep_nulls)) act |= 1u << k;
      }
      return act;
    }
    if constexpr (LP != LP_ANY) return act;
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t off = base + k * WAVE;
      if (off >= ch.size) continue;
      const hy_row_id rid1 = rid[k];
      const bool has = rid1.chunk_offset != 0xFFFFFFFFu;
      T v = T{};
      const bool valid = has && read_column_value<T>(rc, rid1.chunk_offset, &v, false);
      pays[k] = s.fuse_deref ? ref_payload<P>(has, rid1, rrow) : own_payload<P>(ch.row_begin, ch.chunk_id, off);
      keys[k] = static_cast<H>(v);
      if (valid || s.keep_nulls) act |= 1u << k;
    }
    return act;
  }
  if constexpr (LP == LP_REFM) {
    // PosLists over several value chunks (a join output as the next join's input, TPC-H 3's second build side): the
    // RowIDs, then each row's chunk data pointer, then the values - three phases of PART_ITEMS independent loads
    // instead of one dependent chain per item (the general path below). NULL RowIDs read row 0 of referenced chunk 0
    // (non-empty: load_path) and take part only with keep_nulls.
    const uint32_t last = ch.size - 1;
    hy_row_id rid[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) rid[k] = ch.pos_list[min(base + k * WAVE, last)];
    const T* dp[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool has = rid[k].chunk_offset != 0xFFFFFFFFu;
      dp[k] = static_cast<const T*>(s.referenced[has ? rid[k].chunk_id - s.ref_base + ch.ref_offset : 0u].data);
    }
    T v[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) v[k] = dp[k][rid[k].chunk_offset != 0xFFFFFFFFu ? rid[k].chunk_offset : 0u];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t off = base + k * WAVE;
      const bool has = rid[k].chunk_offset != 0xFFFFFFFFu;
      if (s.fuse_deref) {
        const uint32_t rc = has ? rid[k].chunk_id - s.ref_base + ch.ref_offset : 0u;
        pays[k] = ref_payload<P>(has, rid[k], s.referenced_row_begin[rc]);
      } else {
        pays[k] = own_payload<P>(ch.row_begin, ch.chunk_id, off);
      }
      keys[k] = static_cast<H>(has ? v[k] : T{});
      if (off < ch.size && (has || s.keep_nulls)) act |= 1u << k;
    }
    return act;
  }
  if constexpr (LP == LP_ANY) {
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t off = base + k * WAVE;
      if (off < ch.size && load_row<T, H, P>(s, ch, off, &keys[k], &pays[k])) act |= 1u << k;
    }
  }
  return act;
}

// ------------------------------------------------------------------------------------------------------------
// Fused TableScan predicate (reference SingleColumnTableScanImpl, single_column_table_scan_impl.cpp:38-205, with the
// dictionary rewrite done on the host per chunk): match mask of this lane's PART_ITEMS rows base + k * WAVE + lane of
// predicate chunk f (rows >= f.column.size are 0). Loads are unconditional from clamped rows (see load_items).
// ------------------------------------------------------------------------------------------------------------
template <typename E, bool DICT>
__device__ __forceinline__ uint32_t filter_items_t(const hy_scan_chunk& f, uint32_t base, uint64_t cbits) {
  const E* data = static_cast<const E*>(f.column.data);
  const uint32_t n = f.column.size, last = n - 1;
  E v[PART_ITEMS];
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) v[k] = data[min(base + k * WAVE, last)];
  uint32_t m = 0;
  const int op = f.op;
  if constexpr (DICT) {
    const DictPred pr = dict_pred(op, static_cast<E>(f.search_vid), static_cast<E>(f.column.dictionary_size));
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) m |= static_cast<uint32_t>(dict_match(pr, v[k])) << k;
  } else {
    E c;
    __builtin_memcpy(&c, &cbits, sizeof(E));
    if (f.column.nulls != nullptr) {
      uint8_t nl[PART_ITEMS];
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) nl[k] = f.column.nulls[min(base + k * WAVE, last)];
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) m |= static_cast<uint32_t>(nl[k] == 0 && cmp_op<E>(op, v[k], c)) << k;
    } else {
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) m |= static_cast<uint32_t>(cmp_op<E>(op, v[k], c)) << k;
    }
  }
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k)
    if (base + k * WAVE >= n) m &= ~(1u << k);
  return m;
}

// Filter kinds a side can be specialised for (the host picks one per side from its predicate chunks): every chunk
// dictionary-encoded with 1-, 2- or 4-byte value ids, or anything (value columns of any type, mixed widths).
constexpr int FK_NONE = 0;
constexpr int FK_DICT8 = 1;
constexpr int FK_DICT16 = 2;
constexpr int FK_DICT32 = 3;
constexpr int FK_ANY = 4;

template <int FK>
__device__ __forceinline__ uint32_t filter_items(const Side& s, uint32_t c, uint32_t base) {
  const hy_scan_chunk f = s.filter[c];
  base += __lane_id();
  if (f.op == HY_OP_NONE || f.column.size == 0) return 0u;
  if constexpr (FK == FK_DICT8) return filter_items_t<uint8_t, true>(f, base, 0);
  if constexpr (FK == FK_DICT16) return filter_items_t<uint16_t, true>(f, base, 0);
  if constexpr (FK == FK_DICT32) return filter_items_t<uint32_t, true>(f, base, 0);
  if (f.column.kind == HY_COL_DICT) {
    if (f.column.vid_width == 1) return filter_items_t<uint8_t, true>(f, base, 0);
    if (f.column.vid_width == 2) return filter_items_t<uint16_t, true>(f, base, 0);
    return filter_items_t<uint32_t, true>(f, base, 0);
  }
  switch (s.filter_type) {
    case HY_TYPE_INT32:
      return filter_items_t<int32_t, false>(f, base, s.filter_const);
    case HY_TYPE_INT64:
      return filter_items_t<int64_t, false>(f, base, s.filter_const);
    case HY_TYPE_FLOAT:
      return filter_items_t<float, false>(f, base, s.filter_const);
    default:
      return filter_items_t<double, false>(f, base, s.filter_const);
  }
}

struct Digit {
  uint32_t mask;   // (1 << radix_bits) - 1
  uint32_t shift;  // digit = (hash & mask) >> shift
  uint32_t dmask;  // digit &= dmask
  uint32_t seed;
  // string join keys (hy_join_params.key_hash): int32 keys are ids of distinct strings and key_hash[id] is the
  // string's murmur2 (murmur_hash.hpp:16-20), so partitioning follows the reference's string hashes; else null
  const uint32_t* key_hash;
  // 1: stable ranking by per-bit ballots (wave_rank) instead of one LDS fetch-add per item (wave_rank_add): the
  // fallback for a device whose rank_order_check failed (join_host.hpp check_rank_order), or HY_RANK_BALLOT=1
  uint32_t ballot_rank;
};

// The partitioning hash of a key: murmur2 over its bytes (join_hash.cpp:253), or the precomputed string hash.
template <typename H>
__device__ __forceinline__ uint32_t key_hash_of(const Digit& dg, H key) {
  if constexpr (std::is_same_v<H, int32_t>) {
    if (dg.key_hash != nullptr) return dg.key_hash[static_cast<uint32_t>(key)];
  }
  return murmur2<H>(key, dg.seed);
}

template <typename H>
__device__ __forceinline__ uint32_t digit_of(const Digit& dg, H key) {
  return ((key_hash_of<H>(dg, key) & dg.mask) >> dg.shift) & dg.dmask;
}

// The next pass's digit of each record, written beside the records so that the next histogram reads one byte per
// record instead of the record (and its hash). bytes == null: no next pass.
struct NextDigit {
  uint8_t* bytes;
  uint32_t shift;
  uint32_t dmask;
};

__device__ __forceinline__ uint32_t find_tile_owner(const uint64_t* begin, uint32_t n, uint64_t tile) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (begin[mid] <= tile)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Stable in-tile ranking by digit: wave w owns rows [w*1024, (w+1)*1024) of the tile, lane l handles row
// k*64 + l at step k, so processing steps in order per wave and waves in order reproduces row order.
// Returns rank of the item among the same-digit items of its wave that precede it, and updates the per-wave
// digit counter.
__device__ __forceinline__ uint32_t wave_rank(uint32_t digit, bool active, int dbits, uint32_t* wave_cnt) {
  uint64_t peers = __ballot(active);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b < dbits) {
      const uint64_t bb = __ballot(active && ((digit >> b) & 1u));
      peers &= ((digit >> b) & 1u) ? bb : ~bb;
    }
  }
  uint32_t rank = 0;
  if (active) {
    const uint32_t before = __popcll(peers & lanemask_lt());
    rank = wave_cnt[digit] + before;
  }
  // all lanes read wave_cnt before anyone writes (LDS ops of one wave execute in order)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  if (active) {
    const uint64_t higher = peers & ~(lanemask_lt() | (1ull << __lane_id()));
    if (higher == 0) wave_cnt[digit] += __popcll(peers);
  }
  return rank;
}

// The same ranking without per-bit ballots: each active lane ORs its lane bit into its digit's 64-bit mask in LDS
// and reads the mask back - the set of lanes holding the same digit (a match-any) - then clears it. LDS instructions
// of one wave execute in order, so the read sees every lane's OR and the next item starts from a cleared mask. Three
// LDS operations replace the 8 ballots and ~60 vector instructions per item of wave_rank (the partition passes were
// VALU-bound on them).
__device__ __forceinline__ uint32_t wave_rank_lds(uint32_t digit, bool active, uint64_t* wave_mask, uint32_t* wave_cnt) {
  uint32_t rank = 0;
  if (active) {
    const uint64_t me = 1ull << __lane_id();
    __hip_atomic_fetch_or(&wave_mask[digit], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t peers = __hip_atomic_load(&wave_mask[digit], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&wave_mask[digit], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t c = __hip_atomic_load(&wave_cnt[digit], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    rank = c + static_cast<uint32_t>(__popcll(peers & (me - 1)));
    if ((peers & ~((me << 1) - 1)) == 0)  // highest lane of the group advances the counter
      __hip_atomic_store(&wave_cnt[digit], c + static_cast<uint32_t>(__popcll(peers)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  return rank;
}

// The same stable ranking with ONE returning LDS add per item: gfx950's LDS applies the lanes of an atomic that hit the
// same counter in ascending lane order, and a wave's LDS instructions in program order, so the old value an item's add
// returns is its rank among the wave's same-digit items before it in (item, lane) order, and the counter ends at the
// digit's count (what wave_rank_lds computes with an or / read / clear of the digit's lane mask and a read / advance of
// its counter). Measured on MI355X (tools/rank_probe.hip, profiles/r05_rank_probe_*.jsonl): equal to the stable ranks
// for all of 201 M items in uniform, 4-digit, single-digit and half-active waves; >= 1.8x wave_rank_lds's throughput.
// The property is checked on each device before its first partition launch (rank_order_check, join_host.hpp), and a
// device that breaks it fails the join with HY_ERR_KERNEL instead of producing an unstable order.
__device__ __forceinline__ uint32_t wave_rank_add(uint32_t digit, bool active, uint32_t* wave_cnt) {
  return active ? __hip_atomic_fetch_add(&wave_cnt[digit], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
}

// The stable rank of a partition pass's item: wave_rank_add, or on a device that failed rank_order_check (and under
// HY_RANK_BALLOT=1) the per-bit ballot ranking, which relies on nothing but ballots and one wave's in-order LDS access
// (dg.ballot_rank is a kernel argument: the branch is uniform). Every lane of the wave calls it for every item.
__device__ __forceinline__ uint32_t rank_item(const Digit& dg, uint32_t digit, bool active, uint32_t* wave_cnt) {
  if (dg.ballot_rank) return wave_rank(digit, active, 8, wave_cnt);
  return wave_rank_add(digit, active, wave_cnt);
}

// Self-check of wave_rank_add against wave_rank_lds (one 256-thread workgroup; *bad counts mismatching items): waves
// of uniform, 4-digit, single-digit and half-active items, the collision patterns of skewed keys included.
static __global__ __launch_bounds__(256) void rank_order_check(uint32_t rounds, uint32_t* __restrict__ bad) {
  __shared__ uint32_t s_cnt_a[4][256];
  __shared__ uint32_t s_cnt_m[4][256];
  __shared__ uint64_t s_mask[4][256];
  const int w = threadIdx.x / WAVE, lane = __lane_id();
  uint32_t nbad = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    for (int i = lane; i < 256; i += WAVE) {
      s_cnt_a[w][i] = 0;
      s_cnt_m[w][i] = 0;
      s_mask[w][i] = 0;
    }
    const uint32_t kind = (r * 4 + w) % 6;
    const uint32_t span = kind % 3 == 0 ? 256u : kind % 3 == 1 ? 4u : 1u;
    uint32_t dig[16], ra[16];
    bool act[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t h = murmur2<int32_t>(static_cast<int32_t>((r * 4 + w) * 1024 + k * WAVE + lane), 0x5EEDu);
      dig[k] = (h % span) * (256u / span);
      act[k] = kind < 3 || ((h >> 16) & 1u);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) ra[k] = wave_rank_add(dig[k], act[k], s_cnt_a[w]);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t rm = wave_rank_lds(dig[k], act[k], s_mask[w], s_cnt_m[w]);
      if (act[k] && rm != ra[k]) ++nbad;
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

// Zeroes this wave's 256 digit masks (the wave alone uses them until the next block barrier).
__device__ __forceinline__ void clear_wave_masks(uint64_t* wave_mask) {
#pragma unroll
  for (int i = 0; i < 256 / WAVE; ++i) wave_mask[i * WAVE + __lane_id()] = 0;
}

// LDS-staged scatter of one tile's records. On entry s_cnt[w][d] holds wave w's count of digit d and dr[k] = digit << 24
// | rank of item k among its wave's same-digit items (wave_rank). The tile's records are first placed in LDS in
// (digit, wave, rank) order - the order they take in the output - and then stored from consecutive LDS entries by
// consecutive lanes, so each bucket's run of the tile is written with coalesced stores instead of one scattered 8-byte
// store per lane. Thread d holds run = output position of this tile's first digit-d record and advances it by the
// tile's digit-d count.
static_assert(PART_THREADS >= 256, "one thread per digit");
static_assert(PART_TILE * 8 >= PART_WAVES * 256 * 8, "ranking masks fit the staging area");

// Where a partition pass writes its records: {key, payload} records, or - the last pass of a side whose 4-byte keys
// murmur2 maps one-to-one onto hashes (int32; see HashSrc) - two arrays: the hash bits above the radix bits (16 of
// them when radix_bits >= 16; they identify the key inside its partition) and the payloads, 6 B per record instead of
// 8. A SoA build side of a prefiltered join also sets its Bloom words (by hash, bloom_slot_hash) here.
template <typename H, typename P>
struct RecOut {
  Rec<H, P>* recs;
  uint16_t* hk;         // non-null: SoA output
  P* pay;
  uint32_t hk_shift;    // radix bits
  uint32_t* bloom;      // or null
  uint32_t bloom_mask;  // words - 1
};

template <typename H, typename P>
__device__ __forceinline__ void store_record(const RecOut<H, P>& out, uint32_t o, const Rec<H, P>& r, uint32_t hash) {
  if (out.hk != nullptr) {
    out.hk[o] = static_cast<uint16_t>(hash >> out.hk_shift);
    out.pay[o] = r.payload;
    if (out.bloom != nullptr) {
      const uint2 sl = bloom_slot_hash(hash, out.bloom_mask);
      atomicOr(out.bloom + sl.x, sl.y);
    }
  } else {
    out.recs[o] = r;
  }
}

template <typename H, typename P>
__device__ __forceinline__ void staged_scatter(const Rec<H, P> (&recs)[PART_ITEMS], uint32_t act,
                                               const uint32_t (&dr)[PART_ITEMS], uint32_t (*s_cnt)[256],
                                               uint32_t* s_delta, Rec<H, P>* s_stage, uint32_t* s_scratch,
                                               uint32_t n_digits, const Digit& dg, const NextDigit& nd,
                                               uint32_t& run, Rec<H, P>* __restrict__ out) {
  staged_scatter<H, P>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run,
                       RecOut<H, P>{out, nullptr, nullptr, 0u, nullptr, 0u});
}

template <typename H, typename P>
__device__ __forceinline__ void staged_scatter(const Rec<H, P> (&recs)[PART_ITEMS], uint32_t act,
                                               const uint32_t (&dr)[PART_ITEMS], uint32_t (*s_cnt)[256],
                                               uint32_t* s_delta, Rec<H, P>* s_stage, uint32_t* s_scratch,
                                               uint32_t n_digits, const Digit& dg, const NextDigit& nd,
                                               uint32_t& run, const RecOut<H, P>& out) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  __syncthreads();  // every wave's counts are in s_cnt
  const uint32_t d = threadIdx.x;
  uint32_t tot = 0;
  if (d < n_digits) {
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) {
      const uint32_t t = s_cnt[ww][d];
      s_cnt[ww][d] = tot;
      tot += t;
    }
  }
  uint32_t total;
  const uint32_t loc = block_exclusive_sum<PART_THREADS>(tot, s_scratch, &total);  // tile-local start of digit d
  if (d < n_digits) {
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) s_cnt[ww][d] += loc;
    s_delta[d] = run - loc;
    run += tot;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k)
    if ((act >> k) & 1u) s_stage[s_cnt[w][dr[k] >> 24] + (dr[k] & 0xFFFFFFu)] = recs[k];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += PART_THREADS) {
    const Rec<H, P> r = s_stage[i];
    const uint32_t hash = key_hash_of<H>(dg, r.key);
    const uint32_t h = hash & dg.mask;
    const uint32_t o = i + s_delta[(h >> dg.shift) & dg.dmask];
    store_record<H, P>(out, o, r, hash);
    if (nd.bytes != nullptr) nd.bytes[o] = static_cast<uint8_t>((h >> nd.shift) & nd.dmask);
  }
}

// Zeroes this wave's digit counters (only the wave itself uses its row before the next block barrier).
__device__ __forceinline__ void clear_wave_counts(uint32_t* wave_cnt) {
#pragma unroll
  for (int i = 0; i < 256 / WAVE; ++i) wave_cnt[i * WAVE + __lane_id()] = 0;
}

// ------------------------------------------------------------------------------------------------------------
// Pass 1: from column chunks.
// ------------------------------------------------------------------------------------------------------------
// Histogram rows: hist[d * n_tiles + tile] = rows of span `tile` with digit d.
template <typename SD, typename T, typename H, int LP>
__global__ __launch_bounds__(PART_THREADS) void part1_hist(Side s, Digit dg, uint32_t n_digits,
                                                          uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_hist[256];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  for (int i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  __syncthreads();
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    const uint32_t act =
        bloom_filter_act<H>(s, keys, load_items<T, H, uint32_t, LP>(s, ch, base + j * PART_TILE + w * WAVE_SPAN, keys, pays));
    uint32_t dig[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) dig[k] = digit_of<H>(dg, keys[k]);
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if ((act >> k) & 1u) atomicAdd(&s_hist[dig[k]], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[d * s.n_tiles + tile] = s_hist[d];
}

template <typename SD, typename T, typename H, typename P, int LP>
__global__ __launch_bounds__(PART_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void part1_scatter(
    Side s, Digit dg, NextDigit nd, int dbits, uint32_t n_digits, const uint32_t* __restrict__ offsets,
    RecOut<H, P> out) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ Rec<H, P> s_stage[PART_TILE];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  uint32_t run = threadIdx.x < n_digits ? offsets[threadIdx.x * s.n_tiles + tile] : 0u;

#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    if (j) __syncthreads();  // the previous tile's write-out has read s_stage
    clear_wave_counts(s_cnt[w]);
    H keys[PART_ITEMS];
    P pays[PART_ITEMS];
    uint32_t dr[PART_ITEMS];  // digit << 24 | rank within the wave (rank < WAVE_SPAN)
    const uint32_t act =
        bloom_filter_act<H>(s, keys, load_items<T, H, P, LP>(s, ch, base + j * PART_TILE + w * WAVE_SPAN, keys, pays));
    Rec<H, P> recs[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, keys[k]) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
      recs[k].key = keys[k];
      recs[k].payload = pays[k];
    }
    staged_scatter<H, P>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run, out);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Pass 1 of a side with a fused TableScan, in two streaming kernels (the default; HY_FILTER_COMPACT=0 selects
// part1_mask / part1_spread_mask below, which move 1.9 GB less at SF100 but measured slower: join_host.hpp
// filter_compact_enabled):
//   part1_compact: evaluates the predicate and reads the join column of every row of a span once, writes the span's
//     matching rows as records in row order into the span's own slot of a gapped buffer (slot = span * SPAN
//     records; no prefix across spans is needed), counts them per digit (histogram rows as part1_hist, plus the scan
//     row) and per span (span_count). A matching row whose join key is NULL (and does not take part: no keep_nulls)
//     is still a scan match; its record carries NULL_FLAG in the payload and no digit.
//   part1_spread: reads each span's records back (coalesced), writes the scan's output (chunk offsets, in row order)
//     and scatters the taking-part records by digit exactly as part1_scatter would (stable LDS-staged scatter).
// Without a scan output (scan_out null: the caller wants the join output and the scan's counts only), part1_compact
// writes the records of the rows taking part alone - after a selective prefilter a few percent of the scan's matches
// (TPC-H 3's lineitem side: 6 of 323 M) - and the scan row of the histogram still counts every match.
// Traffic per matched row is one 8-byte record more than the single fused scatter, but both kernels are plain
// streams, while the single kernel's load -> rank -> stage -> store chain per tile left it latency-bound. (Round 5
// measured 6-byte SoA gapped records - key + 16-bit in-span offset - and reverted them: part1_spread 1.27-1.32 ->
// 1.50 ms for the 2 bytes less per match, part1_compact unchanged.)
// ------------------------------------------------------------------------------------------------------------
constexpr uint32_t NULL_FLAG = 0x80000000u;  // payloads of filtered sides are row indexes < 2^31

// PF: the side has a probe-side prefilter (s.bloom). A separate instance: the prefilter's lookups hold registers
// (151 VGPRs, 3 waves per SIMD, against 96 without them) that the headline's unprefiltered probe side does not need.
template <typename SD, typename T, typename H, int LP, int FK, bool PF>
__global__ __launch_bounds__(PART_THREADS) void part1_compact(Side s, Digit dg, uint32_t n_digits,
                                                             uint32_t* __restrict__ hist, uint32_t* __restrict__ span_count,
                                                             Rec<H, uint32_t>* __restrict__ gap_out) {
  __shared__ uint32_t s_hist[257];
  __shared__ uint32_t s_sc[WAVE + 2];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  for (int i = threadIdx.x; i < 257; i += PART_THREADS) s_hist[i] = 0;
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  Rec<H, uint32_t>* out = gap_out + tile * (static_cast<uint64_t>(s.sub) * PART_TILE);
  const bool scan_records = s.scan_out != nullptr;  // records of every scan match, or of the rows taking part only
  uint32_t run = 0;
  if (threadIdx.x == 0) s_sc[WAVE + 1] = 0;  // scan matches of the span (without scan records)
  __syncthreads();
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    const uint32_t m_scan = filter_items<FK>(s, c, rb);
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    uint32_t act = load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m_scan;
    if constexpr (PF) act = bloom_filter_act<H>(s, keys, act);
    const uint32_t m = scan_records ? m_scan : act;  // the rows written as records
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if ((act >> k) & 1u) atomicAdd(&s_hist[digit_of<H>(dg, keys[k])], 1u);
    if (!scan_records) {
      uint32_t nm = 0;
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) nm += static_cast<uint32_t>(__popcll(__ballot((m_scan >> k) & 1u)));
      if (lane == 0 && nm) atomicAdd(&s_sc[WAVE + 1], nm);
    }
    // row-order compaction of the records: (wave, item) ballot counts -> prefix -> lane rank
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint64_t b = __ballot((m >> k) & 1u);
      if (lane == 0) s_sc[w * PART_ITEMS + k] = static_cast<uint32_t>(__popcll(b));
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {
      const uint32_t v = s_sc[threadIdx.x];
      const uint32_t incl = wave_inclusive_sum(v);
      s_sc[threadIdx.x] = incl - v;
      if (threadIdx.x == WAVE - 1) s_sc[WAVE] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint64_t b = __ballot((m >> k) & 1u);
      if ((m >> k) & 1u) {
        Rec<H, uint32_t> r;
        r.key = keys[k];
        r.payload = pays[k] | (((act >> k) & 1u) ? 0u : NULL_FLAG);
        out[run + s_sc[w * PART_ITEMS + k] + static_cast<uint32_t>(__popcll(b & lanemask_lt()))] = r;
      }
    }
    run += s_sc[WAVE];
    __syncthreads();  // s_sc is rewritten by the next tile
  }
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[d * s.n_tiles + tile] = s_hist[d];
  if (threadIdx.x == 0) {
    hist[n_digits * s.n_tiles + tile] = scan_records ? run : s_sc[WAVE + 1];
    span_count[tile] = run;
  }
}

template <typename SD, typename H>
__global__ __launch_bounds__(PART_THREADS) void part1_spread(Side s, Digit dg, NextDigit nd, int dbits,
                                                            uint32_t n_digits, const uint32_t* __restrict__ offsets,
                                                            const uint32_t* __restrict__ span_count,
                                                            const Rec<H, uint32_t>* __restrict__ gap_in,
                                                            RecOut<H, uint32_t> out) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ Rec<H, uint32_t> s_stage[PART_TILE];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  const uint32_t n = span_count[tile];
  const uint32_t c = s.tile_chunk[tile];
  const uint32_t row0 = static_cast<uint32_t>(s.chunks[c].row_begin);  // payload -> chunk offset
  const Rec<H, uint32_t>* in = gap_in + tile * (static_cast<uint64_t>(s.sub) * PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  uint32_t run = threadIdx.x < n_digits ? offsets[threadIdx.x * s.n_tiles + tile] : 0u;
  const uint32_t srun = offsets[n_digits * s.n_tiles + tile] - offsets[n_digits * s.n_tiles];
  const uint32_t n_sub = (n + PART_TILE - 1) / PART_TILE;
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    if (j) __syncthreads();  // the previous tile's write-out has read s_stage
    clear_wave_counts(s_cnt[w]);
    Rec<H, uint32_t> recs[PART_ITEMS];
    uint32_t dr[PART_ITEMS];
    uint32_t act = 0;
    const uint32_t r0 = j * PART_TILE + w * WAVE_SPAN + __lane_id();
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) recs[k] = in[min(r0 + k * WAVE, n - 1)];  // unconditional (see load_items)
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t i = r0 + k * WAVE;
      if (i < n) {
        if (s.scan_rows != nullptr)
          s.scan_rows[srun + i] = hy_row_id{c, (recs[k].payload & ~NULL_FLAG) - row0};
        else if (s.scan_out != nullptr)
          s.scan_out[srun + i] = (recs[k].payload & ~NULL_FLAG) - row0;
        if (!(recs[k].payload & NULL_FLAG)) act |= 1u << k;
      }
    }
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, recs[k].key) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
    }
    staged_scatter<H, uint32_t>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run, out);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Pass 1 of a side with a fused TableScan, without the gapped record round trip (HY_FILTER_COMPACT=0; the default is
// part1_compact / part1_spread above):
//   part1_mask: the predicate and the join column of every row of a span: digit histogram of the rows that take part
//     (+ the span's scan-match count as an extra histogram row) and the scan's match bits - one 64-bit ballot per
//     (tile, wave, item), 1 bit per row. Writes 1/8 B per row instead of an 8-byte record per match.
//   part1_spread_mask: re-reads the span's join column (the predicate column is not read again: its result is the
//     bits), writes the scan output (chunk offsets of the matches, row order) and compacts the rows that take part into
//     LDS in row order; the compacted records are then ranked and scattered by digit in rounds of one tile (stable
//     LDS-staged scatter, as part1_scatter). Per matched row it moves 4 B of key again instead of the 8-byte record
//     written and read back.
// ------------------------------------------------------------------------------------------------------------
constexpr int MASK_WORDS = PART_WAVES * PART_ITEMS;  // ballots per tile

template <typename SD, typename T, typename H, int LP, int FK>
__global__ __launch_bounds__(PART_THREADS) void part1_mask(Side s, Digit dg, uint32_t n_digits,
                                                          uint32_t* __restrict__ hist,
                                                          uint64_t* __restrict__ match_bits) {
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_wc[PART_WAVES];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  for (int i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  uint32_t matches = 0;  // this wave's scan matches in the span (wave-uniform)
  __syncthreads();
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    const uint32_t m = filter_items<FK>(s, c, rb);
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    const uint32_t act = bloom_filter_act<H>(s, keys, load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m);
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if ((act >> k) & 1u) atomicAdd(&s_hist[digit_of<H>(dg, keys[k])], 1u);
    uint64_t mine = 0;  // lane k < PART_ITEMS keeps item k's ballot: one coalesced 128-B store per wave
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint64_t b = __ballot((m >> k) & 1u);
      if (lane == k) mine = b;
      matches += static_cast<uint32_t>(__popcll(b));
    }
    if (lane < PART_ITEMS) match_bits[(tile * s.sub + j) * MASK_WORDS + w * PART_ITEMS + lane] = mine;
  }
  if (lane == 0) s_wc[w] = matches;
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[d * s.n_tiles + tile] = s_hist[d];
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) t += s_wc[ww];
    hist[n_digits * s.n_tiles + tile] = t;
  }
}

// SUB: tiles per span (the host's sub_filtered); the LDS holds the span's compacted records (at most SUB tiles).
template <typename SD, typename T, typename H, int LP, int SUB>
__global__ __launch_bounds__(PART_THREADS) void part1_spread_mask(Side s, Digit dg, NextDigit nd, uint32_t n_digits,
                                                                 const uint32_t* __restrict__ offsets,
                                                                 const uint64_t* __restrict__ match_bits,
                                                                 Rec<H, uint32_t>* __restrict__ out) {
  static_assert(SUB >= 1 && SUB * PART_TILE * sizeof(Rec<H, uint32_t>) >= PART_WAVES * 256 * 8, "mask area");
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ uint32_t s_wm[PART_WAVES], s_wa[PART_WAVES];
  __shared__ Rec<H, uint32_t> s_comp[SUB * PART_TILE];  // the span's compacted records; rounds stage in its front
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);  // span
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (SUB * PART_TILE);
  const uint32_t n_sub = min(static_cast<uint32_t>(SUB), (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  uint32_t run = threadIdx.x < n_digits ? offsets[threadIdx.x * s.n_tiles + tile] : 0u;
  uint32_t scan_pos = offsets[n_digits * s.n_tiles + tile] - offsets[n_digits * s.n_tiles];  // span's first match
  uint32_t comp_n = 0;
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    const uint64_t* mb = match_bits + (tile * SUB + j) * MASK_WORDS + w * PART_ITEMS;
    uint64_t b[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) b[k] = mb[k];  // wave-uniform words
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) m |= static_cast<uint32_t>((b[k] >> lane) & 1u) << k;
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    const uint32_t act = bloom_filter_act<H>(s, keys, load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m);
    uint64_t a[PART_ITEMS];
    uint32_t mc = 0, ac = 0;
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      a[k] = __ballot((act >> k) & 1u);
      mc += static_cast<uint32_t>(__popcll(b[k]));
      ac += static_cast<uint32_t>(__popcll(a[k]));
    }
    if (lane == 0) {
      s_wm[w] = mc;
      s_wa[w] = ac;
    }
    __syncthreads();
    uint32_t mp = scan_pos, ap = comp_n, mt = 0, at = 0;
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) {
      if (ww < w) {
        mp += s_wm[ww];
        ap += s_wa[ww];
      }
      mt += s_wm[ww];
      at += s_wa[ww];
    }
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      if (((m >> k) & 1u) && s.scan_out != nullptr)
        s.scan_out[mp + static_cast<uint32_t>(__popcll(b[k] & lt))] = rb + k * WAVE + lane;
      if ((act >> k) & 1u) {
        Rec<H, uint32_t> r;
        r.key = keys[k];
        r.payload = pays[k];
        s_comp[ap + static_cast<uint32_t>(__popcll(a[k] & lt))] = r;
      }
      mp += static_cast<uint32_t>(__popcll(b[k]));
      ap += static_cast<uint32_t>(__popcll(a[k]));
    }
    scan_pos += mt;
    comp_n += at;
    __syncthreads();  // s_wm / s_wa are rewritten by the next tile; s_comp complete after the last
  }
  // stable scatter of the compacted records by digit, one tile-sized round at a time
#pragma unroll 1
  for (uint32_t r0 = 0; r0 < comp_n; r0 += PART_TILE) {
    if (r0) __syncthreads();  // the previous round's write-out has read the staging area
    Rec<H, uint32_t> recs[PART_ITEMS];
    uint32_t act = 0;
    const uint32_t i0 = r0 + w * WAVE_SPAN + lane;
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint32_t i = i0 + k * WAVE;
      recs[k] = s_comp[min(i, comp_n - 1)];
      if (i < comp_n) act |= 1u << k;
    }
    __syncthreads();  // every record of the round is in registers before the masks / staging overwrite the front
    clear_wave_counts(s_cnt[w]);
    uint32_t dr[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool aa = (act >> k) & 1u;
      const uint32_t dig = aa ? digit_of<H>(dg, recs[k].key) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, aa, s_cnt[w]);
    }
    staged_scatter<H, uint32_t>(recs, act, dr, s_cnt, s_delta, s_comp, s_scratch, n_digits, dg, nd, run, out);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Pass 1 in row blocks sized for the Infinity Cache (the default for large sides; join_host.hpp block_plan): the
// side's spans are cut into K contiguous blocks of ~100-200 MB of input each, and every block runs
//   part1_count : the predicate (fused TableScan) and the join column of every row of the block's spans - digit
//                 histogram of the rows taking part, plus the scan-match row - as part1_hist / part1_compact count;
//   exclusive scan of the block's histogram (digit-major over its spans) and block_totals;
//   part1_fill  : the same rows read AGAIN - served by the 256 MiB Infinity Cache, which still holds the block that
//                 part1_count has just streamed (MI355X_MICROARCH.md "Infinity Cache": a table stays resident while it
//                 plus the bytes moved in between fit; profiles/r05_mall_probe.jsonl: a re-read of 96-256 MB blocks
//                 costs ~0.14 ms/GB less than from HBM, i.e. close to nothing) - writes the scan's output (chunk
//                 offsets, row order) and the stable LDS-staged scatter of the records by the high digit.
// Block k's records land in a region of its own, [row_base_k, row_base_k + records_k) (rows of the earlier blocks:
// records <= rows), digit-major inside it, so no prefix across blocks is needed before a block's fill; the first
// record pass then reads bucket d as the K runs (d, k) in block order - the interleaved-segment geometry of the
// distributed receiver (block_geometry). Against part1_compact + part1_spread this drops the gapped record round trip
// (write + re-read of 8 B per match) from HBM; against part1_hist + part1_scatter the second read of the column.
// ------------------------------------------------------------------------------------------------------------
// part1_count's loads for value chunks with 16-byte aligned data: lane l takes the 16 consecutive rows r0 .. r0 + 15
// (r0 = wave span + 16 l) with 16-byte vector loads - a count does not care which lane holds which row - instead of 16
// strided element loads per column. Rows past the chunk are masked out.
template <typename T, typename H>
__device__ __forceinline__ uint32_t load_keys_contig(const SrcChunk& ch, uint32_t r0, H (&keys)[PART_ITEMS]) {
  static_assert(PART_ITEMS * sizeof(T) % 16 == 0, "whole vectors");
  const T* data = static_cast<const T*>(ch.data);
  if (r0 + PART_ITEMS <= ch.size) {
    constexpr int NV = PART_ITEMS * sizeof(T) / 16;
    uint4 u[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) u[j] = reinterpret_cast<const uint4*>(data + r0)[j];
    T v[PART_ITEMS];
    __builtin_memcpy(v, u, sizeof(v));
#pragma unroll
    for (int i = 0; i < PART_ITEMS; ++i) keys[i] = static_cast<H>(v[i]);
    return 0xFFFFu;
  }
  uint32_t act = 0;
#pragma unroll
  for (int i = 0; i < PART_ITEMS; ++i) {
    const uint32_t r = r0 + i;
    keys[i] = static_cast<H>(data[min(r, ch.size - 1)]);
    if (r < ch.size) act |= 1u << i;
  }
  return act;
}

template <typename E>
__device__ __forceinline__ uint32_t filter_dict_contig(const hy_scan_chunk& f, uint32_t r0) {
  static_assert(PART_ITEMS * sizeof(E) % 16 == 0, "whole vectors");
  const E* data = static_cast<const E*>(f.column.data);
  const uint32_t n = f.column.size;
  E v[PART_ITEMS];
  if (r0 + PART_ITEMS <= n) {
    constexpr int NV = PART_ITEMS * sizeof(E) / 16;
    uint4 u[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) u[j] = reinterpret_cast<const uint4*>(data + r0)[j];
    __builtin_memcpy(v, u, sizeof(v));
  } else {
#pragma unroll
    for (int i = 0; i < PART_ITEMS; ++i) v[i] = data[min(r0 + i, n - 1)];
  }
  const DictPred pr = dict_pred(f.op, static_cast<E>(f.search_vid), static_cast<E>(f.column.dictionary_size));
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < PART_ITEMS; ++i) m |= static_cast<uint32_t>((r0 + i < n) & dict_match(pr, v[i])) << i;
  return m;
}

template <typename SD, typename T, typename H, int LP, int FK, bool PF>
__global__ __launch_bounds__(PART_THREADS) void part1_count(Side s, Digit dg, uint32_t n_digits, uint64_t t0,
                                                           uint32_t* __restrict__ hist) {
  // value chunks with a dictionary (or no) predicate: the contiguous vector loads
  constexpr bool CONTIG = LP == LP_VALUE && (FK == FK_NONE || FK == FK_DICT8 || FK == FK_DICT16 || FK == FK_DICT32);
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_sc;
  const uint32_t nt = gridDim.x;
  const uint32_t lt = xcd_tile(blockIdx.x, nt);
  const uint64_t tile = t0 + lt;  // span
  for (int i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  if (threadIdx.x == 0) s_sc = 0;
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  __syncthreads();
  uint32_t nm = 0;  // this wave's scan matches (wave-uniform)
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    uint32_t m_scan = 0xFFFFu;
    H keys[PART_ITEMS];
    uint32_t act;
    bool contig = false;
    if constexpr (CONTIG) {
      const hy_scan_chunk* f = FK != FK_NONE ? &s.filter[c] : nullptr;
      contig = (reinterpret_cast<uintptr_t>(ch.data) & 15u) == 0 &&
               (FK == FK_NONE || f->op == HY_OP_NONE || f->column.size == 0 ||
                (reinterpret_cast<uintptr_t>(f->column.data) & 15u) == 0);  // (uniform)
      if (contig) {
        const uint32_t r0 = rb + lane * PART_ITEMS;
        if constexpr (FK != FK_NONE) {
          if (f->op == HY_OP_NONE || f->column.size == 0)
            m_scan = 0u;
          else if constexpr (FK == FK_DICT8)
            m_scan = filter_dict_contig<uint8_t>(*f, r0);
          else if constexpr (FK == FK_DICT16)
            m_scan = filter_dict_contig<uint16_t>(*f, r0);
          else
            m_scan = filter_dict_contig<uint32_t>(*f, r0);
        }
        act = load_keys_contig<T, H>(ch, r0, keys) & m_scan;
      }
    }
    if (!contig) {
      if constexpr (FK != FK_NONE) m_scan = filter_items<FK>(s, c, rb);
      uint32_t pays[PART_ITEMS];
      act = load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m_scan;
    }
    if constexpr (PF) act = bloom_filter_act<H>(s, keys, act);
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if ((act >> k) & 1u) atomicAdd(&s_hist[digit_of<H>(dg, keys[k])], 1u);
    if constexpr (FK != FK_NONE) {
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) nm += static_cast<uint32_t>(__popcll(__ballot((m_scan >> k) & 1u)));
    }
  }
  if constexpr (FK != FK_NONE)
    if (lane == 0 && nm) atomicAdd(&s_sc, nm);
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[d * nt + lt] = s_hist[d];
  if constexpr (FK != FK_NONE)
    if (threadIdx.x == 0) hist[n_digits * nt + lt] = s_sc;
}

// rec_base: first record position of the block (its first row); scan_base: the scan matches of the earlier blocks
// (device, set by block_totals). offsets: the block's exclusive histogram scan.
template <typename SD, typename T, typename H, int LP, int FK, bool PF>
__global__ __launch_bounds__(PART_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void part1_fill(
    Side s, Digit dg, NextDigit nd, uint32_t n_digits, uint64_t t0, const uint32_t* __restrict__ offsets,
    uint32_t rec_base, const uint64_t* __restrict__ scan_base, Rec<H, uint32_t>* __restrict__ out) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ uint32_t s_sc[WAVE + 1];
  __shared__ Rec<H, uint32_t> s_stage[PART_TILE];
  const uint32_t nt = gridDim.x;
  const uint32_t lt = xcd_tile(blockIdx.x, nt);
  const uint64_t tile = t0 + lt;  // span
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  uint32_t run = threadIdx.x < n_digits ? rec_base + offsets[threadIdx.x * nt + lt] : 0u;
  uint32_t srun = 0;  // the span's first scan match (output position)
  if constexpr (FK != FK_NONE)
    srun = static_cast<uint32_t>(*scan_base) + offsets[n_digits * nt + lt] - offsets[n_digits * nt];
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    if (j) __syncthreads();  // the previous tile's write-out has read s_stage and s_sc
    clear_wave_counts(s_cnt[w]);
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    uint32_t m_scan = 0xFFFFu;
    if constexpr (FK != FK_NONE) m_scan = filter_items<FK>(s, c, rb);
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    uint32_t act = load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m_scan;
    if constexpr (PF) act = bloom_filter_act<H>(s, keys, act);
    const bool scan_out = FK != FK_NONE && s.scan_out != nullptr;
    if (scan_out) {
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {
        const uint64_t b = __ballot((m_scan >> k) & 1u);
        if (lane == 0) s_sc[w * PART_ITEMS + k] = static_cast<uint32_t>(__popcll(b));
      }
    }
    Rec<H, uint32_t> recs[PART_ITEMS];
    uint32_t dr[PART_ITEMS];  // digit << 24 | rank within the wave
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, keys[k]) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
      recs[k].key = keys[k];
      recs[k].payload = pays[k];
    }
    if (scan_out) {  // the tile's scan matches in row order: (wave, item) ballot counts -> prefix -> lane rank
      __syncthreads();
      if (threadIdx.x < WAVE) {
        const uint32_t v = s_sc[threadIdx.x];
        const uint32_t incl = wave_inclusive_sum(v);
        s_sc[threadIdx.x] = incl - v;
        if (threadIdx.x == WAVE - 1) s_sc[WAVE] = incl;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {
        const uint64_t b = __ballot((m_scan >> k) & 1u);
        if ((m_scan >> k) & 1u)
          s.scan_out[srun + s_sc[w * PART_ITEMS + k] + static_cast<uint32_t>(__popcll(b & lanemask_lt()))] =
              rb + k * WAVE + lane;
      }
      srun += s_sc[WAVE];
    }
    staged_scatter<H, uint32_t>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run, out);
  }
}

// After block k's histogram scan (nt spans; records = the scan total, or for a fused scan the first entry of its
// scan row): the block's per-digit runs for block_geometry, the scan matches of blocks <= k (scan_base[k + 1]) and
// the scan's chunk begins of the chunks whose first span lies in this block, [c_lo, c_hi) (the last block also takes the
// trailing span-less chunks and the end entry).
static __global__ __launch_bounds__(256) void block_totals(const uint32_t* __restrict__ offsets, uint32_t nt,
                                                           uint32_t n_digits, int filtered,
                                                           const uint64_t* __restrict__ scan_total, uint32_t k,
                                                           uint32_t rec_base, uint64_t t0, uint64_t n_tiles,
                                                           int last_block, uint32_t* __restrict__ cls_begin,
                                                           uint32_t* __restrict__ cls_count,
                                                           uint64_t* __restrict__ scan_base,
                                                           const uint64_t* __restrict__ chunk_tile_begin,
                                                           uint32_t c_lo, uint32_t c_hi,
                                                           uint64_t* __restrict__ chunk_begin) {
  const uint64_t total = *scan_total;
  const uint32_t records = filtered ? offsets[static_cast<uint64_t>(n_digits) * nt] : static_cast<uint32_t>(total);
  for (uint32_t d = threadIdx.x; d < n_digits; d += blockDim.x) {
    const uint32_t b = offsets[static_cast<uint64_t>(d) * nt];
    const uint32_t e = d + 1 < n_digits ? offsets[static_cast<uint64_t>(d + 1) * nt] : records;
    cls_begin[k * 256 + d] = rec_base + b;
    cls_count[k * 256 + d] = e - b;
  }
  if (!filtered) return;
  const uint64_t sb = scan_base[k];
  if (threadIdx.x == 0) scan_base[k + 1] = sb + (total - records);
  if (chunk_begin == nullptr) return;
  const uint64_t row = static_cast<uint64_t>(n_digits) * nt;
  for (uint32_t cc = c_lo + threadIdx.x; cc < c_hi; cc += blockDim.x) {  // (the host's range of such chunks)
    const uint64_t t = chunk_tile_begin[cc];
    if (t >= t0 && t < t0 + nt)
      chunk_begin[cc] = sb + offsets[row + (t - t0)] - records;
    else if (last_block && t >= n_tiles)
      chunk_begin[cc] = sb + (total - records);
  }
}

// Geometry of the record pass over the blocks' runs (one workgroup, thread g = pass-1 bucket g): bucket g's segments
// are the runs (g, k), k = 0..K-1 in block order; their tiles of `span` records are interleaved in the histogram by
// (bucket, digit, block, tile), as onepass_geometry lays out its classes, and the bucket's output starts at the records
// of all earlier buckets. Writes the segment / group arrays, the tile prefix (n_groups * K + 1) and the record total.
static __global__ __launch_bounds__(256) void block_geometry(const uint32_t* __restrict__ cls_begin,
                                                             const uint32_t* __restrict__ cls_count, uint32_t n_blocks,
                                                             uint32_t n_groups, uint32_t span, uint32_t next_digits,
                                                             uint32_t* seg_begin, uint32_t* seg_end,
                                                             uint32_t* seg_stride, uint32_t* seg_toff,
                                                             uint64_t* seg_hbase, uint64_t* seg_tile_begin,
                                                             uint64_t* group_hbase, uint32_t* group_tiles,
                                                             uint32_t* group_out, uint64_t* total) {
  __shared__ uint32_t s_scratch[256 / WAVE + 1];
  const uint32_t g = threadIdx.x;
  uint32_t gt = 0, gc = 0;
  if (g < n_groups) {
    for (uint32_t k = 0; k < n_blocks; ++k) {
      const uint32_t n = cls_count[k * 256 + g];
      gt += (n + span - 1) / span;
      gc += n;
    }
  }
  uint32_t tiles_total, rows_total;
  const uint32_t tile_base = block_exclusive_sum<256>(gt, s_scratch, &tiles_total);
  const uint32_t out_base = block_exclusive_sum<256>(gc, s_scratch, &rows_total);
  if (g < n_groups) {
    const uint64_t hb = static_cast<uint64_t>(tile_base) * next_digits;
    uint32_t toff = 0;
    for (uint32_t k = 0; k < n_blocks; ++k) {
      const uint32_t q = g * n_blocks + k;
      const uint32_t n = cls_count[k * 256 + g];
      const uint32_t b0 = cls_begin[k * 256 + g];
      seg_begin[q] = b0;
      seg_end[q] = b0 + n;
      seg_stride[q] = gt;
      seg_toff[q] = toff;
      seg_hbase[q] = hb;
      seg_tile_begin[q] = tile_base + toff;
      toff += (n + span - 1) / span;
    }
    group_hbase[g] = hb;
    group_tiles[g] = gt;
    group_out[g] = out_base;
  }
  if (g == 0) {
    seg_tile_begin[n_groups * n_blocks] = tiles_total;
    *total = rows_total;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Single-pass first radix pass (part1_onepass): the histogram, its prefix across tiles and the stable scatter in ONE
// read of the column chunks (and of the fused scan's predicate column), instead of part1_hist + scan + part1_scatter
// (two reads) or part1_compact + scan + part1_spread (one read plus a gapped write and re-read of the records).
//
// The pass-0 tiles are split into NCLASS contiguous ranges ("classes"); workgroups of class x (blockIdx % NCLASS: the
// blocks that share an XCD, so a range's neighbouring tiles complete their shared output lines in one L2) take the
// class's tiles in order from a per-class atomic ticket. Every tile publishes its 256 digit counts as look-back
// granules and resolves, per digit, the count of the same digit in the class's earlier tiles (a decoupled look-back
// per digit, one thread per digit) - so no tile waits on another class. Class x writes digit d's records into their
// own region (d * NCLASS + x) * cap of a gapped buffer, in row order. The regions of digit d, taken in class order,
// are exactly the stable pass-1 bucket d; the next record pass reads them as NCLASS segments per bucket (the
// interleaved-segment geometry of the distributed receiver) and writes compact output. A region that would exceed
// `cap` (skewed keys) sets the overflow flag and the tile writes nothing; the host then runs the two-read path.
//
// The fused TableScan's output cannot be placed in the same pass without a prefix over ALL earlier tiles (a wait
// across classes), so the pass writes each tile's match bitmask (one 64-bit ballot per wave and item, 512 B per
// tile) and match count; part1_scan_expand turns them into the scan's chunk offsets after a scan of the counts.
// ------------------------------------------------------------------------------------------------------------
constexpr uint32_t NCLASS = 8;
constexpr uint32_t LB32_AGG = 1u << 30;
constexpr uint32_t LB32_PREFIX = 2u << 30;
constexpr uint32_t LB32_VALUE = (1u << 30) - 1;
constexpr int LB_WIN = 16;  // predecessors polled per look-back round trip

struct OnePass {
  const uint32_t* class_begin;  // NCLASS + 1 tile bounds of the classes
  uint32_t* ticket;             // NCLASS counters (zeroed before the launch)
  uint32_t* status;             // n_tiles * 256 look-back granules (zeroed before the launch)
  uint32_t* class_count;        // NCLASS * 256: records of digit d in class x (zeroed before the launch)
  uint64_t cap;                 // records per (digit, class) region
  uint32_t* flags;              // [0] bit 0: a region overflowed, bit 1: a look-back timed out
  uint64_t* match_bits;         // n_tiles * 64 ballots (filtered sides with a scan output), or null
  uint32_t* match_count;        // n_tiles match counts (filtered sides with a scan output), or null
  uint32_t win;                 // predecessors polled per look-back round trip (1..LB_WIN)
  uint32_t static_order;        // 1: tile = blockIdx / NCLASS instead of the per-class ticket (experiment)
};

template <typename T, typename H, int LP, int FK>
__global__ __launch_bounds__(PART_THREADS) void part1_onepass(Side s, Digit dg, NextDigit nd, uint32_t n_digits,
                                                             OnePass op, Rec<H, uint32_t>* __restrict__ out) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ Rec<H, uint32_t> s_stage[PART_TILE];
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_bad;
  const uint32_t x = blockIdx.x % NCLASS;
  const uint32_t c0 = op.class_begin[x], n_cls = op.class_begin[x + 1] - c0;
  if (threadIdx.x == 0) {
    s_tile = op.static_order ? blockIdx.x / NCLASS : atomicAdd(&op.ticket[x], 1u);
    s_bad = 0;
  }
  __syncthreads();
  const uint32_t i = s_tile;
  if (i >= n_cls) return;
  const uint64_t tile = c0 + i;
  const uint32_t c = s.tile_chunk[tile];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * PART_TILE;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  clear_wave_counts(s_cnt[w]);
  const uint32_t rb = base + w * WAVE_SPAN;
  uint32_t m = 0xFFFFu;
  if constexpr (FK != FK_NONE) {
    m = filter_items<FK>(s, c, rb);
    if (op.match_bits != nullptr) {
      uint32_t cnt = 0;
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {
        const uint64_t b = __ballot((m >> k) & 1u);
        if (lane == k) op.match_bits[tile * (PART_WAVES * PART_ITEMS) + w * PART_ITEMS + k] = b;
        cnt += static_cast<uint32_t>(__popcll(b));
      }
      if (lane == 0) s_scratch[w] = cnt;
    }
  }
  H keys[PART_ITEMS];
  uint32_t pays[PART_ITEMS];
  const uint32_t act = load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m;
  Rec<H, uint32_t> recs[PART_ITEMS];
  uint32_t dr[PART_ITEMS];
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) {
    const bool a = (act >> k) & 1u;
    const uint32_t dig = a ? digit_of<H>(dg, keys[k]) : 0u;
    dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
    recs[k].key = keys[k];
    recs[k].payload = pays[k];
  }
  __syncthreads();  // every wave's digit counts (and match counts) are in LDS
  if constexpr (FK != FK_NONE) {
    if (op.match_count != nullptr && threadIdx.x == 0) {
      uint32_t t = 0;
#pragma unroll
      for (int ww = 0; ww < PART_WAVES; ++ww) t += s_scratch[ww];
      op.match_count[tile] = t;
    }
  }
  // per digit: publish this tile's count, resolve the class-local prefix of the earlier tiles, publish the inclusive
  const uint32_t d = threadIdx.x;
  uint32_t run = 0;
  if (d < n_digits) {
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) tot += s_cnt[ww][d];
    uint32_t* st = op.status + tile * 256 + d;
    uint32_t prefix = 0;
    if (i == 0) {
      __hip_atomic_store(st, LB32_PREFIX | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(st, LB32_AGG | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // windowed walk: LB_WIN predecessors polled with independent loads per round trip, summed up to the nearest
      // inclusive prefix; a not-yet-published predecessor ends the round (the sum so far is kept) and is re-polled
      uint64_t j = tile;  // tiles [c0, j) remain to be resolved
      uint32_t spins = 0;
      bool done = false;
      while (!done && j > c0) {
        uint32_t v[LB_WIN];
#pragma unroll
        for (int k = 0; k < LB_WIN; ++k)
          v[k] = (k < op.win && j - k > c0) ? __hip_atomic_load(op.status + (j - 1 - k) * 256 + d, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : (j - k > c0 ? 0u : LB32_PREFIX);  // before the class start: inclusive prefix 0
        uint32_t k = 0;
        for (; k < op.win; ++k) {
          const uint32_t f = v[k] & ~LB32_VALUE;
          if (f == 0) break;
          prefix += v[k] & LB32_VALUE;
          if (f == LB32_PREFIX) {
            done = true;
            break;
          }
        }
        if (done) break;
        j -= k;
        if (k < op.win) {  // predecessor j - 1 has not published yet
          if (++spins > LB_MAX_SPINS) {
            atomicOr(op.flags, 2u);
            s_bad = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __hip_atomic_store(st, LB32_PREFIX | (prefix + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (i == n_cls - 1) op.class_count[x * 256 + d] = prefix + tot;
    if (prefix + tot > op.cap) {
      atomicOr(op.flags, 1u);
      s_bad = 1;
    }
    run = static_cast<uint32_t>((static_cast<uint64_t>(d) * NCLASS + x) * op.cap) + prefix;
  }
  __syncthreads();
  if (s_bad) return;  // the host falls back to the two-read path; nothing of this tile is written
  staged_scatter<H, uint32_t>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run, out);
}

// The fused scan's output from part1_onepass's per-tile match bitmasks: tile_off = exclusive scan of the match
// counts (matches in row order), each matching row's chunk offset written at its position; chunk_begin[c] = position
// of chunk c's first match (n_chunks + 1 entries).
static __global__ __launch_bounds__(PART_THREADS) void part1_scan_expand(Side s, const uint64_t* __restrict__ bits,
                                                                       const uint32_t* __restrict__ tile_off,
                                                                       const uint64_t* __restrict__ total,
                                                                       uint64_t* __restrict__ chunk_begin) {
  __shared__ uint32_t s_w[PART_WAVES + 1];
  __shared__ uint32_t s_out[PART_TILE];
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  const uint32_t c = s.tile_chunk[tile];
  const uint32_t base = static_cast<uint32_t>(tile - s.chunk_tile_begin[c]) * PART_TILE + w * WAVE_SPAN;
  uint64_t b[PART_ITEMS];
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) {
    b[k] = bits[tile * (PART_WAVES * PART_ITEMS) + w * PART_ITEMS + k];
    cnt += static_cast<uint32_t>(__popcll(b[k]));
  }
  if (lane == 0) s_w[w] = cnt;
  const uint32_t pos0 = tile_off[tile];
  __syncthreads();
  uint32_t pos = 0, n = 0;
  for (int ww = 0; ww < PART_WAVES; ++ww) {
    if (ww < w) pos += s_w[ww];
    n += s_w[ww];
  }
  // the tile's offsets in row order into LDS, then written out by consecutive lanes (coalesced)
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) {
    if ((b[k] >> lane) & 1u) s_out[pos + __popcll(b[k] & lanemask_lt())] = base + k * WAVE + lane;
    pos += static_cast<uint32_t>(__popcll(b[k]));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += PART_THREADS) s.scan_out[pos0 + i] = s_out[i];
  if (chunk_begin != nullptr && blockIdx.x == 0) {
    for (uint32_t cc = threadIdx.x; cc <= s.n_chunks; cc += PART_THREADS) {
      const uint64_t t = s.chunk_tile_begin[cc];
      chunk_begin[cc] = t < s.n_tiles ? tile_off[t] : *total;
    }
  }
}

// Geometry of the record pass that follows part1_onepass (one workgroup, thread g = pass-1 bucket g): the NCLASS
// regions of bucket g are its segments g * NCLASS + x (begin = region start, end = begin + count), their tiles of
// `span` records are interleaved in the histogram by (bucket, digit, class, tile) - the layout record_pass takes for
// the distributed receiver's (bucket, sender) runs - and the bucket's output starts at the count of all earlier
// buckets. Writes the segment / group arrays, the tile prefix (n_segs + 1) and the record total.
static __global__ __launch_bounds__(256) void onepass_geometry(const uint32_t* __restrict__ class_count, uint32_t n_groups,
                                                               uint64_t cap, uint32_t span, uint32_t next_digits,
                                                               uint32_t* seg_begin, uint32_t* seg_end,
                                                               uint32_t* seg_stride, uint32_t* seg_toff,
                                                               uint64_t* seg_hbase, uint64_t* seg_tile_begin,
                                                               uint64_t* group_hbase, uint32_t* group_tiles,
                                                               uint32_t* group_out, uint64_t* total) {
  __shared__ uint32_t s_scratch[256 / WAVE + 1];
  const uint32_t g = threadIdx.x;
  uint32_t cnt[NCLASS], gt = 0, gc = 0;
#pragma unroll
  for (uint32_t x = 0; x < NCLASS; ++x) {
    cnt[x] = g < n_groups ? static_cast<uint32_t>(min<uint64_t>(class_count[x * 256 + g], cap)) : 0u;
    gt += (cnt[x] + span - 1) / span;
    gc += cnt[x];
  }
  uint32_t tiles_total, rows_total;
  const uint32_t tile_base = block_exclusive_sum<256>(gt, s_scratch, &tiles_total);
  const uint32_t out_base = block_exclusive_sum<256>(gc, s_scratch, &rows_total);
  if (g < n_groups) {
    const uint64_t hb = static_cast<uint64_t>(tile_base) * next_digits;
    uint32_t toff = 0;
#pragma unroll
    for (uint32_t x = 0; x < NCLASS; ++x) {
      const uint32_t q = g * NCLASS + x;
      const uint32_t b0 = static_cast<uint32_t>(static_cast<uint64_t>(q) * cap);
      seg_begin[q] = b0;
      seg_end[q] = b0 + cnt[x];
      seg_stride[q] = gt;
      seg_toff[q] = toff;
      seg_hbase[q] = hb;
      seg_tile_begin[q] = tile_base + toff;
      toff += (cnt[x] + span - 1) / span;
    }
    group_hbase[g] = hb;
    group_tiles[g] = gt;
    group_out[g] = out_base;
  }
  if (g == 0) {
    seg_tile_begin[n_groups * NCLASS] = tiles_total;
    *total = rows_total;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Pass 2: records -> records, inside every pass-1 bucket (segment).
// ------------------------------------------------------------------------------------------------------------
// Pass-2 segments. Single-GPU: the pass-1 buckets, contiguous (seg_begin[i], seg_begin[i+1]) with the histogram of
// segment i at [seg_tile_begin[i] * n_digits, ...) digit-major. Distributed join (receiver): one segment per
// (bucket, sender) run of the received buffer, listed bucket-major / sender-minor; seg_end gives each run's end, and
// the histogram of a segment is interleaved with the other senders' runs of its bucket - entry (digit d, tile t) at
// seg_hbase[i] + d * seg_stride[i] + seg_toff[i] + t - so that the exclusive scan orders the output by (bucket, digit,
// sender, tile): the reference's (partition, chunk, offset) order across ranks.
struct Segs {
  const uint32_t* seg_begin;        // record offset of each segment (n_segs + 1 entries when seg_end is null)
  const uint64_t* seg_tile_begin;   // n_segs + 1 tile prefix (grid is an upper bound)
  const uint32_t* tile_seg;         // segment of each pass-2 tile
  uint32_t n_segs;
  const uint32_t* seg_end;          // null: seg_begin[i + 1]
  const uint64_t* seg_hbase;        // null: seg_tile_begin[i] * n_digits
  const uint32_t* seg_stride;       // null: the segment's tile count
  const uint32_t* seg_toff;         // null: 0
  uint32_t sub;                     // tiles per span
};

__device__ __forceinline__ void seg_geometry(const Segs& sg, uint32_t sgi, uint32_t n_digits, uint32_t* b0, uint32_t* b1,
                                             uint64_t* hbase, uint32_t* stride, uint32_t* toff) {
  const uint32_t nt = static_cast<uint32_t>(sg.seg_tile_begin[sgi + 1] - sg.seg_tile_begin[sgi]);
  *b0 = sg.seg_begin[sgi];
  *b1 = sg.seg_end ? sg.seg_end[sgi] : sg.seg_begin[sgi + 1];
  *hbase = sg.seg_hbase ? sg.seg_hbase[sgi] : sg.seg_tile_begin[sgi] * n_digits;
  *stride = sg.seg_stride ? sg.seg_stride[sgi] : nt;
  *toff = sg.seg_toff ? sg.seg_toff[sgi] : 0u;
}

template <typename SD, typename H, typename P>
__global__ __launch_bounds__(PART_THREADS) void part2_hist(Segs sg, Digit dg, uint32_t n_digits,
                                                          const Rec<H, P>* __restrict__ in, uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_hist[256];
  const uint32_t n_real = static_cast<uint32_t>(sg.seg_tile_begin[sg.n_segs]);
  if (blockIdx.x >= n_real) return;
  const uint64_t tile = xcd_tile(blockIdx.x, n_real);  // XCD-contiguous over the tiles that exist
  for (int i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  __syncthreads();
  const uint32_t sgi = sg.tile_seg[tile];
  const uint32_t t_in = static_cast<uint32_t>(tile - sg.seg_tile_begin[sgi]);
  uint32_t b0, b1, stride, toff;
  uint64_t hbase;
  seg_geometry(sg, sgi, n_digits, &b0, &b1, &hbase, &stride, &toff);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t sb = b0 + t_in * (sg.sub * PART_TILE);
  const uint32_t n_sub = min(sg.sub, (b1 - sb + PART_TILE - 1) / PART_TILE);
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    // unconditional loads from clamped rows (see load_items), then the counts of the rows in range
    const uint32_t r0 = sb + j * PART_TILE + w * WAVE_SPAN + __lane_id();
    uint32_t dig[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) dig[k] = digit_of<H>(dg, in[min(r0 + k * WAVE, b1 - 1)].key);
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if (r0 + k * WAVE < b1) atomicAdd(&s_hist[dig[k]], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[hbase + d * stride + toff + t_in] = s_hist[d];
}

template <typename SD, typename H, typename P>
__global__ __launch_bounds__(PART_THREADS) void part2_scatter(Segs sg, Digit dg, NextDigit nd, int dbits,
                                                             uint32_t n_digits, const Rec<H, P>* __restrict__ in,
                                                             const uint32_t* __restrict__ offsets, RecOut<H, P> out) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ Rec<H, P> s_stage[PART_TILE];
  const uint32_t n_real = static_cast<uint32_t>(sg.seg_tile_begin[sg.n_segs]);
  if (blockIdx.x >= n_real) return;
  const uint64_t tile = xcd_tile(blockIdx.x, n_real);  // span; XCD-contiguous over the tiles that exist
  const uint32_t sgi = sg.tile_seg[tile];
  const uint32_t t_in = static_cast<uint32_t>(tile - sg.seg_tile_begin[sgi]);
  uint32_t b0, b1, stride, toff;
  uint64_t hbase;
  seg_geometry(sg, sgi, n_digits, &b0, &b1, &hbase, &stride, &toff);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t sb = b0 + t_in * (sg.sub * PART_TILE);
  const uint32_t n_sub = min(sg.sub, (b1 - sb + PART_TILE - 1) / PART_TILE);
  uint32_t run = threadIdx.x < n_digits ? offsets[hbase + threadIdx.x * stride + toff + t_in] : 0u;
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    if (j) __syncthreads();  // the previous tile's write-out has read s_stage
    clear_wave_counts(s_cnt[w]);
    Rec<H, P> recs[PART_ITEMS];
    uint32_t dr[PART_ITEMS];  // digit << 24 | rank within the wave
    uint32_t act = 0;
    const uint32_t r0 = sb + j * PART_TILE + w * WAVE_SPAN + __lane_id();
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) recs[k] = in[min(r0 + k * WAVE, b1 - 1)];  // unconditional (see load_items)
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if (r0 + k * WAVE < b1) act |= 1u << k;
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, recs[k].key) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
    }
    staged_scatter<H, P>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, nd, run, out);
  }
}

// part2_hist from the digit bytes the previous pass wrote beside the records (1 B per record instead of the record
// and its hash); same tiles and histogram layout as part2_hist. (Round 5 measured eight tiles per workgroup with every
// load issued first: 0.166 against 0.171 ms at SF100, not adopted. tools/hist_probe.hip: the same counts cost 0.17 ms
// without any LDS atomic when each workgroup writes its 256 entries into the digit-major matrix, 0.09 ms tile-major -
// the histogram's scattered 4-byte writes, not the counting, bound the pass.)
template <typename SD>
__global__ __launch_bounds__(PART_THREADS) void part2_hist_bytes(Segs sg, uint32_t n_digits,
                                                                const uint8_t* __restrict__ dig,
                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_hist[256];
  const uint32_t n_real = static_cast<uint32_t>(sg.seg_tile_begin[sg.n_segs]);
  if (blockIdx.x >= n_real) return;
  const uint64_t tile = xcd_tile(blockIdx.x, n_real);  // XCD-contiguous over the tiles that exist
  for (int i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  __syncthreads();
  const uint32_t sgi = sg.tile_seg[tile];
  const uint32_t t_in = static_cast<uint32_t>(tile - sg.seg_tile_begin[sgi]);
  uint32_t b0, b1, stride, toff;
  uint64_t hbase;
  seg_geometry(sg, sgi, n_digits, &b0, &b1, &hbase, &stride, &toff);
  const uint32_t sb = b0 + t_in * (sg.sub * PART_TILE);
  const uint32_t n_sub = min(sg.sub, (b1 - sb + PART_TILE - 1) / PART_TILE);
  // the tile's bytes [lo, hi) as 16-byte vectors from the aligned address below lo (the digit arrays are 256-byte
  // aligned and padded): one load per thread instead of 16 byte loads per lane
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    const uint32_t lo = sb + j * PART_TILE, hi = min(lo + PART_TILE, b1), a0 = lo & ~15u;
    const uint32_t nv = (hi - a0 + 15) / 16;
    for (uint32_t v = threadIdx.x; v < nv; v += PART_THREADS) {
      const uint4 u = reinterpret_cast<const uint4*>(dig + a0)[v];
      const uint32_t words[4] = {u.x, u.y, u.z, u.w};
      const uint32_t p0 = a0 + v * 16;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t p = p0 + i;
        if (p >= lo && p < hi) atomicAdd(&s_hist[(words[i >> 2] >> (8 * (i & 3))) & 0xFFu], 1u);
      }
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS) hist[hbase + d * stride + toff + t_in] = s_hist[d];
}

// After the exclusive scan of a fused-scan histogram (part1_compact: (n_digits + 1) rows over n_tiles spans): records = first
// entry of the scan row, matches = grand total - records; chunk c's matches start at the scan-row prefix of its first
// span (chunks without spans take the next chunk's start). Writes the record total (for the bucket bounds), the
// scan's per-chunk begins (n_chunks + 1, in matches) and its total.
static __global__ void fused_scan_totals(const uint32_t* __restrict__ offsets, uint64_t n_tiles, uint32_t n_digits,
                                  const uint64_t* __restrict__ grand_total, const uint64_t* __restrict__ chunk_tile_begin,
                                  uint32_t n_chunks, uint64_t* __restrict__ record_total,
                                  uint64_t* __restrict__ chunk_begin) {
  const uint64_t row = static_cast<uint64_t>(n_digits) * n_tiles;
  const uint64_t records = n_tiles ? offsets[row] : 0u;
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c <= n_chunks; c += gridDim.x * blockDim.x) {
    const uint64_t t = chunk_tile_begin[c];
    const uint64_t v = t < n_tiles ? offsets[row + t] : *grand_total;
    if (chunk_begin != nullptr) chunk_begin[c] = v - records;
    if (c == 0) *record_total = records;
  }
}

// Bucket bounds after the pass from column chunks (histogram laid out digit-major over tiles):
// seg_begin[d] = offsets[d * n_tiles] (output position of the first digit-d record), seg_begin[n_digits] = total.
static __global__ void seg_bounds(const uint32_t* __restrict__ offsets, uint64_t n_tiles, uint32_t n_segs,
                           const uint64_t* __restrict__ total, uint32_t* __restrict__ seg_begin) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_segs) seg_begin[p] = n_tiles == 0 ? 0u : offsets[p * n_tiles];
  if (p == n_segs) seg_begin[p] = static_cast<uint32_t>(*total);
}

// Tiles of every segment of a record pass (counts, then an exclusive scan and widen_prefix give seg_tile_begin).
static __global__ void seg_tile_counts(const uint32_t* __restrict__ seg_begin, const uint32_t* __restrict__ seg_end,
                                uint32_t n_segs, uint32_t span, uint32_t* __restrict__ counts) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_segs; i += gridDim.x * blockDim.x) {
    const uint32_t b1 = seg_end ? seg_end[i] : seg_begin[i + 1];
    counts[i] = (b1 - seg_begin[i] + span - 1) / span;
  }
}

static __global__ void widen_prefix(const uint32_t* __restrict__ excl, uint32_t n, const uint64_t* __restrict__ total,
                             uint64_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x)
    out[i] = i < n ? static_cast<uint64_t>(excl[i]) : *total;
}

// Bounds after a record pass: group g (a segment, or for the distributed receiver a bucket whose runs from all
// senders are interleaved in the histogram) splits into n_digits parts; bounds[g * n_digits + d] = output position
// of its first digit-d record, bounds[n_groups * n_digits] = total. Null group arrays: a group is segment g itself
// (histogram at seg_tile_begin[g] * n_digits, output starting where its input starts).
struct Groups {
  const uint64_t* hbase;
  const uint32_t* tiles;
  const uint32_t* out_begin;
};

static __global__ void pass_bounds(const uint32_t* __restrict__ offsets, Segs sg, Groups gr, uint32_t n_groups,
                            uint32_t n_digits, const uint64_t* __restrict__ total, uint32_t* __restrict__ bounds) {
  const uint64_t n = static_cast<uint64_t>(n_groups) * n_digits;
  for (uint64_t p = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; p <= n;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    if (p == n) {
      bounds[p] = static_cast<uint32_t>(*total);
      continue;
    }
    const uint32_t g = static_cast<uint32_t>(p / n_digits), d = static_cast<uint32_t>(p % n_digits);
    const uint64_t hb = gr.hbase ? gr.hbase[g] : sg.seg_tile_begin[g] * n_digits;
    const uint64_t nt = gr.tiles ? gr.tiles[g] : sg.seg_tile_begin[g + 1] - sg.seg_tile_begin[g];
    const uint32_t ob = gr.out_begin ? gr.out_begin[g] : sg.seg_begin[g];
    bounds[p] = nt == 0 ? ob : offsets[hb + d * nt];
  }
}

// ------------------------------------------------------------------------------------------------------------
// Exclusive scan of a uint32 array (decoupled look-back, 8192 elements per workgroup).
// ------------------------------------------------------------------------------------------------------------
constexpr int SCAN_T = 512;
constexpr int SCAN_PER = 16;
constexpr int SCAN_BLOCK = SCAN_T * SCAN_PER;

// Lane t of the workgroup holds the four 4-element groups at (k * SCAN_T + t) * 4, k = 0..3: every load and store
// instruction of a wave then moves 1 KB of consecutive words (16 B per lane). The block's prefix runs over the
// groups in (k, t) order - four workgroup scans - followed by the decoupled look-back across blocks.
// n_dev (optional): the length is min(n, *n_dev * n_mul), read on the device - a record pass's histogram covers the
// tiles that exist (seg_tile_begin's last entry), while the host sizes the grid for the upper bound.
template <bool VEC>
__global__ __launch_bounds__(SCAN_T) void exclusive_scan_u32(const uint32_t* __restrict__ in,
                                                             uint32_t* __restrict__ out, uint64_t n,
                                                             uint64_t* __restrict__ status, uint32_t* ticket,
                                                             uint32_t* error, uint64_t* total_out,
                                                             const uint64_t* __restrict__ n_dev, uint32_t n_mul) {
  static_assert(SCAN_PER == 16, "four groups of four per lane");
  __shared__ uint32_t s_scratch[SCAN_T / WAVE + 1];
  __shared__ uint64_t s_tile;
  __shared__ uint64_t s_prefix;
  if (n_dev != nullptr) n = min(n, *n_dev * n_mul);
  if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint64_t tile = s_tile;
  const uint64_t n_tiles = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
  if (tile >= n_tiles) return;
  const uint64_t base = tile * SCAN_BLOCK;
  const bool full = VEC && base + SCAN_BLOCK <= n;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t e = base + (static_cast<uint64_t>(k) * SCAN_T + threadIdx.x) * 4;
    if (full) {
      v[k] = reinterpret_cast<const uint4*>(in + e)[0];
    } else {
      v[k].x = e < n ? in[e] : 0u;
      v[k].y = e + 1 < n ? in[e + 1] : 0u;
      v[k].z = e + 2 < n ? in[e + 2] : 0u;
      v[k].w = e + 3 < n ? in[e + 3] : 0u;
    }
  }
  uint32_t loc[4], total = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t tk;
    loc[k] = block_exclusive_sum<SCAN_T>(v[k].x + v[k].y + v[k].z + v[k].w, s_scratch, &tk) + total;
    total += tk;
  }
  if (threadIdx.x < WAVE) {
    uint64_t prefix = 0;
    if (tile == 0) {
      if (threadIdx.x == 0) lb_publish(&status[0], LB_FLAG_PREFIX, total);
    } else {
      if (threadIdx.x == 0) lb_publish(&status[tile], LB_FLAG_AGG, total);
      prefix = lb_lookback_wave(status, 0, tile, error);
      if (threadIdx.x == 0) lb_publish(&status[tile], LB_FLAG_PREFIX, prefix + total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == n_tiles - 1 && total_out != nullptr) *total_out = prefix + total;
    }
  }
  __syncthreads();
  const uint32_t pre = static_cast<uint32_t>(s_prefix);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t e = base + (static_cast<uint64_t>(k) * SCAN_T + threadIdx.x) * 4;
    uint4 o;
    o.x = pre + loc[k];
    o.y = o.x + v[k].x;
    o.z = o.y + v[k].y;
    o.w = o.z + v[k].z;
    if (full) {
      reinterpret_cast<uint4*>(out + e)[0] = o;
    } else {
      if (e < n) out[e] = o.x;
      if (e + 1 < n) out[e + 1] = o.y;
      if (e + 2 < n) out[e + 2] = o.z;
      if (e + 3 < n) out[e + 3] = o.w;
    }
  }
}

// Per-partition build + probe, entirely in LDS.
//
// The build records of a partition (up to L = lds_max_build of them) are placed in a bucketed LDS table by a
// counting sort: NB = nb buckets chosen by a key hash independent of the radix bits; pass 1 adds 1 to its bucket's
// size for every record (fire-and-forget LDS adds), a block scan turns sizes into bucket starts, pass 2 claims a slot
// per record with one returning LDS add and stores {key, payload} there. Bucket b then holds entries
// [end[b-1], end[b]). No CAS loops, locks or fences: all inserts of a thread are independent LDS operations.
// A lookup scans one bucket (about two entries) and yields (matches, first matching entry). A key with one build
// row needs nothing else; a key with several build rows is expanded by re-reading the partition's build records in
// order, which reproduces the reference's insertion-ordered PosList (join_hash.cpp:158-175).
//
// A partition with more than L build rows (skewed keys) is processed as consecutive sub-tables of L rows each:
// every probe row's match count is summed over the sub-tables, and its matches are written sub-table by sub-table,
// which is again build order. Nothing ever leaves LDS.
//
// Probe records are loaded once into registers (JP per thread per pass; the host picks JP so that a typical
// partition is one pass) with all loads in flight, matched, counted, and - once one atomic add has reserved the
// partition's output range - written without re-reading them.
// ------------------------------------------------------------------------------------------------------------
// join_partition runs one 1024-thread workgroup per partition, two per CU. (Measured on MI355X at SF100: 256-thread
// workgroups, four per CU by LDS, took 4.4 ms against 1.86 ms - the per-partition phases got longer, not overlapped.)
constexpr int JOIN_THREADS = 1024;
constexpr int JP_PER = 4;                          // probe records per thread per pass (1024-thread workgroups)
constexpr uint32_t LDS_MAX_ROWS = 0xFFFFu;         // entry indexes and counts of one table fit 16 bits

struct JoinDesc {
  const uint32_t* build_begin;  // n_parts + 1
  const uint32_t* probe_begin;  // n_parts + 1
  uint32_t n_parts;
  uint32_t lds_max_build;       // rows per LDS table (larger partitions use several sub-tables)
  int32_t mode;
  RowMap build_map;
  RowMap probe_map;
  uint64_t capacity;            // output capacity in pairs
  uint32_t* error;
  uint32_t* overflow;
  uint64_t* total;              // total pairs (written by the last partition)
  uint64_t* trace;              // debug phase stamps (hy_debug_set_join_trace) or null
  uint32_t* skewed;             // partitions with more build rows than one LDS table (n_parts entries)
  uint32_t* n_skewed;           // their count (zeroed before join_partition)
  uint32_t* multi;              // partitions with more probe records than one pass (n_parts entries)
  uint32_t* n_multi;            // their count (zeroed before join_partition)
  // join_partition_multi: a partition of <= 2 passes whose build side has <= stash_rows rows keeps its first pass's
  // probe payloads and match infos in LDS after a table of stash_rows rows (0: no stash) instead of reloading and
  // re-matching the pass after the count
  uint32_t stash_rows;
};

// Record sources of the partition join: what the last partition pass wrote.
// load_group(i, keys, pays) reads the V records i .. i + V - 1 (i a multiple of V; up to V - 1 records past a side's
// last one may be read and are ignored), so that a lane's consecutive records come in one vector load per array.
template <typename H, typename P>
struct RecSrc {  // {key, payload} records
  using Key = H;
  static constexpr int V = 1;
  const Rec<H, P>* __restrict__ r;
  __device__ __forceinline__ Rec<H, P> operator[](uint32_t i) const { return r[i]; }
  __device__ __forceinline__ void load_group(uint32_t i, H (&k)[V], P (&p)[V]) const {
    const Rec<H, P> x = r[i];
    k[0] = x.key;
    p[0] = x.payload;
  }
};
// Hash records (RecOut's SoA form). murmur2 of a 4-byte key is a bijection: every step of murmur_hash.cpp:36-49, 68-70
// on a 4-byte input - multiplications by the odd constant m, xor-shifts, the xor with (seed ^ 4) * m - is invertible.
// So inside one radix partition (hash & (2^b - 1) fixed) two int32 keys are equal exactly when their hash bits above
// the partition bits are; with b >= 16 those 32 - b <= 16 bits stand in for the key (6 B per record instead of 8).
// GV records per lane and group: GV = 4 loads them with one 8-byte load of their remainders and one 16-byte load of
// their payloads; GV = 1 takes one record per lane (2- and 4-byte loads, the stores of consecutive lanes adjacent).
template <typename P, int GV = 1>
struct HashSrc {
  static_assert(sizeof(P) == 4, "hash records carry 32-bit payloads");
  static_assert(GV == 1 || GV == 4, "groups of 1 or 4 records");
  using Key = uint16_t;
  static constexpr int V = GV;
  const uint16_t* __restrict__ hk;  // 16-byte aligned; readable 3 records past the last
  const P* __restrict__ pay;        // 16-byte aligned; readable 3 records past the last
  __device__ __forceinline__ Rec<uint16_t, P> operator[](uint32_t i) const { return Rec<uint16_t, P>{hk[i], pay[i]}; }
  __device__ __forceinline__ void load_group(uint32_t i, uint16_t (&k)[V], P (&p)[V]) const {
    if constexpr (V == 1) {
      k[0] = hk[i];
      p[0] = pay[i];
    } else {
      const uint2 kk = *reinterpret_cast<const uint2*>(hk + i);
      const uint4 pp = *reinterpret_cast<const uint4*>(pay + i);
      k[0] = static_cast<uint16_t>(kk.x);
      k[1] = static_cast<uint16_t>(kk.x >> 16);
      k[2] = static_cast<uint16_t>(kk.y);
      k[3] = static_cast<uint16_t>(kk.y >> 16);
      p[0] = pp.x;
      p[1] = pp.y;
      p[2] = pp.z;
      p[3] = pp.w;
    }
  }
};

template <typename H, typename P>
struct BTable {
  Rec<H, P>* ents;   // nb entries, bucket by bucket
  uint32_t* end;  // NB bucket ends
  uint32_t nb;
  uint32_t NB;
};

__host__ __device__ inline size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

// LDS bytes of a table over nb build rows
template <typename H, typename P>
__host__ __device__ inline size_t table_bytes(uint32_t nb) {
  return align16(sizeof(Rec<H, P>) * nb) + align16(4 * size_t(nb ? nb : 1));
}

template <typename H, typename P>
__device__ __forceinline__ BTable<H, P> table_at(unsigned char* smem, uint32_t nb) {
  BTable<H, P> t;
  t.nb = nb;
  t.NB = nb ? nb : 1;
  t.ents = reinterpret_cast<Rec<H, P>*>(smem);
  t.end = reinterpret_cast<uint32_t*>(smem + align16(sizeof(Rec<H, P>) * nb));
  return t;
}

template <typename H>
__device__ __forceinline__ uint32_t slot_hash(H key) {
  uint64_t b = 0;
  H k = key;
  if constexpr (std::is_floating_point_v<H>) {
    if (k == H(0)) k = H(0);  // -0.0 and 0.0 compare equal: hash them alike
  }
  __builtin_memcpy(&b, &k, sizeof(H));
  return murmur_final(static_cast<uint32_t>(b) * 0x9E3779B1u ^ static_cast<uint32_t>(b >> 32) * 0x85EBCA77u);
}

template <bool TRACE>
__device__ __forceinline__ void trace_stamp(const JoinDesc& d, uint32_t p, int i) {
  if constexpr (TRACE) {
    if (threadIdx.x == 0) d.trace[5ull * p + i] = wall_clock64();
  }
}

__device__ __forceinline__ uint32_t emitted_for(int mode, uint32_t count) {
  switch (mode) {
    case HY_JOIN_INNER:
      return count;
    case HY_JOIN_LEFT:
    case HY_JOIN_RIGHT:
      return count > 0 ? count : 1u;
    case HY_JOIN_SEMI:
      return count > 0 ? 1u : 0u;
    case HY_JOIN_ANTI:
      return count > 0 ? 0u : 1u;
  }
  return 0u;
}

template <typename H>
__device__ __forceinline__ uint32_t bucket_of(H key, uint32_t NB) {
  return static_cast<uint32_t>((static_cast<uint64_t>(slot_hash<H>(key)) * NB) >> 32);
}

// Builds the LDS table over build records [b0, b0 + n) (n <= LDS_MAX_ROWS). Each thread holds up to build_per<NT>()
// records whose loads are all in flight together - the first batch's while the bucket sizes are being cleared. A
// partition larger than one batch re-reads its records (from L2) for the second counting-sort pass. Ends with a
// barrier.
template <int NT>
constexpr int build_per() {  // >= the largest 4-byte-key table in the default LDS budget / NT
  return NT >= 1024 ? 3 : 14;
}
template <typename Src, typename P, int NT>
__device__ __forceinline__ void build_table(const BTable<typename Src::Key, P>& t, const Src& build, uint32_t b0,
                                            uint32_t n, uint32_t* s_scratch) {
  using H = typename Src::Key;
  constexpr int V = Src::V;                           // consecutive records per lane and group
  constexpr int G = (build_per<NT>() + V - 1) / V;    // groups per lane and batch
  constexpr uint32_t BATCH = G * V * NT;
  // groups start at multiples of V: records [a0, a0 + lead) before the partition are loaded and ignored
  const uint32_t a0 = b0 & ~uint32_t(V - 1), lead = b0 - a0, nr = n + lead;
  H key[G][V];
  P pay[G][V];
  auto load_batch = [&](uint32_t base) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const uint32_t r = base + (q * NT + threadIdx.x) * V;
      if (r < nr) build.load_group(a0 + r, key[q], pay[q]);
    }
  };
  auto in = [&](uint32_t base, int q, int v) {
    const uint32_t r = base + (q * NT + threadIdx.x) * V + v;
    return r >= lead && r < nr;
  };
  load_batch(0);
  for (uint32_t i = threadIdx.x; i < t.NB; i += NT) t.end[i] = 0;
  __syncthreads();
  // pass 1: bucket sizes
  for (uint32_t base = 0; base < nr; base += BATCH) {
    if (base) load_batch(base);
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (in(base, q, v)) atomicAdd(&t.end[bucket_of<H>(key[q][v], t.NB)], 1u);
  }
  __syncthreads();
  // bucket sizes -> bucket starts (each thread owns a contiguous run of buckets)
  const uint32_t per = (t.NB + NT - 1) / NT;
  const uint32_t lo = threadIdx.x * per, hi = min(lo + per, t.NB);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += t.end[i];
  uint32_t total;
  uint32_t run = block_exclusive_sum<NT>(sum, s_scratch, &total);
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = t.end[i];
    t.end[i] = run;
    run += c;
  }
  __syncthreads();
  // pass 2: claim slots; afterwards end[b] is the end of bucket b
  for (uint32_t base = 0; base < nr; base += BATCH) {
    if (base || nr > BATCH) load_batch(base);
#pragma unroll
    for (int q = 0; q < G; ++q) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if (in(base, q, v)) {
          const uint32_t pos = atomicAdd(&t.end[bucket_of<H>(key[q][v], t.NB)], 1u);
          t.ents[pos] = Rec<H, P>{key[q][v], pay[q][v]};
        }
      }
    }
  }
  __syncthreads();
}

// Matches of key in the table, packed as (count << 16) | index of the first matching entry; 0 = no match.
template <typename H, typename P>
__device__ __forceinline__ uint32_t table_lookup(const BTable<H, P>& t, H key) {
  if (t.nb == 0) return 0u;
  const uint32_t b = bucket_of<H>(key, t.NB);
  const uint32_t lo = b ? t.end[b - 1] : 0u, hi = t.end[b];
  uint32_t count = 0, first = 0;
  for (uint32_t i = lo; i < hi; ++i) {
    if (t.ents[i].key == key) {
      if (count == 0) first = i;
      ++count;
    }
  }
  return (count << 16) | first;
}

__device__ __forceinline__ uint32_t info_count(uint32_t info) { return info >> 16; }
__device__ __forceinline__ uint32_t info_index(uint32_t info) { return info & 0xFFFFu; }

// Reserves this partition's output range with one atomic add on the running total. The reference emits one output
// chunk per partition, each with its own PosList (join_hash.cpp:571-590), so partition ranges need not follow
// partition order in the buffer: part_out_begin/count locate each one. Nothing waits on another partition.
// Returns the range start; the block must not write when it ends beyond the capacity (overflow is raised instead,
// and *total still reaches the exact number of pairs required).
__device__ __forceinline__ uint64_t allocate_output(const JoinDesc& d, uint32_t p, uint32_t part_total,
                                                    uint64_t* __restrict__ part_out_begin,
                                                    uint32_t* __restrict__ part_out_count, uint64_t* s_base) {
  if (threadIdx.x == 0) {
    const uint64_t base =
        part_total ? atomicAdd(reinterpret_cast<unsigned long long*>(d.total), static_cast<unsigned long long>(part_total))
                   : 0ull;
    *s_base = base;
    part_out_begin[p] = base;
    part_out_count[p] = part_total;
    if (base + part_total > d.capacity) atomicOr(d.overflow, 1u);
  }
  __syncthreads();
  return *s_base;
}

// Output offsets of one pass's records (k, thread): records (k' < k) first, then waves (w' < w), then lanes.
// Leaves per-(k, wave) offsets in s_tot (valid until the caller's next barrier) and returns the pass total; a
// record's position is then record_pos(e, k, s_tot).
template <int JP, int NT, typename EF>
__device__ __forceinline__ uint32_t pass_offsets(EF e_of, uint32_t* s_tot) {
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
#pragma unroll
  for (int k = 0; k < JP; ++k) {
    const uint32_t e = e_of(k);
    // common case (unique build keys): every record emits 0 or 1 pairs -> a ballot count is the wave total
    const uint32_t total = __ballot(e > 1) ? wave_sum(e) : static_cast<uint32_t>(__popcll(__ballot(e != 0)));
    if (lane == 0) s_tot[k * (NT / WAVE) + w] = total;
  }
  __syncthreads();
  if (threadIdx.x < WAVE) {  // exclusive prefix over the JP * (NT / WAVE) wave totals, (k, w) order
    constexpr int N = JP * (NT / WAVE);
    constexpr int PER_LANE = (N + WAVE - 1) / WAVE;
    uint32_t v[PER_LANE], sum = 0;
#pragma unroll
    for (int q = 0; q < PER_LANE; ++q) {
      const int idx = lane * PER_LANE + q;
      v[q] = idx < N ? s_tot[idx] : 0u;
      sum += v[q];
    }
    const uint32_t incl = wave_inclusive_sum(sum);
    uint32_t runl = incl - sum;
#pragma unroll
    for (int q = 0; q < PER_LANE; ++q) {
      const int idx = lane * PER_LANE + q;
      if (idx < N) s_tot[idx] = runl;
      runl += v[q];
    }
    if (lane == WAVE - 1) s_tot[N] = incl;
  }
  __syncthreads();
  return s_tot[JP * (NT / WAVE)];
}

template <int JP, int NT>
__device__ __forceinline__ uint32_t record_pos(uint32_t e, int k, const uint32_t* s_tot) {
  const uint32_t before = __ballot(e > 1) ? wave_inclusive_sum(e) - e
                                          : static_cast<uint32_t>(__popcll(__ballot(e != 0) & lanemask_lt()));
  return s_tot[k * (NT / WAVE) + threadIdx.x / WAVE] + before;
}

// Writes the build rows with `key` among build records [b0, b0 + n) in order, each paired with prow.
template <typename Src>
__device__ __forceinline__ void write_duplicates(const JoinDesc& d, const Src& build, uint32_t b0, uint32_t n,
                                                 typename Src::Key key, uint32_t count, hy_row_id prow, uint64_t o,
                                                 hy_row_id* __restrict__ out_build, hy_row_id* __restrict__ out_probe) {
  for (uint32_t i = 0, m = 0; i < n && m < count; ++i) {
    const auto br = build[b0 + i];
    if (br.key == key) {
      put_row(out_build + (o), map_row(d.build_map, br.payload));
      put_row(out_probe + (o), prow);
      ++o;
      ++m;
    }
  }
}

// A partition whose build side fits one LDS table. Its probe records fit one pass of JP per thread in the common case
// (!MULTI; join_partition defers the others to join_partition_multi): the table is built once and every probe
// record's (count, first entry) stays in registers from counting to writing. A lane takes its records in groups of
// Src::V consecutive ones (JP / V groups per pass), so the records' order is (pass, group, thread, record in group):
// pass_offsets places the groups, a lane its group's records one after the other.
template <typename Src, typename P, bool TRACE, int JP, int NT, bool MULTI = false>
__device__ __forceinline__ void partition_one_table(const JoinDesc& d, uint32_t p, unsigned char* smem,
                                                    const Src& build, const Src& probe,
                                                    hy_row_id* __restrict__ out_build, hy_row_id* __restrict__ out_probe,
                                                    uint64_t* __restrict__ part_out_begin,
                                                    uint32_t* __restrict__ part_out_count, uint32_t* s_tot,
                                                    uint64_t* s_base) {
  using H = typename Src::Key;
  constexpr int V = Src::V;
  constexpr int K = JP / V;  // groups per thread per pass
  static_assert(K * V == JP, "JP is a multiple of the group size");
  const uint32_t bb = d.build_begin[p], nb = d.build_begin[p + 1] - bb;
  const uint32_t pb = d.probe_begin[p], np = d.probe_begin[p + 1] - pb;
  const int mode = d.mode;
  const BTable<H, P> t = table_at<H, P>(smem, nb);
  // groups start at multiples of V: probe records [a0, a0 + lead) before the partition are loaded and ignored
  const uint32_t a0 = pb & ~uint32_t(V - 1), lead = pb - a0, nr = np + lead;
  constexpr uint32_t JP_PASS_ = JP * NT;  // (!MULTI: nr <= JP_PASS_, one pass)
  auto rel = [&](uint32_t pass, int k, int v) { return pass * JP_PASS_ + (k * NT + threadIdx.x) * V + v; };
  auto in = [&](uint32_t pass, int k, int v) {
    const uint32_t r = rel(pass, k, v);
    return r >= lead && r < nr;
  };
  // Per probe record only its payload and match info (count << 16 | first entry) stay in registers.
  H key[K][V];
  P ppay[K][V];
  uint32_t pinfo[K][V];
  auto load = [&](uint32_t pass) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (rel(pass, k, 0) < nr) probe.load_group(a0 + rel(pass, k, 0), key[k], ppay[k]);
  };
  auto match = [&](uint32_t pass) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) pinfo[k][v] = in(pass, k, v) ? table_lookup<H, P>(t, key[k][v]) : 0u;
  };
  auto emit = [&](uint32_t pass, int k, int v) { return in(pass, k, v) ? emitted_for(mode, info_count(pinfo[k][v])) : 0u; };

  // records of <= 8 bytes: the first pass's probe records are in flight while the table is built (wider ones would
  // spill at this kernel's register budget)
  constexpr bool PREFETCH = !MULTI && sizeof(Rec<H, P>) <= 8;
  if (PREFETCH) load(0);
  build_table<Src, P, NT>(t, build, bb, nb, s_tot);
  trace_stamp<TRACE>(d, p, 1);

  auto e_of = [&](uint32_t pass, int k) {
    uint32_t e = 0;
#pragma unroll
    for (int v = 0; v < V; ++v) e += emit(pass, k, v);
    return e;
  };
  // writes the pairs of one pass from `run` on (pass_offsets has left the pass's per-(group, wave) offsets in s_tot)
  auto write_pass = [&](uint32_t pass, uint64_t run) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      uint64_t o = run + record_pos<K, NT>(e_of(pass, k), k, s_tot);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const uint32_t c = info_count(pinfo[k][v]);
        const uint32_t e = emit(pass, k, v);
        if (e == 0) continue;
        const hy_row_id prow = map_row(d.probe_map, ppay[k][v]);
        if (mode == HY_JOIN_SEMI || mode == HY_JOIN_ANTI) {
          put_row(out_probe + (o), prow);
        } else if (c == 0) {  // outer: probe row without a match
          put_row(out_build + (o), hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu});
          put_row(out_probe + (o), prow);
        } else if (c == 1) {
          put_row(out_build + (o), map_row(d.build_map, t.ents[info_index(pinfo[k][v])].payload));
          put_row(out_probe + (o), prow);
        } else {
          write_duplicates<Src>(d, build, bb, nb, t.ents[info_index(pinfo[k][v])].key, c, prow, o, out_build,
                                out_probe);
        }
        o += e;
      }
    }
  };

  if constexpr (!MULTI) {
    // one pass (join_partition defers larger partitions): one scan over the records' emit counts gives the
    // partition's total and every record's position
    if (!PREFETCH) load(0);
    match(0);
    trace_stamp<TRACE>(d, p, 2);
    const uint32_t part_total = pass_offsets<K, NT>([&](int k) { return e_of(0, k); }, s_tot);
    const uint64_t obase = allocate_output(d, p, part_total, part_out_begin, part_out_count, s_base);
    trace_stamp<TRACE>(d, p, 3);
    if (obase + part_total > d.capacity) return;
    write_pass(0, obase);
  } else {
    const uint32_t n_pass = (nr + JP_PASS_ - 1) / JP_PASS_;
    if (n_pass <= 1 || (n_pass == 2 && nb <= d.stash_rows)) {
      // one pass, or two with the first one's payloads and match infos stashed in LDS (thread-private slots after the
      // table): every record is loaded and matched once; the second pass is written from registers behind the first
      // one's total, then the first pass is restored and written at the range's start
      load(0);
      match(0);
      uint32_t my0 = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) my0 += e_of(0, k);
      if (n_pass <= 1) {
        const uint32_t part_total = pass_offsets<K, NT>([&](int k) { return e_of(0, k); }, s_tot);
        const uint64_t obase = allocate_output(d, p, part_total, part_out_begin, part_out_count, s_base);
        if (obase + part_total > d.capacity) return;
        write_pass(0, obase);
        return;
      }
      P* st_pay = reinterpret_cast<P*>(smem + table_bytes<H, P>(d.stash_rows));
      uint32_t* st_info = reinterpret_cast<uint32_t*>(st_pay + JP_PASS_);
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          st_pay[(k * V + v) * NT + threadIdx.x] = ppay[k][v];
          st_info[(k * V + v) * NT + threadIdx.x] = pinfo[k][v];
        }
      load(1);
      match(1);
      uint32_t my1 = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) my1 += e_of(1, k);
      uint32_t total0, total1;
      block_exclusive_sum<NT>(my0, s_tot, &total0);
      block_exclusive_sum<NT>(my1, s_tot, &total1);
      const uint64_t obase = allocate_output(d, p, total0 + total1, part_out_begin, part_out_count, s_base);
      if (obase + total0 + total1 > d.capacity) return;
      pass_offsets<K, NT>([&](int k) { return e_of(1, k); }, s_tot);
      write_pass(1, obase + total0);
      __syncthreads();  // s_tot is reused by the first pass's offsets
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          ppay[k][v] = st_pay[(k * V + v) * NT + threadIdx.x];
          pinfo[k][v] = st_info[(k * V + v) * NT + threadIdx.x];
        }
      pass_offsets<K, NT>([&](int k) { return e_of(0, k); }, s_tot);
      write_pass(0, obase);
      return;
    }
    // more passes: count them all, reserve the partition's range, then reload, match and write pass by pass
    uint32_t my = 0;
    for (uint32_t pass = 0; pass < n_pass; ++pass) {
      if (pass || !PREFETCH) load(pass);
      match(pass);
#pragma unroll
      for (int k = 0; k < K; ++k) my += e_of(pass, k);
    }
    uint32_t part_total;
    block_exclusive_sum<NT>(my, s_tot, &part_total);
    const uint64_t obase = allocate_output(d, p, part_total, part_out_begin, part_out_count, s_base);
    if (obase + part_total > d.capacity) return;
    uint64_t run = obase;
    for (uint32_t pass = 0; pass < n_pass; ++pass) {
      load(pass);
      match(pass);
      const uint32_t pass_total = pass_offsets<K, NT>([&](int k) { return e_of(pass, k); }, s_tot);
      write_pass(pass, run);
      run += pass_total;
      __syncthreads();  // s_tot is reused by the next pass
    }
  }
}

// A partition with more build rows than one LDS table holds (skewed keys): consecutive sub-tables of L build rows.
// Counts are summed over the sub-tables; matches are written sub-table by sub-table, i.e. in build order. Each
// probe pass rebuilds the sub-tables twice (count, write), a cost only skewed partitions pay.
constexpr int JS_PER = 2;  // probe records per thread per pass of a skewed partition (1024-thread workgroups)
template <typename Src, typename P, int NT>
__device__ __forceinline__ void partition_sub_tables(const JoinDesc& d, uint32_t p, unsigned char* smem,
                                                     const Src& build, const Src& probe,
                                                     hy_row_id* __restrict__ out_build, hy_row_id* __restrict__ out_probe,
                                                     uint64_t* __restrict__ part_out_begin,
                                                     uint32_t* __restrict__ part_out_count, uint32_t* s_tot,
                                                     uint64_t* s_base) {
  using H = typename Src::Key;
  const uint32_t bb = d.build_begin[p], nb = d.build_begin[p + 1] - bb;
  const uint32_t pb = d.probe_begin[p], np = d.probe_begin[p + 1] - pb;
  const uint32_t L = d.lds_max_build;
  const uint32_t n_sub = (nb + L - 1) / L;
  const int mode = d.mode;
  constexpr int JS = JS_PER;
  constexpr uint32_t JS_PASS = JS * NT;
  const uint32_t n_pass = (np + JS_PASS - 1) / JS_PASS;

  Rec<H, P> pr[JS];
  uint32_t pcn[JS];
  auto load_and_count = [&](uint32_t pass) {
#pragma unroll
    for (int k = 0; k < JS; ++k) {
      const uint32_t j = pass * JS_PASS + k * NT + threadIdx.x;
      if (j < np) pr[k] = probe[pb + j];
      pcn[k] = 0;
    }
    for (uint32_t sub = 0; sub < n_sub; ++sub) {
      const uint32_t b0 = bb + sub * L, n = (sub + 1 == n_sub) ? nb - sub * L : L;
      const BTable<H, P> t = table_at<H, P>(smem, n);
      build_table<Src, P, NT>(t, build, b0, n, s_tot);
#pragma unroll
      for (int k = 0; k < JS; ++k) {
        const uint32_t j = pass * JS_PASS + k * NT + threadIdx.x;
        if (j < np) pcn[k] += info_count(table_lookup<H, P>(t, pr[k].key));
      }
      __syncthreads();  // before the next table overwrites LDS
    }
  };

  uint32_t my = 0;
  for (uint32_t pass = 0; pass < n_pass; ++pass) {
    load_and_count(pass);
#pragma unroll
    for (int k = 0; k < JS; ++k) {
      const uint32_t j = pass * JS_PASS + k * NT + threadIdx.x;
      if (j < np) my += emitted_for(mode, pcn[k]);
    }
  }
  uint32_t part_total;
  block_exclusive_sum<NT>(my, s_tot, &part_total);
  const uint64_t obase = allocate_output(d, p, part_total, part_out_begin, part_out_count, s_base);
  if (obase + part_total > d.capacity) return;

  uint64_t run = obase;
  for (uint32_t pass = 0; pass < n_pass; ++pass) {
    if (n_pass > 1) load_and_count(pass);
    auto e_of = [&](int k) {
      const uint32_t j = pass * JS_PASS + k * NT + threadIdx.x;
      return j < np ? emitted_for(mode, pcn[k]) : 0u;
    };
    const uint32_t pass_total = pass_offsets<JS, NT>(e_of, s_tot);
    uint32_t pos[JS];
#pragma unroll
    for (int k = 0; k < JS; ++k) {
      const uint32_t e = e_of(k);
      pos[k] = record_pos<JS, NT>(e, k, s_tot);
      if (e == 0) continue;
      if (mode == HY_JOIN_SEMI || mode == HY_JOIN_ANTI) {
        put_row(out_probe + (run + pos[k]), map_row(d.probe_map, pr[k].payload));
      } else if (pcn[k] == 0) {
        put_row(out_build + (run + pos[k]), hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu});
        put_row(out_probe + (run + pos[k]), map_row(d.probe_map, pr[k].payload));
      }
    }
    __syncthreads();  // s_tot consumed; LDS table region free
    if (mode != HY_JOIN_SEMI && mode != HY_JOIN_ANTI) {
      for (uint32_t sub = 0; sub < n_sub; ++sub) {
        const uint32_t b0 = bb + sub * L, n = (sub + 1 == n_sub) ? nb - sub * L : L;
        const BTable<H, P> t = table_at<H, P>(smem, n);
        build_table<Src, P, NT>(t, build, b0, n, s_tot);
#pragma unroll
        for (int k = 0; k < JS; ++k) {
          const uint32_t j = pass * JS_PASS + k * NT + threadIdx.x;
          if (j >= np || pcn[k] == 0) continue;
          const uint32_t info = table_lookup<H, P>(t, pr[k].key);
          const uint32_t cnt = info_count(info);
          if (cnt == 0) continue;
          const hy_row_id prow = map_row(d.probe_map, pr[k].payload);
          const uint64_t o = run + pos[k];
          if (cnt == 1) {
            put_row(out_build + (o), map_row(d.build_map, t.ents[info_index(info)].payload));
            put_row(out_probe + (o), prow);
          } else {
            write_duplicates<Src>(d, build, b0, n, pr[k].key, cnt, prow, o, out_build, out_probe);
          }
          pos[k] += cnt;
        }
        __syncthreads();  // before the next table overwrites LDS
      }
    }
    run += pass_total;
  }
}

// One 1024-thread workgroup per partition whose build side fits one LDS table and whose probe records fit one pass -
// every partition unless keys are skewed. Any other partition is appended to d.skewed and left to
// join_partition_skewed, so that this kernel carries only the fast path's registers (the sub-table and multi-pass
// paths would spill at this kernel's 8-waves-per-SIMD budget).
template <typename Src, typename P, bool TRACE, int JP, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT >= 1024 ? 8 : 4, 8))) void join_partition(
    JoinDesc d, Src build, Src probe, hy_row_id* __restrict__ out_build, hy_row_id* __restrict__ out_probe,
    uint64_t* __restrict__ part_out_begin, uint32_t* __restrict__ part_out_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t s_tot[JP * (NT / WAVE) + 1];
  __shared__ uint64_t s_base;
  const uint32_t p = blockIdx.x;
  if (p >= d.n_parts) return;
  if (d.build_begin[p + 1] - d.build_begin[p] > d.lds_max_build) {
    if (threadIdx.x == 0) d.skewed[atomicAdd(d.n_skewed, 1u)] = p;
    return;
  }
  // (the probe records of one pass start at a multiple of the group size: up to V - 1 leading ones are skipped)
  if (d.probe_begin[p + 1] - d.probe_begin[p] + (Src::V - 1) > static_cast<uint32_t>(JP * NT)) {
    if (threadIdx.x == 0) d.multi[atomicAdd(d.n_multi, 1u)] = p;
    return;
  }
  trace_stamp<TRACE>(d, p, 0);
  partition_one_table<Src, P, TRACE, JP, NT>(d, p, smem, build, probe, out_build, out_probe, part_out_begin,
                                             part_out_count, s_tot, &s_base);
  trace_stamp<TRACE>(d, p, 4);
}

// Partitions with more probe records than one pass of join_partition (their build side fits one table): a grid of at
// most two workgroups per CU loops over the list join_partition wrote (launched after it on the same stream) - or,
// with d.multi null (the host expects most partitions to need several passes), one workgroup per partition instead of
// join_partition.
template <typename Src, typename P, int JP, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT >= 1024 ? 8 : 4, 8))) void join_partition_multi(
    JoinDesc d, Src build, Src probe, hy_row_id* __restrict__ out_build, hy_row_id* __restrict__ out_probe,
    uint64_t* __restrict__ part_out_begin, uint32_t* __restrict__ part_out_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t s_tot[JP * (NT / WAVE) + 1];
  __shared__ uint64_t s_base;
  if (d.multi == nullptr) {  // every partition (most need several passes): one workgroup each, skewed ones deferred
    const uint32_t p = blockIdx.x;
    if (p >= d.n_parts) return;
    if (d.build_begin[p + 1] - d.build_begin[p] > d.lds_max_build) {
      if (threadIdx.x == 0) d.skewed[atomicAdd(d.n_skewed, 1u)] = p;
      return;
    }
    partition_one_table<Src, P, false, JP, NT, true>(d, p, smem, build, probe, out_build, out_probe, part_out_begin,
                                                     part_out_count, s_tot, &s_base);
    return;
  }
  const uint32_t n = *d.n_multi;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    partition_one_table<Src, P, false, JP, NT, true>(d, d.multi[i], smem, build, probe, out_build, out_probe,
                                                     part_out_begin, part_out_count, s_tot, &s_base);
    __syncthreads();  // s_tot / s_base / LDS reused by the next partition
  }
}

// The skewed partitions join_partition listed (launched after it on the same stream): a small grid loops over them,
// each as consecutive LDS sub-tables and probe passes of JS_PER records per thread.
// Partition ranges are located by part_out_begin / count, so their order in the buffer does not matter.
template <typename Src, typename P, int NT>
__global__ __launch_bounds__(NT) void join_partition_skewed(JoinDesc d, Src build, Src probe,
                                                            hy_row_id* __restrict__ out_build,
                                                            hy_row_id* __restrict__ out_probe,
                                                            uint64_t* __restrict__ part_out_begin,
                                                            uint32_t* __restrict__ part_out_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t s_tot[JS_PER * (NT / WAVE) + 1];
  __shared__ uint64_t s_base;
  const uint32_t n = *d.n_skewed;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    partition_sub_tables<Src, P, NT>(d, d.skewed[i], smem, build, probe, out_build, out_probe, part_out_begin,
                                     part_out_count, s_tot, &s_base);
    __syncthreads();  // s_tot / s_base / LDS reused by the next partition
  }
}

static __global__ void murmur_kernel_u32(const uint32_t* keys, uint64_t n, uint32_t seed, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = murmur2_u32(keys[i], seed);
}

static __global__ void murmur_kernel_u64(const uint64_t* keys, uint64_t n, uint32_t seed, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = murmur2_u64(keys[i], seed);
}

// Dereference join outputs of a reference input through its per-chunk PosLists (write_output_columns,
// join_hash.cpp:584-592): out[i] = row is NULL ? row : chunk_pos_lists[row.chunk_id][row.chunk_offset].
static __global__ void dereference_kernel(const hy_row_id* __restrict__ rows, uint64_t n,
                                   const hy_row_id* const* __restrict__ chunk_pos_lists, hy_row_id* __restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const hy_row_id r = rows[i];
    out[i] = r.chunk_offset == 0xFFFFFFFFu ? r : chunk_pos_lists[r.chunk_id][r.chunk_offset];
  }
}

}  // namespace hyk
