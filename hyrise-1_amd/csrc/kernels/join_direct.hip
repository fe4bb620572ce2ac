// Direct partitioning of a JoinHash side with a fused TableScan (the headline's lineitem side): the first radix pass
// reads the predicate ids and the join keys ONCE and writes every record straight into a region of its own (span,
// bucket) - no compacted record buffer written and read back (part1_compact + part1_spread, join.hip), no per-tile
// histogram of the first digit. The second pass then reads each bucket as the concatenation of its spans' regions in
// span (= row) order, so both passes stay stable and the output order is the reference's (join_hash.cpp:287-355:
// partition-major, rows in (chunk, offset) order inside a partition).
//
//   span_match_count  : scan matches per span (1 B of predicate id per row) and the span's region capacity; two small
//                       exclusive scans turn them into each span's first scan-output position and first record index.
//   part1_direct      : one workgroup per span (S consecutive tiles of one chunk): predicate + key per row, the scan
//                       output in row order (chunk offsets at the span's scan position), the records ranked by their
//                       first digit (wave_rank_add) and stored through the LDS stage into region (span, digit) - a
//                       region is sized from the span's match count (direct_cap), so no workgroup waits on another.
//                       A region that would overflow (keys far more skewed than murmur2 spreads them) sets a flag and
//                       the host reruns the join on the classic passes.
//   part2g_hist       : per (bucket, group of spans) histogram of the second digit from the digit bytes part1_direct
//                       wrote beside the records (256 x 256 x H counters in all, not one row per tile).
//   part2g_scatter    : one workgroup per (bucket, group): its spans' regions as one virtual sequence, 4096-record tiles,
//                       stable scatter by the second digit into the final partitions (hash records for int32 keys).
//
// Traffic per matched row at SF100 (u8 predicate ids, int32 keys): 1 + 4 B read per row in both first-pass kernels
// (ids twice), 8 B record + 1 B digit + 4 B scan offset written; the second pass reads 1 + 8 B and writes 6 B.
#pragma once

namespace hyk {

// Records per (span, bucket) region for a span with m matching rows: the mean plus eight standard deviations of a
// bucket count whose keys come in clusters of up to ~7 equal keys (variance <= 5 x mean: TPC-H lineitem's orderkeys),
// plus a constant. Monotonic in m, so the host sizes the workspace from the span's row count.
__host__ __device__ inline uint32_t direct_cap(uint32_t m, uint32_t n_digits) {
  const uint32_t mean = (m + n_digits - 1) / n_digits;
  const uint32_t x = 5u * mean;
  uint32_t r = static_cast<uint32_t>(sqrtf(static_cast<float>(x)));
  while (r * r > x) --r;
  while ((r + 1) * (r + 1) <= x) ++r;
  return mean + 8u * (r + 1u) + 32u;
}

// Spans of the direct pass and where their output goes.
struct DirectGeo {
  const uint64_t* span_rbase;  // n_spans: first record index of the span's regions (regions: digit-major, cap each)
  const uint32_t* span_cap;    // n_spans: records per region
  const uint32_t* span_scan;   // n_spans: the span's first position in the scan output
  uint32_t* counts;            // [digit * n_spans + span]: records written into each region
  uint32_t* overflow;          // set when a region would overflow
  uint32_t n_spans;
};

// Matches of each span's rows (one workgroup per span), the span's region capacity (direct_cap) and n_digits x it.
template <int FK>
__global__ __launch_bounds__(PART_THREADS) void span_match_count(Side s, uint32_t n_digits, uint32_t* __restrict__ cnt,
                                                                 uint32_t* __restrict__ cap,
                                                                 uint32_t* __restrict__ cap_words) {
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  const uint64_t span = blockIdx.x;
  const uint32_t c = s.tile_chunk[span];
  const uint32_t size = s.chunks[c].size;
  const uint32_t base = static_cast<uint32_t>(span - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  uint32_t n = 0;
  if constexpr (FK == FK_DICT8 || FK == FK_DICT16 || FK == FK_DICT32) {
    // 16 consecutive ids per thread in 16-byte vector loads (the ranking layout of the partition passes is not
    // needed for a count)
    using E = std::conditional_t<FK == FK_DICT8, uint8_t, std::conditional_t<FK == FK_DICT16, uint16_t, uint32_t>>;
    const hy_scan_chunk f = s.filter[c];
    if (f.op != HY_OP_NONE && f.column.size != 0) {
#pragma unroll 1
      for (uint32_t j = 0; j < n_sub; ++j)
        n += __popc(filter_dict_contig<E>(f, base + j * PART_TILE + threadIdx.x * PART_ITEMS));
    }
  } else {
#pragma unroll 1
    for (uint32_t j = 0; j < n_sub; ++j) n += __popc(filter_items<FK>(s, c, base + j * PART_TILE + w * WAVE_SPAN));
  }
  uint32_t total;
  block_exclusive_sum<PART_THREADS>(n, s_scratch, &total);
  if (threadIdx.x == 0) {
    const uint32_t k = direct_cap(total, n_digits);
    cnt[span] = total;
    cap[span] = k;
    cap_words[span] = k * n_digits;
  }
}

// The fused scan's per-chunk output begins (n_chunks + 1, in matches) from the spans' exclusive prefix: chunk c starts
// where its first span starts (a chunk without spans where the next one does).
static __global__ void direct_chunk_begin(const uint32_t* __restrict__ span_scan, uint32_t n_spans,
                                          const uint64_t* __restrict__ chunk_span_begin, uint32_t n_chunks,
                                          const uint64_t* __restrict__ total, uint64_t* __restrict__ chunk_begin) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c <= n_chunks; c += gridDim.x * blockDim.x) {
    const uint64_t t = chunk_span_begin[c];
    chunk_begin[c] = t < n_spans ? span_scan[t] : *total;
  }
}

// span_rbase as 64-bit record indexes from the 32-bit exclusive scan of the capacities (the regions of all spans
// together stay below 2^32 records: the host checks the bound).
static __global__ void widen_u32(const uint32_t* __restrict__ in, uint32_t n, uint64_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = in[i];
}

// staged_scatter (join.hip) for a workgroup whose digit-d output is a region of `cap` records starting at d * cap:
// `run` (thread d) starts at d * cap. A tile that would run past a region's end writes nothing and raises *overflow;
// every later tile of the workgroup does the same (s_ovf stays set).
template <typename H, typename P>
__device__ __forceinline__ void staged_scatter_capped(const Rec<H, P> (&recs)[PART_ITEMS], uint32_t act,
                                                      const uint32_t (&dr)[PART_ITEMS], uint32_t (*s_cnt)[256],
                                                      uint32_t* s_delta, Rec<H, P>* s_stage, uint32_t* s_scratch,
                                                      uint32_t* s_ovf, uint32_t n_digits, uint32_t cap,
                                                      const Digit& dg, const NextDigit& nd, uint32_t& run,
                                                      const RecOut<H, P>& out, uint32_t* overflow) {
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
  const uint32_t loc = block_exclusive_sum<PART_THREADS>(tot, s_scratch, &total);
  if (d < n_digits) {
#pragma unroll
    for (int ww = 0; ww < PART_WAVES; ++ww) s_cnt[ww][d] += loc;
    s_delta[d] = run - loc;
    if (run + tot > (d + 1) * cap) *s_ovf = 1u;
    run += tot;
  }
  __syncthreads();
  if (*s_ovf) {
    if (threadIdx.x == 0) __hip_atomic_store(overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
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

// First radix pass with the fused scan, one workgroup per span (see the file comment). recs / nd.bytes: the regions'
// records and digit bytes, indexed by record (span_rbase[span] + d * cap + i).
template <typename SD, typename T, typename H, int LP, int FK>
__global__ __launch_bounds__(PART_THREADS) void part1_direct(Side s, Digit dg, NextDigit nd, uint32_t n_digits,
                                                            DirectGeo g, Rec<H, uint32_t>* __restrict__ recs) {
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ uint32_t s_sc[WAVE + 2];
  __shared__ uint32_t s_ovf;
  __shared__ Rec<H, uint32_t> s_stage[PART_TILE];
  const uint32_t span = xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t c = s.tile_chunk[span];
  const SrcChunk ch = s.chunks[c];
  const uint32_t base = static_cast<uint32_t>(span - s.chunk_tile_begin[c]) * (s.sub * PART_TILE);
  const uint32_t n_sub = min(s.sub, (ch.size - base + PART_TILE - 1) / PART_TILE);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  const uint32_t cap = g.span_cap[span];
  const uint64_t rbase = g.span_rbase[span];
  const RecOut<H, uint32_t> out{recs + rbase, nullptr, nullptr, 0u, nullptr, 0u};
  NextDigit ndl = nd;
  if (ndl.bytes != nullptr) ndl.bytes += rbase;
  uint32_t run = threadIdx.x < n_digits ? threadIdx.x * cap : 0u;
  uint32_t scan_pos = g.span_scan[span];
  if (threadIdx.x == 0) s_ovf = 0;
#pragma unroll 1
  for (uint32_t j = 0; j < n_sub; ++j) {
    __syncthreads();  // the previous tile's write-out has read s_stage / s_sc
    clear_wave_counts(s_cnt[w]);
    const uint32_t rb = base + j * PART_TILE + w * WAVE_SPAN;
    const uint32_t m_scan = filter_items<FK>(s, c, rb);
    H keys[PART_ITEMS];
    uint32_t pays[PART_ITEMS];
    const uint32_t act = load_items<T, H, uint32_t, LP>(s, ch, rb, keys, pays) & m_scan;
    // the scan's output in row order: (wave, item) ballot counts -> prefix -> lane rank
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const uint64_t b = __ballot((m_scan >> k) & 1u);
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
    if (s.scan_out != nullptr) {
#pragma unroll
      for (int k = 0; k < PART_ITEMS; ++k) {
        const uint64_t b = __ballot((m_scan >> k) & 1u);
        if ((m_scan >> k) & 1u)
          s.scan_out[scan_pos + s_sc[w * PART_ITEMS + k] + static_cast<uint32_t>(__popcll(b & lanemask_lt()))] =
              rb + k * WAVE + lane;
      }
    }
    scan_pos += s_sc[WAVE];
    uint32_t dr[PART_ITEMS];
    Rec<H, uint32_t> r[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, keys[k]) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
      r[k].key = keys[k];
      r[k].payload = pays[k];
    }
    staged_scatter_capped<H, uint32_t>(r, act, dr, s_cnt, s_delta, s_stage, s_scratch, &s_ovf, n_digits, cap, dg, ndl,
                                       run, out, g.overflow);
  }
  // (after an overflow the counts are clamped to the regions, so that the passes after this one stay in bounds)
  if (threadIdx.x < n_digits)
    g.counts[threadIdx.x * g.n_spans + span] = min(run - threadIdx.x * cap, cap);
}

// ------------------------------------------------------------------------------------------------------------
// Second pass over (bucket, group) run lists. Group h of bucket b is the regions of spans [h * per, (h + 1) * per)
// in span order; its records form one virtual sequence, cut into 4096-record tiles.
// ------------------------------------------------------------------------------------------------------------
constexpr uint32_t GROUP_MAX_RUNS = 1024;

struct GroupGeo {
  const uint64_t* span_rbase;
  const uint32_t* span_cap;
  const uint32_t* counts;  // [bucket * n_spans + span]
  uint32_t n_spans;
  uint32_t n_groups;       // H
  uint32_t per;            // spans per group (<= GROUP_MAX_RUNS)
};

// Loads the workgroup's runs: s_pre[r] = exclusive prefix of their counts (s_pre[nr] = total), s_base[r] = record
// index of run r's first record. Returns nr. Ends with a barrier.
__device__ __forceinline__ uint32_t load_group_runs(const GroupGeo& gg, uint32_t b, uint32_t h, uint32_t* s_pre,
                                                    uint64_t* s_base, uint32_t* s_scratch) {
  const uint32_t s0 = h * gg.per;
  const uint32_t nr = s0 >= gg.n_spans ? 0u : min(gg.per, gg.n_spans - s0);
  constexpr uint32_t PER = GROUP_MAX_RUNS / PART_THREADS;  // runs per thread
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t r = threadIdx.x * PER + q;
    v[q] = r < nr ? gg.counts[static_cast<uint64_t>(b) * gg.n_spans + s0 + r] : 0u;
    if (r < nr) s_base[r] = gg.span_rbase[s0 + r] + static_cast<uint64_t>(b) * gg.span_cap[s0 + r];
    sum += v[q];
  }
  uint32_t total;
  uint32_t run = block_exclusive_sum<PART_THREADS>(sum, s_scratch, &total);
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t r = threadIdx.x * PER + q;
    if (r <= nr) s_pre[r] = run;
    run += v[q];
  }
  if (threadIdx.x == 0) s_pre[nr] = total;
  __syncthreads();
  return nr;
}

// The run holding virtual index v (s_pre[r] <= v < s_pre[r + 1]), searched from the run `r` of a smaller index.
__device__ __forceinline__ uint32_t advance_run(const uint32_t* s_pre, uint32_t nr, uint32_t r, uint32_t v) {
  while (r + 1 < nr && s_pre[r + 1] <= v) ++r;
  return r;
}
__device__ __forceinline__ uint32_t find_run(const uint32_t* s_pre, uint32_t nr, uint32_t v) {
  uint32_t lo = 0, hi = nr;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s_pre[mid] <= v)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Record indexes of this lane's PART_ITEMS items of a tile (virtual indexes v0 + k * WAVE, clamped to the last record
// of the group): addr[k]. Returns the in-range mask.
__device__ __forceinline__ uint32_t group_item_addrs(const uint32_t* s_pre, const uint64_t* s_base, uint32_t nr,
                                                     uint32_t n, uint32_t v0, uint64_t (&addr)[PART_ITEMS]) {
  uint32_t act = 0;
  uint32_t v = min(v0, n - 1);
  uint32_t r = find_run(s_pre, nr, v);
#pragma unroll
  for (int k = 0; k < PART_ITEMS; ++k) {
    const uint32_t vk = v0 + k * WAVE;
    const uint32_t vc = min(vk, n - 1);
    r = advance_run(s_pre, nr, r, vc);
    addr[k] = s_base[r] + (vc - s_pre[r]);
    if (vk < n) act |= 1u << k;
  }
  return act;
}

// Digit histogram of each (bucket, group) from the digit bytes: hist[(b * n_digits + d) * H + h].
template <typename SD>
__global__ __launch_bounds__(PART_THREADS) void part2g_hist(GroupGeo gg, uint32_t n_digits, const uint8_t* __restrict__ dig,
                                                           uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_pre[GROUP_MAX_RUNS + 1];
  __shared__ uint64_t s_base[GROUP_MAX_RUNS];
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  const uint32_t b = blockIdx.x / gg.n_groups, h = blockIdx.x % gg.n_groups;
  for (uint32_t i = threadIdx.x; i < 256; i += PART_THREADS) s_hist[i] = 0;
  const uint32_t nr = load_group_runs(gg, b, h, s_pre, s_base, s_scratch);
  const uint32_t n = s_pre[nr];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
#pragma unroll 1
  for (uint32_t t0 = 0; t0 < n; t0 += PART_TILE) {
    uint64_t addr[PART_ITEMS];
    const uint32_t act = group_item_addrs(s_pre, s_base, nr, n, t0 + w * WAVE_SPAN + __lane_id(), addr);
    uint8_t d[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) d[k] = dig[addr[k]];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k)
      if ((act >> k) & 1u) atomicAdd(&s_hist[d[k]], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_digits; d += PART_THREADS)
    hist[(static_cast<uint64_t>(b) * n_digits + d) * gg.n_groups + h] = s_hist[d];
}

// Stable scatter of each (bucket, group) by the second digit into the partitions: thread d starts at the scanned
// histogram's entry of (b, d, h).
template <typename SD, typename H, typename P>
__global__ __launch_bounds__(PART_THREADS) void part2g_scatter(GroupGeo gg, Digit dg, uint32_t n_digits,
                                                              const Rec<H, P>* __restrict__ in,
                                                              const uint32_t* __restrict__ offsets, RecOut<H, P> out) {
  __shared__ uint32_t s_pre[GROUP_MAX_RUNS + 1];
  __shared__ uint64_t s_base[GROUP_MAX_RUNS];
  __shared__ uint32_t s_cnt[PART_WAVES][256];
  __shared__ uint32_t s_delta[256];
  __shared__ uint32_t s_scratch[PART_WAVES + 1];
  __shared__ Rec<H, P> s_stage[PART_TILE];
  const uint32_t b = blockIdx.x / gg.n_groups, h = blockIdx.x % gg.n_groups;
  const uint32_t nr = load_group_runs(gg, b, h, s_pre, s_base, s_scratch);
  const uint32_t n = s_pre[nr];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  uint32_t run = threadIdx.x < n_digits ? offsets[(static_cast<uint64_t>(b) * n_digits + threadIdx.x) * gg.n_groups + h] : 0u;
  const NextDigit none{nullptr, 0u, 0u};
#pragma unroll 1
  for (uint32_t t0 = 0; t0 < n; t0 += PART_TILE) {
    if (t0) __syncthreads();  // the previous tile's write-out has read s_stage
    clear_wave_counts(s_cnt[w]);
    uint64_t addr[PART_ITEMS];
    const uint32_t act = group_item_addrs(s_pre, s_base, nr, n, t0 + w * WAVE_SPAN + __lane_id(), addr);
    Rec<H, P> recs[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) recs[k] = in[addr[k]];
    uint32_t dr[PART_ITEMS];
#pragma unroll
    for (int k = 0; k < PART_ITEMS; ++k) {
      const bool a = (act >> k) & 1u;
      const uint32_t dig = a ? digit_of<H>(dg, recs[k].key) : 0u;
      dr[k] = (dig << 24) | rank_item(dg, dig, a, s_cnt[w]);
    }
    staged_scatter<H, P>(recs, act, dr, s_cnt, s_delta, s_stage, s_scratch, n_digits, dg, none, run, out);
  }
}

// Partition bounds after the second pass: partition p = (b, d) starts at the scanned histogram's entry (b, d, 0).
static __global__ void group_bounds(const uint32_t* __restrict__ offsets, uint32_t n_parts, uint32_t n_groups,
                                    const uint64_t* __restrict__ total, uint32_t* __restrict__ bounds) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p <= n_parts; p += gridDim.x * blockDim.x)
    bounds[p] = p < n_parts ? offsets[static_cast<uint64_t>(p) * n_groups] : static_cast<uint32_t>(*total);
}

}  // namespace hyk
