// Host orchestration of the JoinHash kernels (kernels/join.hip): side plans, workspace carving, the radix passes and
// the per-partition LDS build/probe launch. Shared by the per-hashed-type translation units (hyrise_amd_join_*.hip),
// which instantiate it for one hashed type each so that `make -j` compiles them in parallel; the C entry points
// (hyrise_amd_join.hip) dispatch on the hashed type.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "hyrise_amd.h"
#include "../kernels/common.hpp"
#include "../kernels/join.hip"
#include "../kernels/join_direct.hip"
#include "capi_common.hpp"

namespace hyj {

using namespace hyc;

// Stream capture of a prepared plan's execution (hy_scan_join_plan_execute): while `capturing`, the final join launch
// leaves its flags / total on the device (no D2H, no synchronisation inside the captured region) and reports where
// they are; the plan reads them after each replay of the graph.
struct CaptureState {
  bool capturing = false;
  const uint32_t* misc = nullptr;
  const uint64_t* totals = nullptr;
  const uint32_t* direct_overflow = nullptr;  // the direct pass's region-overflow flag (join_direct.hip), or null
};
inline CaptureState& capture_state() {
  static thread_local CaptureState c;
  return c;
}

// Per-call tuning and test knobs of a join: environment variables, read once per C-ABI call (KnobScope at the entry
// points) so that tests can switch them between calls. A prepared plan snapshots them when it is created and executes
// under that snapshot, so its workspace carve, every eager execution and a captured graph's replays all use the layout
// the plan was sized and captured with, whatever the environment says later (HY_HASH_RECORDS /
// HY_HASH_GROUP / HY_ONEPASS were read per call and could differ between a capture and the plan's sizing).
struct JoinKnobs {
  int bloom = -1;                      // HY_JOIN_BLOOM: -1 heuristic, 0 never, 1 always
  bool hash_records = true;            // HY_HASH_RECORDS
  int hash_group = 1;                  // HY_HASH_GROUP: 1 or 4 records per lane and load
  bool blocked = false;                // HY_BLOCKED: pass 0 in Infinity-Cache row blocks (opt-in, see block_count)
  uint64_t block_bytes = 128ull << 20; // HY_BLOCK_MB
  uint64_t block_rows = 0;             // HY_BLOCK_ROWS (test knob: rows per block instead of bytes)
  uint64_t lds_budget = 0;             // HY_JOIN_LDS_BUDGET (test knob; 0: the default budget)
  bool onepass = false;                // HY_ONEPASS
  uint64_t onepass_cap_div = 8;        // HY_ONEPASS_CAP_DIV
  uint64_t onepass_cap = 0;            // HY_ONEPASS_CAP (0: computed)
  bool filter_buckets = true;          // HY_FILTER_BUCKETS: prefilter words set per LDS region (0: global atomics)
  bool rank_ballot = false;            // HY_RANK_BALLOT: rank by ballots (the fallback of a failed rank_order_check)
  bool direct = false;                 // HY_JOIN_DIRECT: direct partitioning of a filtered side (join_direct.hip)
  uint32_t direct_span = 16;           // HY_DIRECT_SPAN: tiles per span of the direct first pass
  uint32_t direct_groups = 0;          // HY_DIRECT_GROUPS: span groups per bucket of the direct second pass (0: auto)
  bool join_stash = false;             // HY_JOIN_STASH=1: two-pass partitions keep their first pass in LDS (opt-in)
};

inline JoinKnobs knobs_from_env() {
  JoinKnobs k;
  auto num = [](const char* name, long long dflt) {
    const char* e = std::getenv(name);
    return e ? std::strtoll(e, nullptr, 10) : dflt;
  };
  if (const char* e = std::getenv("HY_JOIN_BLOOM")) k.bloom = std::strtol(e, nullptr, 10) == 0 ? 0 : std::strtol(e, nullptr, 10) == 1 ? 1 : -1;
  k.hash_records = num("HY_HASH_RECORDS", 1) != 0;
  k.hash_group = num("HY_HASH_GROUP", 1) == 4 ? 4 : 1;
  k.blocked = num("HY_BLOCKED", 0) != 0;
  const long long mb = num("HY_BLOCK_MB", 128);
  k.block_bytes = uint64_t(mb > 0 ? mb : 128) << 20;
  k.block_rows = static_cast<uint64_t>(std::max<long long>(0, num("HY_BLOCK_ROWS", 0)));
  k.lds_budget = static_cast<uint64_t>(std::max<long long>(0, num("HY_JOIN_LDS_BUDGET", 0)));
  k.onepass = num("HY_ONEPASS", 0) != 0;
  k.onepass_cap_div = static_cast<uint64_t>(std::max<long long>(1, num("HY_ONEPASS_CAP_DIV", 8)));
  k.onepass_cap = static_cast<uint64_t>(std::max<long long>(0, num("HY_ONEPASS_CAP", 0)));
  k.filter_buckets = num("HY_FILTER_BUCKETS", 1) != 0;
  k.rank_ballot = num("HY_RANK_BALLOT", 0) != 0;
  k.direct = num("HY_JOIN_DIRECT", 0) != 0;
  k.direct_span = static_cast<uint32_t>(std::min<long long>(std::max<long long>(1, num("HY_DIRECT_SPAN", 16)), 64));
  k.direct_groups = static_cast<uint32_t>(std::min<long long>(std::max<long long>(0, num("HY_DIRECT_GROUPS", 0)), 4096));
  k.join_stash = num("HY_JOIN_STASH", 0) != 0;
  return k;
}

inline const JoinKnobs*& knob_override() {
  static thread_local const JoinKnobs* k = nullptr;
  return k;
}
inline JoinKnobs knobs() {
  const JoinKnobs* k = knob_override();
  return k ? *k : knobs_from_env();
}
// The knobs of one C-ABI call: a snapshot of the environment, or a prepared plan's own.
struct KnobScope {
  JoinKnobs own;
  const JoinKnobs* prev;
  KnobScope() : own(knobs_from_env()), prev(knob_override()) { knob_override() = &own; }
  explicit KnobScope(const JoinKnobs& k) : own(k), prev(knob_override()) { knob_override() = &own; }
  ~KnobScope() { knob_override() = prev; }
  KnobScope(const KnobScope&) = delete;
  KnobScope& operator=(const KnobScope&) = delete;
};

// Tiles per span of the pass from column chunks (sub1) and of the record passes (sub2); HY_PART_SUB1 / HY_PART_SUB2
// override them (tuning). Read once: workspace sizes and launches must agree.
inline uint32_t sub_from_env(const char* name, uint32_t dflt) {
  const char* e = std::getenv(name);
  const long v = e ? std::strtol(e, nullptr, 10) : 0;
  return v >= 1 && v <= hyk::PART_SUB_MAX ? static_cast<uint32_t>(v) : dflt;
}
inline uint32_t sub1() {
  static const uint32_t v = sub_from_env("HY_PART_SUB1", 1);
  return v;
}
// Spans of a side with a fused TableScan: two tiles, so that part1_spread's spans hold about as many matches as
// a record pass's tile (measured on MI355X at SF100: 1.70 ms for part1_spread vs 2.52 ms with one-tile spans);
// HY_PART_SUB_FILTERED overrides it.
inline uint32_t sub_filtered() {
  static const uint32_t v = sub_from_env("HY_PART_SUB_FILTERED", 2);
  return v;
}
// Next-digit bytes beside the records of a pass that has a successor (HY_DIGIT_BYTES=0 turns them off: the next
// histogram then reads the records and re-hashes them).
inline bool digit_bytes_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("HY_DIGIT_BYTES");
    return !(e && std::strtol(e, nullptr, 10) == 0);
  }();
  return v;
}
// Probe-side Bloom prefilter (hyk::bloom_filter_act) of INNER / SEMI joins whose build side is much smaller than the
// probe side (probe rows >= 16x build rows: most probe rows are expected to find no partner, as in TPC-H 3's joins;
// a foreign-key join like the headline's, probe / build ~ 4, keeps the plain path). 16 bits per build key.
// HY_JOIN_BLOOM=0 / 1 turns it off / on regardless of the ratio. Returns the filter's words (0: none).
inline uint64_t bloom_words(uint64_t build_rows, uint64_t probe_rows) {
  const int mode = knobs().bloom;
  const bool force = mode == 1;
  if (mode == 0 || build_rows == 0) return 0;
  if (!force && probe_rows < 16 * build_rows) return 0;
  uint64_t w = 1024;
  while (w < build_rows / 2 && w < (uint64_t(1) << 31)) w <<= 1;
  return w;
}

// Words reserved for a key-range bitmap prefilter (hyk::range_bitmap_words) next to the Bloom filter's: 64 bits per
// build row, enough for key ranges up to 64x the build rows (TPC-H 3's join 2: 14.6 M orders over the 600 M
// orderkey range at SF100, 41 bits per row); a wider range keeps the Bloom filter.
inline uint64_t range_bitmap_words(uint64_t build_rows) {
  return std::min<uint64_t>(2 * build_rows + 1024, uint64_t(1) << 28);
}
// The prefilter built per LDS region (hyk::filter_bucket_*) when its words allow it: the count / scatter grid, the
// largest region shift the device can pick (it sizes the set kernel's LDS), an upper bound of the regions and the
// region x workgroup matrix's length. blocks == 0: the global-atomic build (filter_clear + filter_set).
struct FilterBuckets {
  uint32_t blocks = 0, shift = 0, bins = 0;
  uint64_t scan_len = 0;
};
inline FilterBuckets filter_buckets(uint64_t bloom_n, uint64_t build_rows) {
  FilterBuckets f;
  if (!bloom_n || !knobs().filter_buckets) return f;
  const uint64_t maxw = std::max(bloom_n, range_bitmap_words(build_rows));
  uint32_t shift = hyk::FB_SHIFT_MIN;
  while (((maxw + (uint64_t(1) << shift) - 1) >> shift) > hyk::FB_BINS) ++shift;
  if (shift > hyk::FB_SHIFT_MAX) return f;
  f.shift = shift;
  // (the device may pick a smaller shift for a narrower key range: up to FB_BINS regions of the smallest size)
  f.bins = static_cast<uint32_t>(std::min<uint64_t>(hyk::FB_BINS, (maxw + (uint64_t(1) << hyk::FB_SHIFT_MIN) - 1) >>
                                                                      hyk::FB_SHIFT_MIN));
  f.blocks = static_cast<uint32_t>(std::clamp<uint64_t>(build_rows / 16384, 1, 256));
  f.scan_len = uint64_t(f.bins) * f.blocks;
  return f;
}
// The prefilter area: a 64-byte header (hyk::FilterHdr), then the larger of the two filters' words, then the bucketed
// build's matrix (twice: counts and offsets), its items (one word per build row) and two 64-bit counters.
inline uint64_t prefilter_words(uint64_t bloom_n, uint64_t build_rows) {
  if (!bloom_n) return 1;
  const FilterBuckets f = filter_buckets(bloom_n, build_rows);
  const uint64_t fb = f.blocks ? 2 * f.scan_len + build_rows + 8 : 0;
  return 16 + ((std::max(bloom_n, range_bitmap_words(build_rows)) + 3) & ~uint64_t(3)) + fb;
}

inline uint32_t sub2() {
  static const uint32_t v = sub_from_env("HY_PART_SUB2", 1);
  return v;
}
inline uint64_t span1() { return uint64_t(sub1()) * hyk::PART_TILE; }
inline uint64_t span2() { return uint64_t(sub2()) * hyk::PART_TILE; }

struct SidePlan {
  uint64_t n_rows = 0;
  uint64_t n_tiles1 = 0;
  uint32_t sub = 1;                      // tiles per pass-0 span
  std::vector<hyk::SrcChunk> chunks;
  std::vector<uint64_t> tile_begin;
  std::vector<uint64_t> row_begin;       // this table
  std::vector<hyk::SrcChunk> referenced;
  std::vector<uint64_t> ref_row_begin;   // referenced table
  int32_t fuse = 0;
  uint32_t ref_base = 0;                 // referenced_chunk_base of the side
  // fused TableScan (hy_join_filter): predicate chunk per side chunk
  bool filtered = false;
  std::vector<hy_scan_chunk> filter;
  int32_t filter_type = 0;
  uint64_t filter_const = 0;
  uint32_t* scan_out = nullptr;
  uint64_t* scan_chunk_begin = nullptr;
  hy_row_id* scan_rows = nullptr;        // hy_join_filter.out_row_ids
  // a prepared plan (hy_scan_join_plan_*) whose own workspace already holds this side's descriptors from an earlier
  // execution: the upload is skipped (the carve of the workspace is deterministic for a plan)
  bool device_ready = false;
};

inline uint32_t uniform_of(const std::vector<uint64_t>& row_begin) {
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

inline hyk::SrcChunk src_from(const hy_column_chunk& c, const hy_row_id* pos_list, uint32_t size, uint64_t row_begin,
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

inline int type_bytes(int32_t t) {
  return (t == HY_TYPE_INT32 || t == HY_TYPE_FLOAT) ? 4 : (t == HY_TYPE_INT64 || t == HY_TYPE_DOUBLE) ? 8 : 0;
}

// Pass-0 spans of the side's chunks (a span never crosses a chunk).
inline void plan_spans(SidePlan& p, uint32_t sub) {
  p.sub = sub;
  const uint64_t span = uint64_t(sub) * hyk::PART_TILE;
  uint64_t tiles = 0;
  for (size_t i = 0; i < p.chunks.size(); ++i) {
    p.tile_begin[i] = tiles;
    tiles += (uint64_t(p.chunks[i].size) + span - 1) / span;
  }
  p.tile_begin[p.chunks.size()] = tiles;
  p.n_tiles1 = tiles;
}

// The LDS ordering that the partition passes' ranking relies on (hyk::wave_rank_add), checked once per device before
// its first join (hyk::rank_order_check against the mask ranking). Skipped while the device cannot run it (a stream
// capture in progress elsewhere); on a device that breaks it the passes rank by ballots (rank_ballot), slower but
// independent of the LDS atomics' lane order.
inline std::atomic<bool>* rank_broken() {
  static std::atomic<bool> broken[64] = {};
  return broken;
}
inline hy_status check_rank_order() {
  static std::mutex m;
  static int state[64] = {};  // 0: not checked yet, 1: holds, 2: broken
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return HY_OK;
  std::lock_guard<std::mutex> lock(m);
  if (state[dev] == 0) {
    uint32_t* d = nullptr;
    hipStream_t cs = nullptr;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return HY_OK;
    uint32_t bad = 0;
    bool ran = false;
    if (hipMalloc(&d, 4) == hipSuccess) {
      ran = hipMemsetAsync(d, 0, 4, cs) == hipSuccess;
      if (ran) {
        hipLaunchKernelGGL(hyk::rank_order_check, dim3(1), dim3(256), 0, cs, 96u, d);
        ran = hipGetLastError() == hipSuccess && hipMemcpyAsync(&bad, d, 4, hipMemcpyDeviceToHost, cs) == hipSuccess &&
              hipStreamSynchronize(cs) == hipSuccess;
      }
      (void)hipFree(d);
    }
    (void)hipStreamDestroy(cs);
    (void)hipGetLastError();
    if (ran) state[dev] = bad == 0 ? 1 : 2;
  }
  if (state[dev] == 2) rank_broken()[dev] = true;  // the partition passes rank by ballots on this device instead
  return HY_OK;
}

// 1 when the partition passes rank by ballots (hyk::rank_item): the device failed rank_order_check, or
// HY_RANK_BALLOT=1 (tests force the fallback with it).
inline uint32_t rank_ballot() {
  int dev = 0;
  if (knobs().rank_ballot) return 1u;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0u;
  return rank_broken()[dev] ? 1u : 0u;
}

inline hy_status plan_side(const hy_join_side* side, SidePlan& p) {
  if (!side || (side->n_chunks && !side->chunks)) return fail(HY_ERR_INVALID_ARGUMENT, "join side");
  if (hy_status st = check_rank_order()) return st;
  p.ref_base = side->referenced_chunk_base;
  p.chunks.resize(side->n_chunks);
  p.tile_begin.resize(side->n_chunks + 1);
  p.row_begin.resize(side->n_chunks + 1);
  bool is_ref = false;
  uint64_t rows = 0;
  for (uint32_t i = 0; i < side->n_chunks; ++i) {
    const hy_join_chunk& c = side->chunks[i];
    if (c.pos_list) is_ref = true;
    if (!c.pos_list && !row_readable(c.column))
      return fail(HY_ERR_UNSUPPORTED, "join chunk kind (RunLength / FrameOfReference: join the value mirror)");
    p.chunks[i] = src_from(c.column, c.pos_list, c.size, rows, c.single_chunk);
    p.chunks[i].chunk_id = c.chunk_id;
    p.chunks[i].ref_offset = c.pos_list ? c.referenced_offset : 0u;
    p.row_begin[i] = rows;
    rows += c.size;
  }
  p.row_begin[side->n_chunks] = rows;
  p.n_rows = rows;
  plan_spans(p, sub1());
  if (rows >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "join side exceeds 2^32-1 rows");
  if (is_ref) {
    p.referenced.resize(side->n_referenced);
    p.ref_row_begin.resize(side->n_referenced + 1);
    uint64_t rr = 0;
    for (uint32_t i = 0; i < side->n_referenced; ++i) {
      if (!row_readable(side->referenced[i]))
        return fail(HY_ERR_UNSUPPORTED, "referenced chunk kind (RunLength / FrameOfReference: join the value mirror)");
      p.referenced[i] = src_from(side->referenced[i], nullptr, side->referenced[i].size, rr);
      p.ref_row_begin[i] = rr;
      rr += side->referenced[i].size;
    }
    p.ref_row_begin[side->n_referenced] = rr;
    for (const auto& c : p.chunks) {
      if (c.pos_list && c.single_chunk != HY_MIXED_CHUNKS && c.single_chunk >= side->n_referenced)
        return fail(HY_ERR_INVALID_ARGUMENT, "single_chunk outside the referenced chunks");
      if (c.pos_list && c.ref_offset > side->n_referenced)
        return fail(HY_ERR_INVALID_ARGUMENT, "referenced_offset outside the referenced chunks");
      if (c.ref_offset && side->fuse_dereference)
        return fail(HY_ERR_INVALID_ARGUMENT, "fuse_dereference needs one referenced table");
    }
    if (rr >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "referenced table exceeds 2^32-1 rows");
  }
  return HY_OK;
}

// Attaches a fused TableScan predicate to a data-table side.
inline hy_status plan_filter(const hy_join_filter* f, SidePlan& p, int32_t column_type, int32_t hashed_type) {
  if (f == nullptr) return HY_OK;
  if (column_type != hashed_type)
    return fail(HY_ERR_UNSUPPORTED, "a fused scan needs the side's join column to have the hashed type");
  if (p.chunks.size() && !f->chunks) return fail(HY_ERR_INVALID_ARGUMENT, "filter chunks");
  if (f->n_chunks < p.chunks.size())
    return fail(HY_ERR_INVALID_ARGUMENT, "filter has " + std::to_string(f->n_chunks) + " predicate chunks for a side of " +
                                             std::to_string(p.chunks.size()) + " chunks");
  if (p.n_rows >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "filtered join side exceeds 2^31-1 rows");
  p.filtered = true;
  p.filter.assign(f->chunks, f->chunks + p.chunks.size());
  p.filter_type = f->value_type;
  p.scan_out = f->out_offsets;
  p.scan_chunk_begin = f->out_chunk_begin;
  p.scan_rows = f->out_row_ids;
  if (p.scan_rows && (!p.scan_out || !p.scan_chunk_begin))
    return fail(HY_ERR_INVALID_ARGUMENT, "out_row_ids needs out_offsets and out_chunk_begin");
  bool value = false;
  for (size_t i = 0; i < p.chunks.size(); ++i) {
    if (p.chunks[i].pos_list) return fail(HY_ERR_UNSUPPORTED, "a filtered join side must be a data table");
    const hy_scan_chunk& sc = p.filter[i];
    if (sc.op < HY_OP_EQ || sc.op > HY_OP_IS_NOT_NULL || sc.op == HY_OP_IS_NULL)
      return fail(HY_ERR_UNSUPPORTED, "fused scan filter op");
    if (!row_readable(sc.column)) return fail(HY_ERR_UNSUPPORTED, "fused scan filter chunk kind");
    if (sc.column.size != p.chunks[i].size) return fail(HY_ERR_INVALID_ARGUMENT, "filter chunk size != join chunk size");
    if (sc.column.size && !aligned16(sc.column.data)) return fail(HY_ERR_ALIGNMENT, "filter data not 16-byte aligned");
    if (sc.column.kind == HY_COL_DICT) {
      if (sc.column.vid_width != 1 && sc.column.vid_width != 2 && sc.column.vid_width != 4)
        return fail(HY_ERR_INVALID_ARGUMENT, "filter vid width");
    } else if (sc.op != HY_OP_NONE) {
      value = true;
    }
  }
  plan_spans(p, sub_filtered());
  if (value) {
    const int tb = type_bytes(f->value_type);
    if (!tb) return fail(HY_ERR_UNSUPPORTED, "filter value type");
    if (!f->constant) return fail(HY_ERR_INVALID_ARGUMENT, "filter constant");
    std::memcpy(&p.filter_const, f->constant, tb);
  }
  return HY_OK;
}

// Radix digits from the most significant: the partition id has `bits` bits; the first digit may be narrower than 8 so
// that the others are 8 bits wide; min_top forces the first digit to be at least that wide (the distributed join
// assigns whole first-digit buckets to ranks).
inline std::vector<uint32_t> digit_plan(uint32_t bits, uint32_t min_top) {
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
  hy_scan_chunk* filter;     // fused TableScan predicate chunks (filtered sides)
  uint32_t* hist;            // histogram of the current pass (largest pass)
  uint32_t* off;             // its exclusive scan
  hyk::Rec<H, P>* recA;
  hyk::Rec<H, P>* recB;      // filtered sides: first the gapped per-span records of part1_compact
  uint32_t* span_count;      // filtered sides: matches per pass-0 span
  uint64_t* mbits;           // filtered sides: the fused scan's match ballots (part1_mask), one per (tile, wave, item)
  uint8_t* digA;             // next-pass digit bytes beside recA / recB (sides with more than one pass)
  uint8_t* digB;
  uint32_t* segA;            // segment / partition bounds, ping-pong (2^bits + 1 entries)
  uint32_t* segB;
  uint64_t* seg_tile_begin;  // 2^bits + 1
  uint32_t* tile_counts;     // 2^bits
  uint32_t* tile_excl;       // 2^bits
  uint32_t* tile_owner;      // largest pass's tiles
  uint64_t* total;           // rows taking part (device)
  uint64_t* grand_total;     // total of a fused-scan histogram (records + scan matches)
  // pass 0 in row blocks (block_plan; null when the side is not blocked): per (block, digit) run begin / count, the
  // scan matches before each block, and the first record pass's segments (runs) and groups (buckets)
  uint32_t* cls_begin;
  uint32_t* cls_count;
  uint64_t* scan_base;
  uint32_t* bseg_begin;
  uint32_t* bseg_end;
  uint32_t* bseg_stride;
  uint32_t* bseg_toff;
  uint64_t* bseg_hbase;
  uint64_t* group_hbase;
  uint32_t* group_tiles;
  uint32_t* group_out;
};

struct SideSizes {
  uint64_t rows = 0, tiles1 = 0;   // pass-0 spans (0: the side starts from received records)
  uint32_t sub = 1;                // tiles per pass-0 span
  size_t n_chunks = 0, n_referenced = 0;
  bool filtered = false;           // one more histogram row in pass 0 (the scan's matches)
  bool digit_bytes = false;        // next-digit byte arrays (single-GPU sides with more than one pass)
  uint32_t blocks = 0;             // pass 0 in row blocks (block_plan): their number, else 0
};

// Largest histogram of any pass, and the largest tile count of any record pass.
inline void pass_sizes(const SideSizes& z, const std::vector<uint32_t>& w, uint64_t first_segs, uint64_t* hist_words,
                       uint64_t* max_tiles) {
  *hist_words = 1;
  *max_tiles = 1;
  uint64_t segs = first_segs;
  for (size_t i = 0; i < w.size(); ++i) {
    const uint64_t digits = 1ull << w[i];
    if (i == 0 && z.tiles1) {
      *hist_words = std::max(*hist_words, (digits + (z.filtered ? 1 : 0)) * z.tiles1);
      *max_tiles = std::max(*max_tiles, z.tiles1);
    } else {
      const uint64_t t = (z.rows + span2() - 1) / span2() + segs;
      *hist_words = std::max(*hist_words, digits * t);
      *max_tiles = std::max(*max_tiles, t);
      segs *= digits;
      continue;
    }
    segs = digits * std::max<uint64_t>(1, z.blocks);  // a blocked pass 0: one run per (digit, block)
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
  b.filter = z.filtered ? cv.take<hy_scan_chunk>(std::max<size_t>(1, z.n_chunks)) : nullptr;
  uint64_t hist_words, max_tiles;
  pass_sizes(z, w, first_segs, &hist_words, &max_tiles);
  b.hist = cv.take<uint32_t>(hist_words);
  b.off = cv.take<uint32_t>(hist_words);
  b.recA = own_recA ? cv.take<hyk::Rec<H, P>>(std::max<uint64_t>(1, z.rows)) : nullptr;
  b.recB = cv.take<hyk::Rec<H, P>>(std::max<uint64_t>(1, z.filtered ? std::max(z.rows, z.tiles1 * z.sub * hyk::PART_TILE) : z.rows));
  b.span_count = z.filtered ? cv.take<uint32_t>(std::max<uint64_t>(1, z.tiles1)) : nullptr;
  b.mbits = z.filtered ? cv.take<uint64_t>(std::max<uint64_t>(1, z.tiles1 * z.sub * hyk::MASK_WORDS)) : nullptr;
  b.digA = z.digit_bytes ? cv.take<uint8_t>(std::max<uint64_t>(16, z.rows)) : nullptr;
  b.digB = z.digit_bytes ? cv.take<uint8_t>(std::max<uint64_t>(16, z.rows)) : nullptr;
  const uint64_t parts = (uint64_t(1) << bits) + 1;
  b.segA = cv.take<uint32_t>(parts);
  b.segB = cv.take<uint32_t>(parts);
  b.seg_tile_begin = cv.take<uint64_t>(parts);
  b.tile_counts = cv.take<uint32_t>(parts);
  b.tile_excl = cv.take<uint32_t>(parts);
  b.tile_owner = cv.take<uint32_t>(max_tiles);
  b.total = cv.take<uint64_t>(1);
  b.grand_total = cv.take<uint64_t>(1);
  b.cls_begin = b.cls_count = b.bseg_begin = b.bseg_end = b.bseg_stride = b.bseg_toff = nullptr;
  b.scan_base = b.bseg_hbase = b.group_hbase = nullptr;
  b.group_tiles = b.group_out = nullptr;
  if (z.blocks && !w.empty()) {
    const uint64_t nd0 = uint64_t(1) << w[0], nseg = nd0 * z.blocks;
    b.cls_begin = cv.take<uint32_t>(uint64_t(z.blocks) * 256);
    b.cls_count = cv.take<uint32_t>(uint64_t(z.blocks) * 256);
    b.scan_base = cv.take<uint64_t>(z.blocks + 1);
    b.bseg_begin = cv.take<uint32_t>(nseg);
    b.bseg_end = cv.take<uint32_t>(nseg);
    b.bseg_stride = cv.take<uint32_t>(nseg);
    b.bseg_toff = cv.take<uint32_t>(nseg);
    b.bseg_hbase = cv.take<uint64_t>(nseg);
    b.group_hbase = cv.take<uint64_t>(nd0);
    b.group_tiles = cv.take<uint32_t>(nd0);
    b.group_out = cv.take<uint32_t>(nd0);
  }
}

struct Common {
  uint64_t* scan_status;
  uint64_t scan_status_words;
  uint32_t* misc;  // [0] ticket [1] error [2] overflow ...
  uint64_t* totals;
  uint64_t* join_status;
};

inline void carve_common(Carver& cv, uint64_t max_scan, uint32_t bits, Common* c) {
  c->scan_status_words = max_scan / hyk::SCAN_BLOCK + 3;  // look-back words of every tile + the ticket
  c->scan_status = cv.take<uint64_t>(c->scan_status_words);
  c->misc = cv.take<uint32_t>(64);
  c->totals = cv.take<uint64_t>(8);
  c->join_status = cv.take<uint64_t>((uint64_t(1) << bits) + 1);
}

// n: the length, or with n_dev its upper bound (the device length is *n_dev * n_mul, exclusive_scan_u32).
inline hy_status run_scan(const uint32_t* in, uint32_t* out, uint64_t n, const Common& c, hipStream_t s,
                          uint64_t* total_out = nullptr, const uint64_t* n_dev = nullptr, uint32_t n_mul = 1) {
  if (n == 0) {
    if (total_out) HY_HIP(hipMemsetAsync(total_out, 0, 8, s));
    return HY_OK;
  }
  const uint64_t tiles = (n + hyk::SCAN_BLOCK - 1) / hyk::SCAN_BLOCK;
  if (tiles + 2 > c.scan_status_words) return fail(HY_ERR_WORKSPACE, "scan status");
  // the look-back words and (in the word after them) the tile ticket, zeroed by one memset
  HY_HIP(hipMemsetAsync(c.scan_status, 0, sizeof(uint64_t) * (tiles + 2), s));
  uint32_t* ticket = reinterpret_cast<uint32_t*>(c.scan_status + tiles + 1);
  KTimer kt_("exclusive_scan", s, n);
  const bool vec = reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
  hipLaunchKernelGGL(vec ? hyk::exclusive_scan_u32<true> : hyk::exclusive_scan_u32<false>,
                     dim3(static_cast<uint32_t>(tiles)), dim3(hyk::SCAN_T), 0, s, in, out, n, c.scan_status, ticket,
                     c.misc + 1, total_out, n_dev, n_mul);
  kt_.done();
  HY_HIP(hipGetLastError());
  return HY_OK;
}

inline uint32_t full_mask(uint32_t bits) { return bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u); }

template <typename H, typename P>
hyk::RecOut<H, P> aos_out(hyk::Rec<H, P>* recs) {
  return hyk::RecOut<H, P>{recs, nullptr, nullptr, 0u, nullptr, 0u};
}

// The SoA form of a last record pass (hyk::RecOut / hyk::HashSrc) inside `area`, a record buffer of at least `rows`
// 8-byte records: 16-bit hash remainders, then (16-byte aligned) the payloads - 6 B per record, so that with rows >= 16
// both arrays stay readable 3 records past their end (HashSrc's group loads). A build side of a prefiltered join also
// sets its Bloom words by hash (bloom_n words).
template <typename H, typename P>
hyk::RecOut<H, P> soa_out(void* area, uint64_t rows, uint32_t bits, uint32_t* bloom = nullptr, uint64_t bloom_n = 0) {
  static_assert(sizeof(P) == 4, "SoA records carry 32-bit payloads");
  auto* hk = static_cast<uint16_t*>(area);
  auto* pay = reinterpret_cast<P*>(static_cast<char*>(area) + hyk::align16(2 * rows));
  return hyk::RecOut<H, P>{nullptr, hk, pay, bits, bloom, bloom ? static_cast<uint32_t>(bloom_n - 1) : 0u};
}


// The load path every chunk of the side allows (hyk::LP_*): lean kernels for the all-value and all-single-chunk
// reference sides, the general one otherwise.
inline int load_path(const SidePlan& p) {
  bool value = true, ref1 = true;
  for (const auto& c : p.chunks) {
    if (c.size == 0) continue;
    value = value && c.pos_list == nullptr && c.kind == HY_COL_VALUE && c.nulls == nullptr;
    ref1 = ref1 && c.pos_list != nullptr && c.single_chunk != HY_MIXED_CHUNKS &&
           p.referenced[c.single_chunk].kind == HY_COL_VALUE && p.referenced[c.single_chunk].nulls == nullptr &&
           p.referenced[c.single_chunk].size > 0;
  }
  if (value) return hyk::LP_VALUE;
  if (ref1) return hyk::LP_REF1;
  // PosLists over several chunks: the batched path when every referenced chunk is a ValueColumn without NULLs and
  // chunk 0 (the NULL RowIDs' stand-in) is not empty
  bool refm = !p.referenced.empty() && p.referenced[0].size > 0;
  for (const auto& c : p.chunks) refm = refm && (c.size == 0 || c.pos_list != nullptr);
  for (const auto& r : p.referenced) refm = refm && (r.size == 0 || (r.kind == HY_COL_VALUE && r.nulls == nullptr));
  return refm ? hyk::LP_REFM : hyk::LP_ANY;
}

// Next-pass digit of pass i of the plan w (bits [shift, shift + w[i + 1])), or none.
inline hyk::NextDigit next_digit(const std::vector<uint32_t>& w, size_t i, uint32_t bits, uint8_t* bytes) {
  if (bytes == nullptr || i + 1 >= w.size()) return hyk::NextDigit{nullptr, 0, 0};
  uint32_t above = 0;
  for (size_t j = 0; j <= i + 1; ++j) above += w[j];
  return hyk::NextDigit{bytes, bits - above, (1u << w[i + 1]) - 1u};
}

// The filter kind every predicate chunk of a filtered side allows (hyk::FK_*).
inline int filter_kind(const SidePlan& p) {
  if (!p.filtered) return hyk::FK_NONE;
  int width = 0;
  for (const auto& f : p.filter) {
    if (f.op == HY_OP_NONE || f.column.size == 0) continue;
    if (f.column.kind != HY_COL_DICT) return hyk::FK_ANY;
    if (width && width != f.column.vid_width) return hyk::FK_ANY;
    width = f.column.vid_width;
  }
  return width == 2 ? hyk::FK_DICT16 : width == 4 ? hyk::FK_DICT32 : width == 1 ? hyk::FK_DICT8 : hyk::FK_ANY;
}

// The fused scan's pass 0 through gapped records (part1_compact / part1_spread; the default) or through match bits
// (part1_mask / part1_spread_mask; HY_FILTER_COMPACT=0). Measured on MI355X at SF100 (round 3): compact 1.43 + 1.52 ms,
// match bits 0.94 + 3.16 ms with two-tile spans (2.08 ms with one-tile spans) - the match-bit spread pass compacts a
// span into LDS before its scatter, which halves the resident workgroups and serialises load, compaction and scatter.
// HY_HASH_RECORDS=0: keep {key, payload} records up to the partition join also where HashSrc applies (A/B).
inline bool hash_records_enabled() { return knobs().hash_records; }

inline bool filter_compact_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("HY_FILTER_COMPACT");
    return !(e && std::strtol(e, nullptr, 10) == 0);
  }();
  return v;
}

// The hy_join_filter.out_row_ids arrays that the current join's part1_spread wrote directly (this thread, reset by
// join_typed); the other pass-0 variants write offsets, which join_typed expands into the RowIDs at the end.
inline std::vector<const hy_row_id*>& scan_rows_written() {
  thread_local std::vector<const hy_row_id*> v;
  return v;
}

// Calls f with the kernel side tag (hyk::OnBuild / hyk::OnProbe) named by a runtime side tag ("build" / "probe").
template <typename F>
hy_status by_side(const char* tag, F&& f) {
  return tag[0] == 'b' ? f(hyk::OnBuild{}) : f(hyk::OnProbe{});
}

// Pass 0 of a side with a fused TableScan: part1_compact (gapped row-order records in recB, histograms with the
// scan-match row), the histogram scan, then part1_spread (scan output + stable scatter into `out`). HY_FILTER_COMPACT=0:
// part1_mask (match bits) + part1_spread_mask (compaction in LDS) instead, on a probe side.
template <typename SD, typename T, typename H, int LP, int FK>
hy_status launch_filtered_pass0(const SidePlan& p, const hyk::Side& sd, const hyk::Digit& d0,
                                const hyk::NextDigit& nd, uint32_t w0, uint32_t n_digits, SideBufs<H, uint32_t>& b,
                                const Common& c, hipStream_t s, const hyk::RecOut<H, uint32_t>& out) {
  const dim3 grid(static_cast<uint32_t>(p.n_tiles1));
  // the match-bit variant is an experiment on the headline's filtered (probe) side: built for that side only
  if constexpr (std::is_same_v<SD, hyk::OnProbe>) if (!filter_compact_enabled() && (p.sub == 1 || p.sub == 2)) {
    {
      KTimer kt_((std::string("part1_mask.") + SD::name).c_str(), s, p.n_rows);
      hipLaunchKernelGGL((hyk::part1_mask<SD, T, H, LP, FK>), grid, dim3(hyk::PART_THREADS), 0, s, sd, d0, n_digits,
                         b.hist, b.mbits);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    hy_status st = run_scan(b.hist, b.off, uint64_t(n_digits + 1) * p.n_tiles1, c, s, b.grand_total);
    if (st != HY_OK) return st;
    hipLaunchKernelGGL(hyk::fused_scan_totals, dim3(grid_for(p.chunks.size() + 1, 256)), dim3(256), 0, s, b.off,
                       p.n_tiles1, n_digits, b.grand_total, b.tile_begin, static_cast<uint32_t>(p.chunks.size()),
                       b.total, p.scan_chunk_begin);
    HY_HIP(hipGetLastError());
    const hyk::Side& sd2 = sd;
    {
      KTimer kt_((std::string("part1_spread.") + SD::name).c_str(), s, p.n_rows);
      if (out.hk != nullptr) return fail(HY_ERR_UNSUPPORTED, "match-bit pass 0 writes {key, payload} records");
      if (p.sub == 2)
        hipLaunchKernelGGL((hyk::part1_spread_mask<SD, T, H, LP, 2>), grid, dim3(hyk::PART_THREADS), 0, s, sd2, d0, nd,
                           n_digits, b.off, b.mbits, out.recs);
      else
        hipLaunchKernelGGL((hyk::part1_spread_mask<SD, T, H, LP, 1>), grid, dim3(hyk::PART_THREADS), 0, s, sd2, d0, nd,
                           n_digits, b.off, b.mbits, out.recs);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    return HY_OK;
  }
  {
    KTimer kt_((std::string("part1_compact.") + SD::name).c_str(), s, p.n_rows);
    bool prefiltered = false;
    if constexpr (std::is_same_v<SD, hyk::OnProbe>) prefiltered = sd.bloom != nullptr;  // (build sides have none)
    if (prefiltered) {
      if constexpr (std::is_same_v<SD, hyk::OnProbe>)
        hipLaunchKernelGGL((hyk::part1_compact<SD, T, H, LP, FK, true>), grid, dim3(hyk::PART_THREADS), 0, s, sd, d0,
                           n_digits, b.hist, b.span_count, b.recB);
    } else {
      hipLaunchKernelGGL((hyk::part1_compact<SD, T, H, LP, FK, false>), grid, dim3(hyk::PART_THREADS), 0, s, sd, d0,
                         n_digits, b.hist, b.span_count, b.recB);
    }
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  hy_status st = run_scan(b.hist, b.off, uint64_t(n_digits + 1) * p.n_tiles1, c, s, b.grand_total);
  if (st != HY_OK) return st;
  hipLaunchKernelGGL(hyk::fused_scan_totals, dim3(grid_for(p.chunks.size() + 1, 256)), dim3(256), 0, s, b.off,
                     p.n_tiles1, n_digits, b.grand_total, b.tile_begin, static_cast<uint32_t>(p.chunks.size()), b.total,
                     p.scan_chunk_begin);
  HY_HIP(hipGetLastError());
  hyk::Side sdr = sd;
  if (p.scan_rows) {  // the scan's PosLists straight from the ranking pass (no expansion of the offsets afterwards)
    sdr.scan_rows = p.scan_rows;
    scan_rows_written().push_back(p.scan_rows);
  }
  {
    KTimer kt_((std::string("part1_spread.") + SD::name).c_str(), s, p.n_rows);
    hipLaunchKernelGGL((hyk::part1_spread<SD, H>), grid, dim3(hyk::PART_THREADS), 0, s, sdr, d0, nd,
                       static_cast<int>(w0), n_digits, b.off, b.span_count, b.recB, out);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

template <typename SD, typename T, typename H, typename P, int LP>
hy_status launch_pass0(const SidePlan& p, const hyk::Side& sd, const hyk::Digit& d0,
                       const hyk::NextDigit& nd, uint32_t w0, uint32_t n_digits, SideBufs<H, P>& b, const Common& c,
                       hipStream_t s, const hyk::RecOut<H, P>& out) {
  const bool filt = p.filtered;
  const int fk = filter_kind(p);
  if constexpr (LP != hyk::LP_REF1 && LP != hyk::LP_REFM && std::is_same_v<T, H> && std::is_same_v<P, uint32_t>) {
    switch (fk) {
      case hyk::FK_DICT8:
        return launch_filtered_pass0<SD, T, H, LP, hyk::FK_DICT8>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
      case hyk::FK_DICT16:
        return launch_filtered_pass0<SD, T, H, LP, hyk::FK_DICT16>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
      case hyk::FK_DICT32:
        return launch_filtered_pass0<SD, T, H, LP, hyk::FK_DICT32>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
      case hyk::FK_ANY:
        return launch_filtered_pass0<SD, T, H, LP, hyk::FK_ANY>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
      default:
        break;
    }
  }
  if (filt) return fail(HY_ERR_UNSUPPORTED, "fused scan on a side whose join column type is not the hashed type");
  const dim3 grid(static_cast<uint32_t>(p.n_tiles1));
  {
    KTimer kt_((std::string("part1_hist.") + SD::name).c_str(), s, p.n_rows);
    hipLaunchKernelGGL((hyk::part1_hist<SD, T, H, LP>), grid, dim3(hyk::PART_THREADS), 0, s, sd, d0, n_digits, b.hist);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  hy_status st = run_scan(b.hist, b.off, uint64_t(n_digits) * p.n_tiles1, c, s, b.total);
  if (st != HY_OK) return st;
  {
    KTimer kt_((std::string("part1_scatter.") + SD::name).c_str(), s, p.n_rows);
    hipLaunchKernelGGL((hyk::part1_scatter<SD, T, H, P, LP>), grid, dim3(hyk::PART_THREADS), 0, s, sd, d0, nd,
                       static_cast<int>(w0), n_digits, b.off, out);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// Pass 0: from column chunks into `out`, bucket bounds into b.segA (2^w0 buckets); next-digit bytes into nd.
template <typename SD, typename T, typename H, typename P>
hy_status pass0_side(const SidePlan& p, SideBufs<H, P>& b, uint32_t bits, uint32_t w0,
                     uint32_t seed, bool keep_nulls, uint32_t ref_base, const hyk::NextDigit& nd, const Common& c,
                     hipStream_t s, const hyk::RecOut<H, P>& out, const uint32_t* bloom = nullptr, uint64_t bloom_n = 0,
                     bool bloom_by_hash = false, const hyk::FilterHdr* bloom_hdr = nullptr,
                     uint64_t range_words = 0);

// The kernels' view of a side inside the workspace (pass 0).
template <typename H, typename P>
hyk::Side make_side(const SidePlan& p, const SideBufs<H, P>& b, uint32_t seed, bool keep_nulls, uint32_t ref_base,
                    const uint32_t* bloom, uint64_t bloom_n, bool bloom_by_hash, const hyk::FilterHdr* bloom_hdr,
                    uint64_t range_words) {
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
  sd.sub = p.sub;
  sd.filter = p.filtered ? b.filter : nullptr;
  sd.filter_const = p.filter_const;
  sd.filter_type = p.filter_type;
  sd.scan_out = p.scan_out;
  sd.scan_rows = nullptr;  // (set by launch_filtered_pass0 for part1_spread only)
  sd.bloom = bloom;
  sd.bloom_mask = bloom ? static_cast<uint32_t>(bloom_n - 1) : 0u;
  sd.bloom_by_hash = bloom_by_hash ? 1 : 0;
  sd.bloom_hdr = bloom ? bloom_hdr : nullptr;
  sd.range_words = range_words;
  sd.seed = seed;
  return sd;
}

template <typename SD, typename T, typename H, typename P>
hy_status pass0_side(const SidePlan& p, SideBufs<H, P>& b, uint32_t bits, uint32_t w0,
                     uint32_t seed, bool keep_nulls, uint32_t ref_base, const hyk::NextDigit& nd, const Common& c,
                     hipStream_t s, const hyk::RecOut<H, P>& out, const uint32_t* bloom, uint64_t bloom_n,
                     bool bloom_by_hash, const hyk::FilterHdr* bloom_hdr, uint64_t range_words) {
  const hyk::Side sd = make_side(p, b, seed, keep_nulls, ref_base, bloom, bloom_n, bloom_by_hash, bloom_hdr, range_words);
  const uint32_t n_digits = 1u << w0;
  hyk::Digit d0{full_mask(bits), bits - w0, n_digits - 1u, seed, g_key_hash, rank_ballot()};
  HY_HIP(hipMemsetAsync(b.total, 0, 8, s));
  if (p.filtered && p.scan_chunk_begin) HY_HIP(hipMemsetAsync(p.scan_chunk_begin, 0, 8 * (p.chunks.size() + 1), s));
  if (p.n_tiles1 > 0) {
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((sd.n_chunks + 255) / 256), dim3(256), 0, s, b.tile_begin,
                       sd.n_chunks, b.tile_owner);
    HY_HIP(hipGetLastError());
    const int lp = load_path(p);
    hy_status st;
    if (lp == hyk::LP_VALUE)
      st = launch_pass0<SD, T, H, P, hyk::LP_VALUE>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
    else if (lp == hyk::LP_REF1)
      st = launch_pass0<SD, T, H, P, hyk::LP_REF1>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
    else if (lp == hyk::LP_REFM)
      st = launch_pass0<SD, T, H, P, hyk::LP_REFM>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
    else
      st = launch_pass0<SD, T, H, P, hyk::LP_ANY>(p, sd, d0, nd, w0, n_digits, b, c, s, out);
    if (st != HY_OK) return st;
  }
  hipLaunchKernelGGL(hyk::seg_bounds, dim3((n_digits + 1 + 255) / 256), dim3(256), 0, s, b.off, p.n_tiles1, n_digits,
                     b.total, b.segA);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// One record pass over segments sg (tile prefix and owners filled, grid = an upper bound of its tiles): histogram
// (from the digit bytes dig_in when the previous pass wrote them, else from the records), scan, stable scatter by digit
// (bits [shift, shift + w)) writing the next pass's digit bytes (nd), then the bounds of the n_groups * 2^w parts.
template <typename SD, typename H, typename P>
hy_status record_pass(const SideBufs<H, P>& b, const hyk::Segs& sg, const hyk::Groups& gr,
                      uint32_t n_groups, uint64_t grid, uint32_t bits, uint32_t shift, uint32_t w, uint32_t seed,
                      const hyk::Rec<H, P>* in, const uint8_t* dig_in, const hyk::NextDigit& nd,
                      const hyk::RecOut<H, P>& out, const uint64_t* total, uint32_t* bounds, const Common& c,
                      hipStream_t s, uint64_t rows) {
  const uint32_t n_digits = 1u << w;
  hyk::Digit dg{full_mask(bits), shift, n_digits - 1u, seed, g_key_hash, rank_ballot()};
  if (grid) {
    {
      KTimer kt_((std::string("part2_hist.") + SD::name).c_str(), s, rows);
      if (dig_in)
        hipLaunchKernelGGL(hyk::part2_hist_bytes<SD>, dim3(static_cast<uint32_t>(grid)), dim3(hyk::PART_THREADS), 0, s,
                           sg, n_digits, dig_in, b.hist);
      else
        hipLaunchKernelGGL((hyk::part2_hist<SD, H, P>), dim3(static_cast<uint32_t>(grid)), dim3(hyk::PART_THREADS), 0, s,
                           sg, dg, n_digits, in, b.hist);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    // (scanned over the tiles that exist, not the grid's upper bound)
    hy_status st = run_scan(b.hist, b.off, grid * n_digits, c, s, nullptr, sg.seg_tile_begin + sg.n_segs, n_digits);
    if (st != HY_OK) return st;
    {
      KTimer kt_((std::string("part2_scatter.") + SD::name).c_str(), s, rows);
      hipLaunchKernelGGL((hyk::part2_scatter<SD, H, P>), dim3(static_cast<uint32_t>(grid)), dim3(hyk::PART_THREADS), 0,
                         s, sg, dg, nd, static_cast<int>(w), n_digits, in, b.off, out);
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
// the two record buffers (and, when dig_in is given, the two digit-byte buffers). On return *recs / *bounds hold the
// final records and partition bounds.
template <typename SD, typename H, typename P>
hy_status local_passes(SideBufs<H, P>& b, const std::vector<uint32_t>& w, size_t first,
                       uint32_t bits, uint32_t seed, hyk::Rec<H, P>* in, hyk::Rec<H, P>* spare, const uint8_t* dig_in,
                       uint8_t* dig_spare, uint32_t* seg, uint32_t* seg_spare, uint64_t n_segs,
                       const uint64_t* total, uint64_t rows, const Common& c, hipStream_t s, hyk::Rec<H, P>** recs,
                       uint32_t** bounds, const hyk::RecOut<H, P>* last_out = nullptr) {
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
    const hyk::NextDigit nd = next_digit(w, i, bits, dig_in ? dig_spare : nullptr);
    const hyk::RecOut<H, P> out = (last_out && i + 1 == w.size()) ? *last_out : aos_out<H, P>(spare);
    st = record_pass<SD, H, P>(b, sg, hyk::Groups{nullptr, nullptr, nullptr}, static_cast<uint32_t>(n_segs), grid,
                           bits, below, w[i], seed, in, dig_in, nd, out, total, seg_spare, c, s, rows);
    if (st != HY_OK) return st;
    std::swap(in, spare);
    std::swap(seg, seg_spare);
    if (nd.bytes) {
      uint8_t* written = nd.bytes;
      dig_spare = const_cast<uint8_t*>(dig_in);
      dig_in = written;
    } else {
      dig_in = nullptr;
    }
    n_segs <<= w[i];
  }
  *recs = in;
  *bounds = seg;
  return HY_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Pass 0 in Infinity-Cache-sized row blocks (hyk::part1_count / part1_fill, join.hip): per block a counting read, the
// block's histogram scan and a second read - served on-die - that writes the scan output and the stable scatter into
// the block's own region; the first record pass then reads every bucket as its runs in block order (block_geometry).
// Opt-in (HY_BLOCKED=1) for single-GPU sides with two or more radix digits; HY_BLOCK_MB sets the input bytes per block
// (default 128 MiB: the block plus what its fill writes stays within the 256 MiB Infinity Cache,
// profiles/r05_mall_probe.jsonl). Measured on MI355X at SF100 (round 5, profiles/r05_blocked_ab.txt): SLOWER than the
// classic passes - headline 8.47 ms against 7.03 ms. The re-read is nearly free, but the passes are not bandwidth-bound:
// per 128 MB block part1_count takes 52-56 us (2.4 TB/s) and part1_fill 108 us, whose ranking and staging run over
// every row of the block where part1_spread handles only the compacted matches (probe side 23 x (56 + 108) us + 23 x
// ~25 us of scans, totals and launch gaps = 4.3 ms against 1.24 + 1.32 ms).
// ---------------------------------------------------------------------------------------------------------------
constexpr uint32_t MAX_BLOCKS = 64;

inline bool blocked_enabled() { return knobs().blocked; }
inline uint64_t block_target_bytes() { return knobs().block_bytes; }
inline uint64_t block_target_rows_override() { return knobs().block_rows; }

// Input bytes per row of a side's pass 0: the join column (through a PosList also the 8-byte RowID) and the fused
// scan's predicate column.
inline uint64_t pass0_row_bytes(const SidePlan& p, uint32_t key_bytes) {
  bool ref = false;
  for (const auto& c : p.chunks) ref = ref || c.pos_list != nullptr;
  uint64_t b = key_bytes + (ref ? 8 : 0);
  if (p.filtered) {
    uint64_t fb = 1;
    for (const auto& f : p.filter)
      if (f.column.size) fb = std::max<uint64_t>(fb, f.column.kind == HY_COL_DICT ? f.column.vid_width : 8);
    b += fb;
  }
  return b;
}

// Blocks of a side (0: not blocked): pass-0 spans split into contiguous ranges of about block_target_bytes() of input.
inline uint32_t block_count(const SidePlan& p, uint32_t key_bytes, size_t plan_digits, bool int32_keys) {
  // (instantiated for int32 hashed keys only: an opt-in experiment need not multiply the other types' kernels)
  if (!int32_keys || !blocked_enabled() || plan_digits < 2 || p.n_tiles1 == 0) return 0;
  uint64_t k;
  if (const uint64_t rows = block_target_rows_override())
    k = (p.n_rows + rows - 1) / std::max<uint64_t>(rows, 1);
  else
    k = (p.n_rows * pass0_row_bytes(p, key_bytes) + block_target_bytes() - 1) / block_target_bytes();
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>({k, MAX_BLOCKS, p.n_tiles1})));
}

struct BlockPlan {
  uint32_t n = 0;
  std::vector<uint64_t> t0;        // n + 1 span bounds
  std::vector<uint32_t> rec_base;  // first row of each block's first span = start of its record region
  std::vector<uint32_t> c_lo;      // n + 1: chunks whose first span lies in block k are [c_lo[k], c_lo[k + 1])
};

inline BlockPlan block_plan(const SidePlan& p, uint32_t n) {
  BlockPlan b;
  b.n = n;
  b.t0.resize(n + 1);
  b.rec_base.resize(n);
  const uint64_t span = uint64_t(p.sub) * hyk::PART_TILE;
  size_t c = 0;
  for (uint32_t k = 0; k <= n; ++k) {
    b.t0[k] = p.n_tiles1 * k / n;
    if (k == n) break;
    while (c + 1 < p.chunks.size() && p.tile_begin[c + 1] <= b.t0[k]) ++c;  // the chunk holding span t0 (non-empty)
    b.rec_base[k] = static_cast<uint32_t>(p.row_begin[c] + (b.t0[k] - p.tile_begin[c]) * span);
  }
  // chunk_begin entries (n_chunks + 1, the last at tile_begin = n_tiles) by the block holding their first span
  b.c_lo.resize(n + 1);
  size_t cc = 0;
  for (uint32_t k = 0; k < n; ++k) {
    while (cc <= p.chunks.size() && p.tile_begin[cc] < b.t0[k]) ++cc;
    b.c_lo[k] = static_cast<uint32_t>(cc);
  }
  b.c_lo[n] = static_cast<uint32_t>(p.chunks.size() + 1);
  return b;
}

template <typename SD, typename T, typename H, int LP, int FK, bool PF>
hy_status launch_blocks(const SidePlan& p, const BlockPlan& bl, const hyk::Side& sd, const hyk::Digit& d0,
                        const hyk::NextDigit& nd, uint32_t n_digits, SideBufs<H, uint32_t>& b, const Common& c,
                        hipStream_t s, hyk::Rec<H, uint32_t>* out) {
  constexpr bool filt = FK != hyk::FK_NONE;
  if (filt) HY_HIP(hipMemsetAsync(b.scan_base, 0, 8, s));
  for (uint32_t k = 0; k < bl.n; ++k) {
    const uint64_t t0 = bl.t0[k];
    const uint32_t nt = static_cast<uint32_t>(bl.t0[k + 1] - t0);
    {
      KTimer kt_((std::string("part1_count.") + SD::name).c_str(), s, p.n_rows);
      hipLaunchKernelGGL((hyk::part1_count<SD, T, H, LP, FK, PF>), dim3(nt), dim3(hyk::PART_THREADS), 0, s, sd, d0,
                         n_digits, t0, b.hist);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    hy_status st = run_scan(b.hist, b.off, uint64_t(n_digits + (filt ? 1 : 0)) * nt, c, s, b.grand_total);
    if (st != HY_OK) return st;
    hipLaunchKernelGGL(hyk::block_totals, dim3(1), dim3(256), 0, s, b.off, nt, n_digits, filt ? 1 : 0, b.grand_total, k,
                       bl.rec_base[k], t0, p.n_tiles1, k + 1 == bl.n ? 1 : 0, b.cls_begin, b.cls_count, b.scan_base,
                       b.tile_begin, bl.c_lo[k], bl.c_lo[k + 1], filt ? p.scan_chunk_begin : nullptr);
    HY_HIP(hipGetLastError());
    {
      KTimer kt_((std::string("part1_fill.") + SD::name).c_str(), s, p.n_rows);
      hipLaunchKernelGGL((hyk::part1_fill<SD, T, H, LP, FK, PF>), dim3(nt), dim3(hyk::PART_THREADS), 0, s, sd, d0, nd,
                         n_digits, t0, b.off, bl.rec_base[k], b.scan_base + k, out);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
  }
  return HY_OK;
}

// Filter kind / prefilter dispatch of one load path. A fused scan needs the join column in the hashed type and a
// data-table side (as launch_pass0); the prefiltered instances exist for probe sides only.
template <typename SD, typename T, typename H, int LP>
hy_status launch_blocks_lp(const SidePlan& p, const BlockPlan& bl, const hyk::Side& sd, const hyk::Digit& d0,
                           const hyk::NextDigit& nd, uint32_t n_digits, SideBufs<H, uint32_t>& b, const Common& c,
                           hipStream_t s, hyk::Rec<H, uint32_t>* out) {
  constexpr bool probe = std::is_same_v<SD, hyk::OnProbe>;
  const bool pf = probe && sd.bloom != nullptr;
  auto go = [&](auto fk_tag) -> hy_status {
    constexpr int FK = decltype(fk_tag)::value;
    if constexpr (probe) {
      if (pf) return launch_blocks<SD, T, H, LP, FK, true>(p, bl, sd, d0, nd, n_digits, b, c, s, out);
    }
    return launch_blocks<SD, T, H, LP, FK, false>(p, bl, sd, d0, nd, n_digits, b, c, s, out);
  };
  if (!p.filtered) return go(std::integral_constant<int, hyk::FK_NONE>{});
  if constexpr (LP != hyk::LP_REF1 && std::is_same_v<T, H>) {
    switch (filter_kind(p)) {
      case hyk::FK_DICT8:
        return go(std::integral_constant<int, hyk::FK_DICT8>{});
      case hyk::FK_DICT16:
        return go(std::integral_constant<int, hyk::FK_DICT16>{});
      case hyk::FK_DICT32:
        return go(std::integral_constant<int, hyk::FK_DICT32>{});
      default:
        return go(std::integral_constant<int, hyk::FK_ANY>{});
    }
  }
  return fail(HY_ERR_UNSUPPORTED, "fused scan on a side whose join column type is not the hashed type");
}

// The side's pass 0 in blocks, then the first record pass over the runs (grouped by bucket) and the remaining record
// passes. On return *recs / *bounds hold the final records and partition bounds (as local_passes).
template <typename SD, typename T, typename H>
hy_status blocked_side(const SidePlan& p, SideBufs<H, uint32_t>& b, uint32_t bits, const std::vector<uint32_t>& w,
                       uint32_t n_blocks, const hyk::Side& sd, const Common& c, hipStream_t s, hyk::Rec<H>** recs,
                       uint32_t** bounds, const hyk::RecOut<H, uint32_t>* last_out) {
  const uint32_t nd0 = 1u << w[0], w1 = w[1];
  const BlockPlan bl = block_plan(p, n_blocks);
  const hyk::Digit d0{full_mask(bits), bits - w[0], nd0 - 1u, sd.seed, g_key_hash, rank_ballot()};
  const hyk::NextDigit nd = next_digit(w, 0, bits, b.digA);
  HY_HIP(hipMemsetAsync(b.total, 0, 8, s));
  if (p.filtered && p.scan_chunk_begin) HY_HIP(hipMemsetAsync(p.scan_chunk_begin, 0, 8 * (p.chunks.size() + 1), s));
  hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((sd.n_chunks + 255) / 256), dim3(256), 0, s, b.tile_begin, sd.n_chunks,
                     b.tile_owner);
  HY_HIP(hipGetLastError());
  const int lp = load_path(p);
  hy_status st;
  if (lp == hyk::LP_VALUE)
    st = launch_blocks_lp<SD, T, H, hyk::LP_VALUE>(p, bl, sd, d0, nd, nd0, b, c, s, b.recA);
  else if (lp == hyk::LP_REF1)
    st = launch_blocks_lp<SD, T, H, hyk::LP_REF1>(p, bl, sd, d0, nd, nd0, b, c, s, b.recA);
  else
    st = launch_blocks_lp<SD, T, H, hyk::LP_ANY>(p, bl, sd, d0, nd, nd0, b, c, s, b.recA);
  if (st != HY_OK) return st;
  const uint32_t nseg = nd0 * bl.n;
  hipLaunchKernelGGL(hyk::block_geometry, dim3(1), dim3(256), 0, s, b.cls_begin, b.cls_count, bl.n, nd0,
                     static_cast<uint32_t>(span2()), 1u << w1, b.bseg_begin, b.bseg_end, b.bseg_stride, b.bseg_toff,
                     b.bseg_hbase, b.seg_tile_begin, b.group_hbase, b.group_tiles, b.group_out, b.total);
  HY_HIP(hipGetLastError());
  hipLaunchKernelGGL(hyk::fill_tile_owner, dim3(grid_for(nseg, 256)), dim3(256), 0, s, b.seg_tile_begin, nseg,
                     b.tile_owner);
  HY_HIP(hipGetLastError());
  const hyk::Segs sg{b.bseg_begin, b.seg_tile_begin, b.tile_owner, nseg, b.bseg_end, b.bseg_hbase, b.bseg_stride,
                     b.bseg_toff, sub2()};
  const hyk::Groups gr{b.group_hbase, b.group_tiles, b.group_out};
  const uint64_t grid = p.n_rows / span2() + 1 + nseg;
  const hyk::NextDigit nd1 = next_digit(w, 1, bits, b.digB);
  const hyk::RecOut<H, uint32_t> out1 = (last_out && w.size() == 2) ? *last_out : aos_out<H, uint32_t>(b.recB);
  st = record_pass<SD, H, uint32_t>(b, sg, gr, nd0, grid, bits, bits - w[0] - w1, w1, sd.seed, b.recA, nd.bytes, nd1,
                                    out1, b.total, b.segA, c, s, p.n_rows);
  if (st != HY_OK) return st;
  if (w.size() == 2) {
    *recs = b.recB;
    *bounds = b.segA;
    return HY_OK;
  }
  return local_passes<SD, H, uint32_t>(b, w, 2, bits, sd.seed, b.recB, b.recA, nd1.bytes, b.digA, b.segA, b.segB,
                                       uint64_t(nd0) << w1, b.total, p.n_rows, c, s, recs, bounds, last_out);
}

inline hyk::RowMap make_map(const uint64_t* dev_row_begin, const std::vector<uint64_t>& host_row_begin) {
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

// LDS rows of one build table: a fixed budget (two 1024-thread workgroups per CU), so the launch needs no partition
// sizes from the device; a partition with more build rows than one table holds (skewed keys) is processed as several
// LDS sub-tables in sequence.
template <typename H, typename P>
uint32_t lds_table_rows() {
  size_t budget = sizeof(hyk::Rec<H, P>) > 8 ? 72 * 1024 : 40 * 1024;
  if (const uint64_t b = knobs().lds_budget) budget = b;  // test knob
  uint32_t rows = hyk::LDS_MAX_ROWS;
  while (rows > 16 && hyk::table_bytes<H, P>(rows) > budget) rows = rows * 7 / 8;
  return rows;
}

// Per-partition LDS build/probe over partitioned records (partition bounds on the device; the records as the last pass
// wrote them: hyk::RecSrc or hyk::HashSrc). probe_rows_hint: an upper bound of the probe rows (probe_exact: their
// number); it picks the probe
// records per thread (JP) from the average partition, and the kernel: join_partition (one pass of probe records per
// partition; a partition needing more passes is listed for join_partition_multi) or, when the average partition needs
// several passes, join_partition_multi over every partition. Partitions with more build rows than one LDS table
// (skewed keys) are listed and joined by join_partition_skewed. The list kernels launch only when their list can be
// non-empty.
template <typename Src, typename P>
hy_status run_join_partitions(const uint32_t* build_begin, const uint32_t* probe_begin, uint32_t n_parts,
                              const Src& bsrc, const Src& psrc, const hyk::RowMap& bmap, const hyk::RowMap& pmap,
                              int32_t mode, hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,
                              uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,
                              const Common& c, hipStream_t s, uint64_t units, uint64_t probe_rows_hint,
                              bool probe_exact) {
  using H = typename Src::Key;
  constexpr int NT = hyk::JOIN_THREADS;
  // probe records per thread per pass: the wide variant (6) when the average partition needs more than 3/4 of JP_PER
  const uint64_t avg_probe = n_parts ? probe_rows_hint / n_parts : 0;
  const bool wide = avg_probe > static_cast<uint64_t>(3 * hyk::JP_PER * NT / 4);
  const uint32_t lds_max = lds_table_rows<H, P>();
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
  jd.n_skewed = c.misc + 3;
  jd.n_multi = c.misc + 4;
  jd.skewed = reinterpret_cast<uint32_t*>(c.join_status);  // (2^bits + 1) words of 8 B: 2 x n_parts entries
  jd.multi = jd.skewed + n_parts;
  jd.total = c.totals + 1;
  jd.trace = g_join_trace;
  HY_HIP(hipMemsetAsync(c.misc, 0, 64 * 4, s));
  HY_HIP(hipMemsetAsync(c.totals, 0, 8 * 2, s));
  constexpr int JW = Src::V == 1 ? 6 : 8;  // the wide variant's probe records per thread (a multiple of V)
  // most partitions need several probe passes (the average plus four standard deviations of a uniform spread exceeds
  // the wide pass): the multi-pass kernel takes every partition directly instead of the one-pass kernel deferring
  // nearly all of them (only when the probe rows are known: a filtered probe side's hint is its rows before the
  // filter). (Round 4 switched at 3/4 of the pass: TPC-H SF10's 7,324 probe rows per partition went to the count +
  // reload + write passes of join_partition_multi although nearly all fit one 8,192-record pass.)
  const double wide_pass = double(JW * NT - (Src::V - 1));
  const bool all_multi = probe_exact && double(avg_probe) + 4.0 * std::sqrt(double(avg_probe)) > wide_pass && !jd.trace;
  // join_partition_multi (JW records per thread): a two-pass partition keeps its first pass in LDS (jd.stash_rows)
  // when its table and the stash fit half a CU's LDS (two 1024-thread workgroups per CU)
  hyk::JoinDesc jdm = jd;
  size_t lds_m = lds;
  if (knobs().join_stash) {
    const size_t stash = size_t(JW) * NT * (sizeof(P) + 4);
    const size_t half = 80 * 1024 - 1024;  // (the kernel's static LDS: s_tot, s_base)
    uint32_t rows = std::min<uint32_t>(lds_max, hyk::LDS_MAX_ROWS);
    while (rows > 16 && hyk::table_bytes<H, P>(rows) + stash > half) rows = rows * 15 / 16;
    // (no hipFuncSetAttribute for the > 64 KB launch: HIP ignores the dynamic-LDS attribute on AMD devices, and calling
    // it from several threads at once while others launched aborted the process in test_concurrent_operators)
    if (rows > 16) {
      jdm.stash_rows = rows;
      lds_m = std::max(lds, hyk::table_bytes<H, P>(rows) + stash);
    }
  }
  if (n_parts && all_multi) {
    jdm.multi = nullptr;
    KTimer kt_("join_partition", s, units);
    hipLaunchKernelGGL((hyk::join_partition_multi<Src, P, JW, NT>), dim3(n_parts), dim3(NT), lds_m, s, jdm, bsrc, psrc,
                       out_build, out_probe, partition_begin, partition_counts);
    kt_.done();
    HY_HIP(hipGetLastError());
  }
  if (n_parts && !all_multi) {
    {
      KTimer kt_("join_partition", s, units);
      auto launch = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(n_parts), dim3(NT), lds, s, jd, bsrc, psrc, out_build, out_probe,
                           partition_begin, partition_counts);
      };
      if (jd.trace)  // debug phase-trace instance (hy_debug_set_join_trace)
        wide ? launch(hyk::join_partition<Src, P, true, JW, NT>) : launch(hyk::join_partition<Src, P, true, 4, NT>);
      else
        wide ? launch(hyk::join_partition<Src, P, false, JW, NT>) : launch(hyk::join_partition<Src, P, false, 4, NT>);
      kt_.done();
    }
    HY_HIP(hipGetLastError());
    // deferred partitions: more probe records than one pass (at most probe_rows / (pass - V + 2) of them), more
    // build rows than one table (at most build_rows / (lds_max + 1)); each list's kernel only when it can be non-empty
    const uint32_t per_pass = static_cast<uint32_t>((wide ? JW : 4) * NT - (Src::V - 1));
    const uint64_t max_multi = std::min<uint64_t>(n_parts, probe_rows_hint / (uint64_t(per_pass) + 1));
    if (max_multi) {
      KTimer kt_("join_partition_multi", s, units);
      const dim3 g(static_cast<uint32_t>(std::min<uint64_t>(max_multi, 512)));
      if (wide)
        hipLaunchKernelGGL((hyk::join_partition_multi<Src, P, JW, NT>), g, dim3(NT), lds_m, s, jdm, bsrc, psrc,
                           out_build, out_probe, partition_begin, partition_counts);
      else
        hipLaunchKernelGGL((hyk::join_partition_multi<Src, P, 4, NT>), g, dim3(NT), lds, s, jd, bsrc, psrc, out_build,
                           out_probe, partition_begin, partition_counts);
      kt_.done();
      HY_HIP(hipGetLastError());
    }
  }
  if (n_parts) {
    const uint64_t build_rows = units > probe_rows_hint ? units - probe_rows_hint : 0;
    const uint64_t max_skewed = std::min<uint64_t>(n_parts, build_rows / (uint64_t(lds_max) + 1));
    if (max_skewed) {
      KTimer kt_("join_partition_skewed", s, units);
      hipLaunchKernelGGL((hyk::join_partition_skewed<Src, P, NT>), dim3(static_cast<uint32_t>(std::min<uint64_t>(max_skewed, 512))),
                         dim3(NT), lds, s, jd, bsrc, psrc, out_build, out_probe, partition_begin, partition_counts);
      kt_.done();
      HY_HIP(hipGetLastError());
    }
  }
  if (capture_state().capturing) {
    capture_state().misc = c.misc;
    capture_state().totals = c.totals;
    return HY_OK;
  }
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

inline SideSizes sizes_of(const SidePlan& p, bool digit_bytes, uint32_t blocks = 0) {
  SideSizes z;
  z.blocks = blocks;
  z.rows = p.n_rows;
  z.tiles1 = p.n_tiles1;
  z.sub = p.sub;
  z.n_chunks = p.chunks.size();
  z.n_referenced = p.referenced.size();
  z.filtered = p.filtered;
  z.digit_bytes = digit_bytes;
  return z;
}

template <typename H>
size_t classic_join_bytes(const SidePlan& bp, const SidePlan& pp, uint32_t bits) {
  const auto w = digit_plan(bits, 0);
  const bool db = w.size() > 1 && digit_bytes_enabled();
  constexpr bool i32 = std::is_same_v<H, int32_t>;
  const uint32_t kb = block_count(bp, sizeof(H), w.size(), i32), kp = block_count(pp, sizeof(H), w.size(), i32);
  Carver cv{nullptr, 0};
  SideBufs<H> a, b;
  carve_side<H, uint32_t>(cv, sizes_of(bp, db, kb), bits, w, 1, true, a);
  carve_side<H, uint32_t>(cv, sizes_of(pp, db, kp), bits, w, 1, true, b);
  uint64_t ha, hb, t;
  pass_sizes(sizes_of(bp, db, kb), w, 1, &ha, &t);
  pass_sizes(sizes_of(pp, db, kp), w, 1, &hb, &t);
  Common c, cb;  // (join_typed: the probe side's and the build side's)
  const uint64_t fb_scan = filter_buckets(bloom_words(bp.n_rows, pp.n_rows), bp.n_rows).scan_len;
  carve_common(cv, std::max({ha, hb, (uint64_t(1) << bits) + 1, fb_scan}), bits, &c);
  carve_common(cv, std::max({ha, hb, (uint64_t(1) << bits) + 1}), bits, &cb);
  cv.take<uint32_t>(prefilter_words(bloom_words(bp.n_rows, pp.n_rows), bp.n_rows));
  return cv.used + 256;
}

template <typename H, typename P>
hy_status upload_side(const SidePlan& p, const SideBufs<H, P>& b, hipStream_t s) {
  if (p.device_ready) return HY_OK;
  auto upload = [&](auto* dst, const auto& v) -> hy_status {
    if (!v.empty()) HY_STAGE(dst, v.data(), sizeof(v[0]) * v.size(), s);
    return HY_OK;
  };
  if (upload(b.chunks, p.chunks) || upload(b.tile_begin, p.tile_begin) || upload(b.row_begin, p.row_begin) ||
      upload(b.referenced, p.referenced) || upload(b.ref_row_begin, p.ref_row_begin))
    return HY_ERR_DEVICE;
  if (p.filtered && upload(b.filter, p.filter)) return HY_ERR_DEVICE;
  return HY_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Single-pass first radix pass (hyk::part1_onepass) for plans of two or more digits: one read of the column chunks
// writes the pass-1 buckets as NCLASS gapped regions each; the first record pass reads them as interleaved segments
// (the distributed receiver's geometry, computed on the device by hyk::onepass_geometry) and writes compact records.
// Opt-in (HY_ONEPASS=1): measured on MI355X at SF100 it is SLOWER than the two-read path (probe side 2.9-3.4 ms vs
// 3.0 ms for part1_compact + part1_spread, build 0.78-0.94 vs 0.71 ms; per-class tickets vs a static order and 1-16
// predecessors per look-back round trip all measured, profiles/r02g_onepass_variants.txt): a workgroup waiting on its
// predecessors' digit counts holds its slot, so fewer loads are in flight than in the two streaming kernels. A region
// overflow (skewed keys) falls back to the two-read path.
// ---------------------------------------------------------------------------------------------------------------
inline bool onepass_enabled() {
  return knobs().onepass;
}

struct OnepassGeo {
  uint64_t cap = 0;                 // records per (bucket, class) region
  uint64_t gapped = 0;              // records of the gapped buffer
  uint32_t grid = 0;
  uint32_t class_begin[hyk::NCLASS + 1] = {};
};

// Classes = NCLASS balanced contiguous tile ranges; cap = the expected records of a region if every row of the
// largest class took part, with 1/8 slack plus one tile (HY_ONEPASS_CAP_DIV overrides the slack divisor: tests).
inline OnepassGeo onepass_geo(const SidePlan& p, uint32_t n_digits0) {
  OnepassGeo g;
  const uint64_t n = p.n_tiles1, q = n / hyk::NCLASS, r = n % hyk::NCLASS;
  for (uint32_t x = 0; x <= hyk::NCLASS; ++x) g.class_begin[x] = static_cast<uint32_t>(x * q + std::min<uint64_t>(x, r));
  const uint64_t max_tiles = q + (r ? 1 : 0);
  g.grid = static_cast<uint32_t>(max_tiles * hyk::NCLASS);
  const uint64_t class_rows = max_tiles * hyk::PART_TILE;
  uint64_t div = 8;
  div = knobs().onepass_cap_div;
  const uint64_t expect = (class_rows + n_digits0 - 1) / n_digits0;
  g.cap = std::min<uint64_t>(class_rows, expect + expect / div + (div > 1000 ? 0 : hyk::PART_TILE));
  if (const uint64_t cap = knobs().onepass_cap) g.cap = cap;
  g.gapped = g.cap * n_digits0 * hyk::NCLASS;
  return g;
}

inline bool onepass_ok(const SidePlan& p, const std::vector<uint32_t>& w) {
  if (!onepass_enabled() || w.size() < 2 || p.n_tiles1 == 0) return false;
  return onepass_geo(p, 1u << w[0]).gapped < (uint64_t(1) << 31);
}

template <typename H>
struct OneBufs {
  SideBufs<H> b;
  uint32_t *class_begin, *ticket, *status, *class_count, *flags, *match_count, *tile_off;
  uint64_t* match_bits;
  uint32_t *seg_begin, *seg_end, *seg_stride, *seg_toff, *group_tiles, *group_out, *owner;
  uint64_t *seg_tile_begin, *seg_hbase, *group_hbase;
  uint64_t hist_words = 1, max_tiles = 1;
};

template <typename H>
void carve_onepass(Carver& cv, const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w, OneBufs<H>& o) {
  const uint32_t nd0 = 1u << w[0];
  const OnepassGeo g = onepass_geo(p, nd0);
  const uint64_t nseg = uint64_t(nd0) * hyk::NCLASS;
  const uint64_t row_tiles = p.n_rows / span2() + 1;
  o.hist_words = (row_tiles + nseg) * (uint64_t(1) << w[1]);
  o.max_tiles = std::max<uint64_t>(p.n_tiles1, row_tiles + nseg);
  uint64_t segs = uint64_t(nd0) << w[1];
  for (size_t i = 2; i < w.size(); ++i) {
    o.hist_words = std::max(o.hist_words, (row_tiles + segs) * (uint64_t(1) << w[i]));
    o.max_tiles = std::max(o.max_tiles, row_tiles + segs);
    segs <<= w[i];
  }
  SideBufs<H>& b = o.b;
  b.chunks = cv.take<hyk::SrcChunk>(std::max<size_t>(1, p.chunks.size()));
  b.tile_begin = cv.take<uint64_t>(p.chunks.size() + 1);
  b.row_begin = cv.take<uint64_t>(p.chunks.size() + 1);
  b.referenced = cv.take<hyk::SrcChunk>(std::max<size_t>(1, p.referenced.size()));
  b.ref_row_begin = cv.take<uint64_t>(p.referenced.size() + 1);
  b.filter = p.filtered ? cv.take<hy_scan_chunk>(std::max<size_t>(1, p.chunks.size())) : nullptr;
  b.hist = cv.take<uint32_t>(o.hist_words);
  b.off = cv.take<uint32_t>(o.hist_words);
  b.recA = cv.take<hyk::Rec<H>>(std::max<uint64_t>(1, g.gapped));
  b.recB = cv.take<hyk::Rec<H>>(std::max<uint64_t>(1, p.n_rows));
  b.span_count = nullptr;
  b.mbits = nullptr;
  b.digA = cv.take<uint8_t>(std::max<uint64_t>(16, g.gapped));
  b.digB = cv.take<uint8_t>(std::max<uint64_t>(16, p.n_rows));
  const uint64_t parts = (uint64_t(1) << bits) + 1;
  b.segA = cv.take<uint32_t>(parts);
  b.segB = cv.take<uint32_t>(parts);
  b.seg_tile_begin = cv.take<uint64_t>(parts);
  b.tile_counts = cv.take<uint32_t>(parts);
  b.tile_excl = cv.take<uint32_t>(parts);
  b.tile_owner = cv.take<uint32_t>(o.max_tiles);
  b.total = cv.take<uint64_t>(1);
  b.grand_total = cv.take<uint64_t>(1);
  o.class_begin = cv.take<uint32_t>(hyk::NCLASS + 1);
  o.ticket = cv.take<uint32_t>(hyk::NCLASS);
  o.status = cv.take<uint32_t>(p.n_tiles1 * 256);
  o.class_count = cv.take<uint32_t>(hyk::NCLASS * 256);
  o.flags = cv.take<uint32_t>(1);
  const bool scan = p.filtered && p.scan_out != nullptr;
  o.match_bits = scan ? cv.take<uint64_t>(p.n_tiles1 * hyk::PART_WAVES * hyk::PART_ITEMS) : nullptr;
  o.match_count = scan ? cv.take<uint32_t>(p.n_tiles1) : nullptr;
  o.tile_off = scan ? cv.take<uint32_t>(p.n_tiles1) : nullptr;
  o.seg_begin = cv.take<uint32_t>(nseg);
  o.seg_end = cv.take<uint32_t>(nseg);
  o.seg_stride = cv.take<uint32_t>(nseg);
  o.seg_toff = cv.take<uint32_t>(nseg);
  o.seg_hbase = cv.take<uint64_t>(nseg);
  o.seg_tile_begin = cv.take<uint64_t>(nseg + 1);
  o.group_hbase = cv.take<uint64_t>(nd0);
  o.group_tiles = cv.take<uint32_t>(nd0);
  o.group_out = cv.take<uint32_t>(nd0);
  o.owner = cv.take<uint32_t>(row_tiles + nseg);
}

template <typename H>
size_t onepass_bytes(const SidePlan& bp, const SidePlan& pp, uint32_t bits) {
  const auto w = digit_plan(bits, 0);
  Carver cv{nullptr, 0};
  OneBufs<H> a, b;
  carve_onepass<H>(cv, bp, bits, w, a);
  carve_onepass<H>(cv, pp, bits, w, b);
  Common c;
  carve_common(cv, std::max({a.hist_words, b.hist_words, bp.n_tiles1, pp.n_tiles1, (uint64_t(1) << bits) + 1}), bits,
               &c);
  return cv.used + 256;
}

// The side's pass 0 (part1_onepass), the fused scan's output, the first record pass over the gapped regions and the
// remaining record passes. *flags_host receives the overflow / look-back flags once the stream has synchronised.
template <typename T, typename H, int LP, int FK>
hy_status onepass_launch(const char* tag, const hyk::Side& sd, const hyk::Digit& d0, const hyk::NextDigit& nd,
                         uint32_t n_digits, const hyk::OnePass& op, uint32_t grid, hyk::Rec<H>* out, hipStream_t s,
                         uint64_t rows) {
  KTimer kt_((std::string("part1_onepass.") + tag).c_str(), s, rows);
  hipLaunchKernelGGL((hyk::part1_onepass<T, H, LP, FK>), dim3(grid), dim3(hyk::PART_THREADS), 0, s, sd, d0, nd,
                     n_digits, op, out);
  kt_.done();
  HY_HIP(hipGetLastError());
  return HY_OK;
}

template <typename T, typename H>
hy_status onepass_side(const char* tag, const SidePlan& p, OneBufs<H>& o, uint32_t bits, const std::vector<uint32_t>& w,
                       uint32_t seed, bool keep_nulls, const Common& c, hipStream_t s, uint32_t* flags_host,
                       hyk::Rec<H>** recs, uint32_t** bounds) {
  SideBufs<H>& b = o.b;
  const uint32_t nd0 = 1u << w[0], w1 = w[1];
  const OnepassGeo g = onepass_geo(p, nd0);
  HY_STAGE(o.class_begin, g.class_begin, sizeof(g.class_begin), s);
  HY_HIP(hipMemsetAsync(o.ticket, 0, 4 * hyk::NCLASS, s));
  HY_HIP(hipMemsetAsync(o.status, 0, 4 * 256 * p.n_tiles1, s));
  HY_HIP(hipMemsetAsync(o.class_count, 0, 4 * 256 * hyk::NCLASS, s));
  HY_HIP(hipMemsetAsync(o.flags, 0, 4, s));
  if (p.filtered && p.scan_chunk_begin) HY_HIP(hipMemsetAsync(p.scan_chunk_begin, 0, 8 * (p.chunks.size() + 1), s));
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
  sd.ref_base = p.ref_base;
  sd.sub = 1;
  sd.filter = p.filtered ? b.filter : nullptr;
  sd.filter_const = p.filter_const;
  sd.filter_type = p.filter_type;
  sd.scan_out = p.scan_out;
  hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((sd.n_chunks + 255) / 256), dim3(256), 0, s, b.tile_begin, sd.n_chunks,
                     b.tile_owner);
  HY_HIP(hipGetLastError());
  const hyk::Digit d0{full_mask(bits), bits - w[0], nd0 - 1u, seed, g_key_hash, rank_ballot()};
  const hyk::NextDigit nd = next_digit(w, 0, bits, b.digA);
  static const uint32_t win = [] {
    const char* e = std::getenv("HY_ONEPASS_WIN");
    const long v = e ? std::strtol(e, nullptr, 10) : 1;
    return static_cast<uint32_t>(std::min<long>(std::max<long>(v, 1), hyk::LB_WIN));
  }();
  static const uint32_t static_order = std::getenv("HY_ONEPASS_STATIC") ? 1u : 0u;
  const hyk::OnePass op{o.class_begin, o.ticket,      o.status, o.class_count, g.cap, o.flags,
                        o.match_bits,  o.match_count, win,      static_order};
  const int lp = load_path(p);
  hy_status st = HY_OK;
  if (p.filtered) {
    if constexpr (std::is_same_v<T, H>) {
      const int fk = filter_kind(p);
      auto go = [&](auto fk_tag) {
        constexpr int FK = decltype(fk_tag)::value;
        return lp == hyk::LP_VALUE
                   ? onepass_launch<T, H, hyk::LP_VALUE, FK>(tag, sd, d0, nd, nd0, op, g.grid, b.recA, s, p.n_rows)
                   : onepass_launch<T, H, hyk::LP_ANY, FK>(tag, sd, d0, nd, nd0, op, g.grid, b.recA, s, p.n_rows);
      };
      if (fk == hyk::FK_DICT8)
        st = go(std::integral_constant<int, hyk::FK_DICT8>{});
      else if (fk == hyk::FK_DICT16)
        st = go(std::integral_constant<int, hyk::FK_DICT16>{});
      else if (fk == hyk::FK_DICT32)
        st = go(std::integral_constant<int, hyk::FK_DICT32>{});
      else
        st = go(std::integral_constant<int, hyk::FK_ANY>{});
    } else {
      return fail(HY_ERR_UNSUPPORTED, "fused scan on a side whose join column type is not the hashed type");
    }
  } else if (lp == hyk::LP_VALUE) {
    st = onepass_launch<T, H, hyk::LP_VALUE, hyk::FK_NONE>(tag, sd, d0, nd, nd0, op, g.grid, b.recA, s, p.n_rows);
  } else if (lp == hyk::LP_REF1) {
    st = onepass_launch<T, H, hyk::LP_REF1, hyk::FK_NONE>(tag, sd, d0, nd, nd0, op, g.grid, b.recA, s, p.n_rows);
  } else {
    st = onepass_launch<T, H, hyk::LP_ANY, hyk::FK_NONE>(tag, sd, d0, nd, nd0, op, g.grid, b.recA, s, p.n_rows);
  }
  if (st != HY_OK) return st;
  if (o.match_bits != nullptr) {  // the fused scan's output
    st = run_scan(o.match_count, o.tile_off, p.n_tiles1, c, s, b.grand_total);
    if (st != HY_OK) return st;
    KTimer kt_((std::string("part1_scan_expand.") + tag).c_str(), s, p.n_rows);
    hipLaunchKernelGGL(hyk::part1_scan_expand, dim3(static_cast<uint32_t>(p.n_tiles1)), dim3(hyk::PART_THREADS), 0, s,
                       sd, o.match_bits, o.tile_off, b.grand_total, p.scan_chunk_begin);
    kt_.done();
    HY_HIP(hipGetLastError());
  }
  HY_HIP(hipMemcpyAsync(flags_host, o.flags, 4, hipMemcpyDeviceToHost, s));
  const uint32_t nseg = nd0 * hyk::NCLASS;
  hipLaunchKernelGGL(hyk::onepass_geometry, dim3(1), dim3(256), 0, s, o.class_count, nd0, g.cap, span2(), 1u << w1,
                     o.seg_begin, o.seg_end, o.seg_stride, o.seg_toff, o.seg_hbase, o.seg_tile_begin, o.group_hbase,
                     o.group_tiles, o.group_out, b.total);
  HY_HIP(hipGetLastError());
  hipLaunchKernelGGL(hyk::fill_tile_owner, dim3(grid_for(nseg, 256)), dim3(256), 0, s, o.seg_tile_begin, nseg, o.owner);
  HY_HIP(hipGetLastError());
  const hyk::Segs sg{o.seg_begin, o.seg_tile_begin, o.owner, nseg, o.seg_end, o.seg_hbase, o.seg_stride, o.seg_toff,
                     sub2()};
  const hyk::Groups gr{o.group_hbase, o.group_tiles, o.group_out};
  const uint64_t grid = p.n_rows / span2() + 1 + nseg;
  const hyk::NextDigit nd1 = next_digit(w, 1, bits, b.digB);
  st = by_side(tag, [&](auto sdt) {
    return record_pass<decltype(sdt), H, uint32_t>(b, sg, gr, nd0, grid, bits, bits - w[0] - w1, w1, seed, b.recA,
                                                   b.digA, nd1, aos_out<H, uint32_t>(b.recB), b.total, b.segA, c, s,
                                                   p.n_rows);
  });
  if (st != HY_OK) return st;
  if (w.size() == 2) {
    *recs = b.recB;
    *bounds = b.segA;
    return HY_OK;
  }
  return by_side(tag, [&](auto sdt) {
    return local_passes<decltype(sdt), H, uint32_t>(b, w, 2, bits, seed, b.recB, b.recA, b.digB, b.digA, b.segA,
                                                    b.segB, uint64_t(nd0) << w1, b.total, p.n_rows, c, s, recs, bounds);
  });
}

// Both sides through onepass_side, then the partition joins. *overflow = the sides' flags (nonzero: results invalid,
// the caller reruns the two-read path).
template <typename TB, typename TP, typename H>
hy_status join_typed_onepass(const SidePlan& bp, const SidePlan& pp, const hy_join_params* prm, hy_row_id* out_build,
                             hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                             uint32_t* partition_counts, hy_join_result* result, void* workspace,
                             size_t workspace_bytes, hipStream_t s, uint32_t* overflow) {
  const uint32_t bits = prm->radix_bits;
  const auto w = digit_plan(bits, 0);
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  OneBufs<H> ob, op;
  carve_onepass<H>(cv, bp, bits, w, ob);
  carve_onepass<H>(cv, pp, bits, w, op);
  Common c{};
  carve_common(cv, std::max({ob.hist_words, op.hist_words, bp.n_tiles1, pp.n_tiles1, (uint64_t(1) << bits) + 1}), bits,
               &c);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "join workspace too small");
  if (upload_side(bp, ob.b, s) || upload_side(pp, op.b, s)) return HY_ERR_DEVICE;
  const bool keep_nulls = prm->mode == HY_JOIN_LEFT || prm->mode == HY_JOIN_RIGHT;
  static thread_local uint32_t flags[2];
  flags[0] = flags[1] = 0;
  hyk::Rec<H>* recs[2] = {nullptr, nullptr};
  uint32_t* bounds[2] = {nullptr, nullptr};
  hy_status st = onepass_side<TB, H>("build", bp, ob, bits, w, prm->seed, false, c, s, &flags[0], &recs[0], &bounds[0]);
  if (st != HY_OK) return st;
  st = onepass_side<TP, H>("probe", pp, op, bits, w, prm->seed, keep_nulls, c, s, &flags[1], &recs[1], &bounds[1]);
  if (st != HY_OK) return st;
  const hyk::RowMap bmap = bp.fuse ? make_map(ob.b.ref_row_begin, bp.ref_row_begin) : make_map(ob.b.row_begin, bp.row_begin);
  const hyk::RowMap pmap = pp.fuse ? make_map(op.b.ref_row_begin, pp.ref_row_begin) : make_map(op.b.row_begin, pp.row_begin);
  st = run_join_partitions<hyk::RecSrc<H, uint32_t>, uint32_t>(bounds[0], bounds[1], 1u << bits,
                                                               hyk::RecSrc<H, uint32_t>{recs[0]},
                                                               hyk::RecSrc<H, uint32_t>{recs[1]}, bmap, pmap, prm->mode,
                                        out_build, out_probe, out_capacity, partition_begin, partition_counts, result,
                                        c, s, bp.n_rows + pp.n_rows, pp.n_rows, !pp.filtered);
  HY_HIP(hipStreamSynchronize(s));  // the flags' copies (run_join_partitions has synchronised on success)
  *overflow = flags[0] | flags[1];
  return st;
}

// ---------------------------------------------------------------------------------------------------------------
// Direct partitioning of a side with a fused TableScan (kernels/join_direct.hip): span match counts, part1_direct
// (one read of the predicate and the keys; records into (span, bucket) regions), part2g_hist / part2g_scatter over
// (bucket, span group) run lists. Replaces part1_compact + part1_spread + the per-tile record pass of a two-digit plan:
// at SF100 the 8-byte record round trip (2.3 GB written, read back) and the per-tile histograms are gone. A region
// overflow (keys far more skewed than murmur2 spreads them) is detected on the device and the join reruns on the
// classic passes (join_typed). HY_JOIN_DIRECT=0 keeps the classic passes (A/B).
// ---------------------------------------------------------------------------------------------------------------
struct DirectPlan {
  bool ok = false;
  SidePlan plan;           // the side with spans of knobs().direct_span tiles
  uint64_t n_spans = 0;
  uint64_t regions = 0;    // records of all regions at their largest (every row matching)
  uint32_t groups = 0;     // span groups per bucket of the second pass (H)
  uint32_t per = 0;        // spans per group
  uint32_t nd0 = 0, nd1 = 0;
};

// Whether the direct passes take a side, and their geometry. keep_nulls / prefiltered sides stay on the classic
// passes (their records carry NULL rows or skip rows the scan matched).
template <typename H>
DirectPlan direct_plan(const SidePlan& p, uint32_t bits, bool keep_nulls, bool prefiltered) {
  DirectPlan d;
  const auto w = digit_plan(bits, 0);
  const JoinKnobs k = knobs();
  if (!k.direct || k.blocked || !p.filtered || w.size() != 2 || keep_nulls || prefiltered || p.fuse ||
      !p.referenced.empty())
    return d;
  if (filter_kind(p) == hyk::FK_NONE) return d;
  const int lp = load_path(p);
  if (lp != hyk::LP_VALUE && lp != hyk::LP_ANY) return d;
  d.plan = p;
  plan_spans(d.plan, k.direct_span);
  d.n_spans = d.plan.n_tiles1;
  if (d.n_spans == 0 || d.n_spans >= 0x7FFFFFFFull) return d;
  d.nd0 = 1u << w[0];
  d.nd1 = 1u << w[1];
  const uint64_t span_rows = uint64_t(d.plan.sub) * hyk::PART_TILE;
  uint64_t regions = 0;
  for (size_t c = 0; c < d.plan.chunks.size(); ++c) {
    const uint64_t rows = d.plan.chunks[c].size;
    for (uint64_t r0 = 0; r0 < rows; r0 += span_rows)
      regions += uint64_t(d.nd0) * hyk::direct_cap(static_cast<uint32_t>(std::min(span_rows, rows - r0)), d.nd0);
  }
  if (regions >= 0xFFFFFFFFull) return d;  // (record indexes of the regions are scanned in 32 bits)
  d.regions = regions;
  const uint64_t min_groups = (d.n_spans + hyk::GROUP_MAX_RUNS - 1) / hyk::GROUP_MAX_RUNS;
  uint64_t h = k.direct_groups ? k.direct_groups : std::max<uint64_t>(1, (1024 + d.nd0 - 1) / d.nd0);
  h = std::min<uint64_t>(std::max(h, min_groups), d.n_spans);
  d.per = static_cast<uint32_t>((d.n_spans + h - 1) / h);
  d.groups = static_cast<uint32_t>((d.n_spans + d.per - 1) / d.per);
  d.ok = true;
  return d;
}

template <typename H>
struct DirectBufs {
  SideBufs<H> b;  // the side's descriptors (chunks, spans, predicate chunks); nothing else of it is used
  uint32_t *span_cnt, *span_scan, *span_cap, *cap_words, *rbase32, *counts, *hist, *off, *bounds, *overflow;
  uint64_t* span_rbase;
  uint64_t* totals;  // [0] scan matches, [1] region records, [2] records taking part
  hyk::Rec<H>* regions;
  uint8_t* dig;
  hyk::Rec<H>* out;  // the last pass's records: {key, payload} or the hash-record (SoA) area
};

template <typename H>
void carve_direct(Carver& cv, const DirectPlan& d, uint32_t bits, DirectBufs<H>& o) {
  const SidePlan& p = d.plan;
  const size_t nc = p.chunks.size();
  o.b = SideBufs<H>{};
  o.b.chunks = cv.take<hyk::SrcChunk>(std::max<size_t>(1, nc));
  o.b.tile_begin = cv.take<uint64_t>(nc + 1);
  o.b.row_begin = cv.take<uint64_t>(nc + 1);
  o.b.referenced = cv.take<hyk::SrcChunk>(1);
  o.b.ref_row_begin = cv.take<uint64_t>(1);
  o.b.filter = cv.take<hy_scan_chunk>(std::max<size_t>(1, nc));
  o.b.tile_owner = cv.take<uint32_t>(std::max<uint64_t>(1, d.n_spans));
  const uint64_t ns = std::max<uint64_t>(1, d.n_spans);
  o.span_cnt = cv.take<uint32_t>(ns);
  o.span_scan = cv.take<uint32_t>(ns);
  o.span_cap = cv.take<uint32_t>(ns);
  o.cap_words = cv.take<uint32_t>(ns);
  o.rbase32 = cv.take<uint32_t>(ns);
  o.span_rbase = cv.take<uint64_t>(ns);
  o.counts = cv.take<uint32_t>(uint64_t(d.nd0) * ns);
  const uint64_t hw = uint64_t(d.nd0) * d.nd1 * std::max<uint32_t>(1, d.groups);
  o.hist = cv.take<uint32_t>(hw);
  o.off = cv.take<uint32_t>(hw);
  o.bounds = cv.take<uint32_t>((uint64_t(1) << bits) + 1);
  o.overflow = cv.take<uint32_t>(4);
  o.totals = cv.take<uint64_t>(4);
  o.regions = cv.take<hyk::Rec<H>>(std::max<uint64_t>(1, d.regions));
  o.dig = cv.take<uint8_t>(std::max<uint64_t>(16, d.regions));
  o.out = cv.take<hyk::Rec<H>>(std::max<uint64_t>(16, p.n_rows));
}

template <typename H>
size_t direct_scan_words(const DirectPlan& d) {
  return std::max<uint64_t>(d.n_spans, uint64_t(d.nd0) * d.nd1 * std::max<uint32_t>(1, d.groups));
}

template <typename SD, typename T, typename H, int LP, int FK>
void launch_part1_direct(const DirectPlan& d, const hyk::Side& sd, const hyk::Digit& d0, const hyk::NextDigit& nd,
                         const hyk::DirectGeo& g, hyk::Rec<H>* regions, hipStream_t s) {
  hipLaunchKernelGGL((hyk::part1_direct<SD, T, H, LP, FK>), dim3(static_cast<uint32_t>(d.n_spans)),
                     dim3(hyk::PART_THREADS), 0, s, sd, d0, nd, d.nd0, g, regions);
}

template <typename SD, typename T, typename H, int LP>
hy_status part1_direct_lp(const DirectPlan& d, int fk, const hyk::Side& sd, const hyk::Digit& d0,
                          const hyk::NextDigit& nd, const hyk::DirectGeo& g, hyk::Rec<H>* regions, hipStream_t s) {
  switch (fk) {
    case hyk::FK_DICT8:
      launch_part1_direct<SD, T, H, LP, hyk::FK_DICT8>(d, sd, d0, nd, g, regions, s);
      break;
    case hyk::FK_DICT16:
      launch_part1_direct<SD, T, H, LP, hyk::FK_DICT16>(d, sd, d0, nd, g, regions, s);
      break;
    case hyk::FK_DICT32:
      launch_part1_direct<SD, T, H, LP, hyk::FK_DICT32>(d, sd, d0, nd, g, regions, s);
      break;
    default:
      launch_part1_direct<SD, T, H, LP, hyk::FK_ANY>(d, sd, d0, nd, g, regions, s);
      break;
  }
  HY_HIP(hipGetLastError());
  return HY_OK;
}

// The direct passes of one side into last_out (the final partitions); *bounds receives the partition bounds.
template <typename SD, typename T, typename H>
hy_status direct_side(const DirectPlan& d, DirectBufs<H>& o, uint32_t bits, uint32_t seed, const Common& c,
                      hipStream_t s, const hyk::RecOut<H, uint32_t>& last_out, uint32_t** bounds) {
  const SidePlan& p = d.plan;
  const uint32_t n_spans = static_cast<uint32_t>(d.n_spans);
  const uint32_t nc = static_cast<uint32_t>(p.chunks.size());
  const hyk::Side sd = make_side(p, o.b, seed, false, p.ref_base, nullptr, 0, false, nullptr, 0);
  HY_HIP(hipMemsetAsync(o.overflow, 0, 16, s));
  hipLaunchKernelGGL(hyk::fill_tile_owner, dim3(grid_for(nc, 256)), dim3(256), 0, s, o.b.tile_begin, nc, o.b.tile_owner);
  HY_HIP(hipGetLastError());
  const int fk = filter_kind(p);
  {
    KTimer kt_((std::string("span_match_count.") + SD::name).c_str(), s, p.n_rows);
    auto count = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3(n_spans), dim3(hyk::PART_THREADS), 0, s, sd, d.nd0, o.span_cnt, o.span_cap,
                         o.cap_words);
    };
    if (fk == hyk::FK_DICT8)
      count(hyk::span_match_count<hyk::FK_DICT8>);
    else if (fk == hyk::FK_DICT16)
      count(hyk::span_match_count<hyk::FK_DICT16>);
    else if (fk == hyk::FK_DICT32)
      count(hyk::span_match_count<hyk::FK_DICT32>);
    else
      count(hyk::span_match_count<hyk::FK_ANY>);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  hy_status st = run_scan(o.span_cnt, o.span_scan, n_spans, c, s, o.totals + 0);
  if (st != HY_OK) return st;
  st = run_scan(o.cap_words, o.rbase32, n_spans, c, s, o.totals + 1);
  if (st != HY_OK) return st;
  hipLaunchKernelGGL(hyk::widen_u32, dim3(grid_for(n_spans, 256)), dim3(256), 0, s, o.rbase32, n_spans, o.span_rbase);
  HY_HIP(hipGetLastError());
  if (p.scan_chunk_begin) {
    hipLaunchKernelGGL(hyk::direct_chunk_begin, dim3(grid_for(nc + 1, 256)), dim3(256), 0, s, o.span_scan, n_spans,
                       o.b.tile_begin, nc, o.totals + 0, p.scan_chunk_begin);
    HY_HIP(hipGetLastError());
  }
  const hyk::DirectGeo g{o.span_rbase, o.span_cap, o.span_scan, o.counts, o.overflow, n_spans};
  const hyk::Digit d0{full_mask(bits), bits - (31 - __builtin_clz(d.nd0)), d.nd0 - 1u, seed, g_key_hash, rank_ballot()};
  // (HY_DIRECT_NOBYTES: an experiment that skips the digit bytes - the second pass's histogram is then wrong)
  static const bool no_bytes = std::getenv("HY_DIRECT_NOBYTES") != nullptr;
  const hyk::NextDigit nd{no_bytes ? nullptr : o.dig, 0u, d.nd1 - 1u};
  {
    KTimer kt_((std::string("part1_direct.") + SD::name).c_str(), s, p.n_rows);
    st = load_path(p) == hyk::LP_VALUE ? part1_direct_lp<SD, T, H, hyk::LP_VALUE>(d, fk, sd, d0, nd, g, o.regions, s)
                                       : part1_direct_lp<SD, T, H, hyk::LP_ANY>(d, fk, sd, d0, nd, g, o.regions, s);
    kt_.done();
    if (st != HY_OK) return st;
  }
  const hyk::GroupGeo gg{o.span_rbase, o.span_cap, o.counts, n_spans, d.groups, d.per};
  const dim3 g2(d.nd0 * d.groups);
  {
    KTimer kt_((std::string("part2g_hist.") + SD::name).c_str(), s, p.n_rows);
    hipLaunchKernelGGL(hyk::part2g_hist<SD>, g2, dim3(hyk::PART_THREADS), 0, s, gg, d.nd1, o.dig, o.hist);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  st = run_scan(o.hist, o.off, uint64_t(d.nd0) * d.nd1 * d.groups, c, s, o.totals + 2);
  if (st != HY_OK) return st;
  const hyk::Digit d1{full_mask(bits), 0u, d.nd1 - 1u, seed, g_key_hash, rank_ballot()};
  {
    KTimer kt_((std::string("part2g_scatter.") + SD::name).c_str(), s, p.n_rows);
    hipLaunchKernelGGL((hyk::part2g_scatter<SD, H, uint32_t>), g2, dim3(hyk::PART_THREADS), 0, s, gg, d1, d.nd1,
                       o.regions, o.off, last_out);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  const uint32_t n_parts = d.nd0 * d.nd1;
  hipLaunchKernelGGL(hyk::group_bounds, dim3(grid_for(n_parts + 1, 256)), dim3(256), 0, s, o.off, n_parts, d.groups,
                     o.totals + 2, o.bounds);
  HY_HIP(hipGetLastError());
  *bounds = o.bounds;
  return HY_OK;
}

// A join whose direct pass overflowed a region reran on the classic passes (read by prepared plans, which then keep
// the classic passes: their workspace holds the classic carve's descriptors from that execution on).
inline bool& direct_fell_back() {
  static thread_local bool v = false;
  return v;
}

// Pass-0 spans of one tile each (part1_onepass handles one tile per workgroup).
inline SidePlan one_tile_spans(const SidePlan& p) {
  SidePlan q = p;
  plan_spans(q, 1);
  return q;
}

// Workspace of a single-GPU join: enough for the single-pass path (when it applies) and for its fallback.
// The build side's passes on a second stream, concurrent with the probe side's (they share nothing until the
// partition join): the small build-side kernels and the probe side's scans leave HBM bandwidth idle that the other
// side's streaming passes then use. One side stream and a fork / join event pair per thread and device, created on
// first use (a stream being captured into a hipGraph forks into it by the event, as HIP capture allows).
// HY_JOIN_OVERLAP=0 runs both sides on the caller's stream (A/B).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  int device = -1;
};
inline bool overlap_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("HY_JOIN_OVERLAP");
    return !(e && std::strtol(e, nullptr, 10) == 0);
  }();
  return v;
}
inline SideStream* side_stream() {
  static thread_local SideStream ss[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SideStream& x = ss[dev];
  if (!x.s) {
    if (hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x.join, hipEventDisableTiming) != hipSuccess)
      return nullptr;
    x.device = dev;
  }
  return &x;
}

// Workspace of a join whose probe side takes the direct passes (join_typed's carve with direct set).
template <typename H>
size_t direct_join_bytes(const SidePlan& bp, const DirectPlan& dpl, uint32_t bits) {
  const auto w = digit_plan(bits, 0);
  const bool db = w.size() > 1 && digit_bytes_enabled();
  constexpr bool i32 = std::is_same_v<H, int32_t>;
  const uint32_t kb = block_count(bp, sizeof(H), w.size(), i32);
  Carver cv{nullptr, 0};
  SideBufs<H> a;
  DirectBufs<H> o;
  carve_side<H, uint32_t>(cv, sizes_of(bp, db, kb), bits, w, 1, true, a);
  carve_direct<H>(cv, dpl, bits, o);
  uint64_t ha, t;
  pass_sizes(sizes_of(bp, db, kb), w, 1, &ha, &t);
  Common c, cb;
  const uint64_t fb_scan = filter_buckets(bloom_words(bp.n_rows, dpl.plan.n_rows), bp.n_rows).scan_len;
  carve_common(cv, std::max({ha, uint64_t(direct_scan_words<H>(dpl)), (uint64_t(1) << bits) + 1, fb_scan}), bits, &c);
  carve_common(cv, std::max({ha, (uint64_t(1) << bits) + 1}), bits, &cb);
  cv.take<uint32_t>(prefilter_words(bloom_words(bp.n_rows, dpl.plan.n_rows), bp.n_rows));
  return cv.used + 256;
}

template <typename H>
size_t join_bytes(const SidePlan& bp, const SidePlan& pp, uint32_t bits) {
  size_t n = classic_join_bytes<H>(bp, pp, bits);
  if constexpr (std::is_integral_v<H>) {
    const DirectPlan dpl = direct_plan<H>(pp, bits, false, false);
    if (dpl.ok) n = std::max(n, direct_join_bytes<H>(bp, dpl, bits));
  }
  const auto w = digit_plan(bits, 0);
  const SidePlan b1 = one_tile_spans(bp), p1 = one_tile_spans(pp);
  if (onepass_ok(b1, w) && onepass_ok(p1, w)) n = std::max(n, onepass_bytes<H>(b1, p1, bits));
  return n;
}

// The classic passes, or (allow_direct) the direct passes for the probe side where they apply; *direct_overflow
// (eager executions) receives whether a direct region overflowed - the output is then invalid.
template <typename TB, typename TP, typename H>
hy_status join_typed_passes(const SidePlan& bp_in, const SidePlan& pp_in, const hy_join_params* prm,
                            hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,
                            uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,
                            void* workspace, size_t workspace_bytes, hipStream_t s, bool allow_direct,
                            bool* direct_overflow) {
  const uint32_t bits = prm->radix_bits;
  const bool keep_nulls = prm->mode == HY_JOIN_LEFT || prm->mode == HY_JOIN_RIGHT;
  const uint64_t bloom_n = bloom_words(bp_in.n_rows, pp_in.n_rows);
  const bool use_bloom = bloom_n && (prm->mode == HY_JOIN_INNER || prm->mode == HY_JOIN_SEMI);
  DirectPlan dpl;
  if constexpr (std::is_same_v<TP, H> && std::is_integral_v<H>)
    if (allow_direct) dpl = direct_plan<H>(pp_in, bits, keep_nulls, use_bloom);
  const bool direct = dpl.ok;
  const SidePlan& bp = bp_in;
  const SidePlan& pp = direct ? dpl.plan : pp_in;
  if (workspace_bytes < (direct ? direct_join_bytes<H>(bp, dpl, bits) : classic_join_bytes<H>(bp, pp, bits)))
    return fail(HY_ERR_WORKSPACE, "join workspace too small");
  const auto w = digit_plan(bits, 0);
  const bool db = w.size() > 1 && digit_bytes_enabled();
  constexpr bool i32 = std::is_same_v<H, int32_t>;
  const uint32_t blocks[2] = {block_count(bp, sizeof(H), w.size(), i32),
                              direct ? 0u : block_count(pp, sizeof(H), w.size(), i32)};
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  SideBufs<H> bb, pb;
  DirectBufs<H> dbuf{};
  carve_side<H, uint32_t>(cv, sizes_of(bp, db, blocks[0]), bits, w, 1, true, bb);
  if (direct) {
    carve_direct<H>(cv, dpl, bits, dbuf);
    pb = dbuf.b;
  } else {
    carve_side<H, uint32_t>(cv, sizes_of(pp, db, blocks[1]), bits, w, 1, true, pb);
  }
  uint64_t ha, hb2, t;
  pass_sizes(sizes_of(bp, db, blocks[0]), w, 1, &ha, &t);
  if (direct)
    hb2 = direct_scan_words<H>(dpl);
  else
    pass_sizes(sizes_of(pp, db, blocks[1]), w, 1, &hb2, &t);
  Common c{}, cb{};  // c: the probe side and the partition join; cb: the build side (it may run concurrently)
  const FilterBuckets fbk = filter_buckets(bloom_n, bp.n_rows);
  carve_common(cv, std::max({ha, hb2, (uint64_t(1) << bits) + 1, fbk.scan_len}), bits, &c);
  carve_common(cv, std::max({ha, (uint64_t(1) << bits) + 1}), bits, &cb);
  uint32_t* filter_area = cv.take<uint32_t>(prefilter_words(bloom_n, bp.n_rows));
  auto* filter_hdr = reinterpret_cast<hyk::FilterHdr*>(filter_area);
  uint32_t* bloom = filter_area + 16;
  // the bucketed build's scratch after the filter words (prefilter_words)
  uint32_t* fb_hist = bloom_n ? bloom + ((std::max(bloom_n, range_bitmap_words(bp.n_rows)) + 3) & ~uint64_t(3)) : nullptr;
  uint32_t* fb_off = fb_hist ? fb_hist + fbk.scan_len : nullptr;
  uint32_t* fb_items = fb_off ? fb_off + fbk.scan_len : nullptr;
  uint64_t* fb_count = fb_items ? reinterpret_cast<uint64_t*>(fb_items + ((bp.n_rows + 1) & ~uint64_t(1))) : nullptr;
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "join workspace too small");
  if (upload_side(bp, bb, s) || upload_side(pp, pb, s)) return HY_ERR_DEVICE;
  // the build side on the side stream unless the probe side needs its Bloom filter first
  // (not while per-kernel timing is on: concurrent kernels' event intervals would overlap and each read slower)
  bool timing = false;
  {
    std::lock_guard<std::mutex> lock(g_kt_mutex);
    timing = g_kt_enabled;
  }
  SideStream* ss = (!use_bloom && !timing && overlap_enabled()) ? side_stream() : nullptr;
  const hipStream_t sb = ss ? ss->s : s;
  // Every return after the fork joins the side stream back into s: an error return that left it forked let the build
  // side's kernels run on past the call, unordered with the caller's stream - which then reuses the workspace (the
  // operators' per-thread block cache relies on stream order), and a capture ended unjoined.
  struct JoinBack {
    SideStream* ss;
    hipStream_t sb, s;
    bool armed = false;
    hipError_t join() {
      if (!armed) return hipSuccess;
      armed = false;
      hipError_t e = hipEventRecord(ss->join, sb);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, ss->join, 0);
      return e;
    }
    ~JoinBack() {
      if (armed && join() != hipSuccess) (void)hipGetLastError();
    }
  } join_back{ss, sb, s};
  if (ss) {
    HY_HIP(hipEventRecord(ss->fork, s));
    HY_HIP(hipStreamWaitEvent(sb, ss->fork, 0));
    join_back.armed = true;
  }

  // int32 keys (no string ids) with b >= 16 radix bits: the last record pass keeps 16 hash bits instead of the key
  // (hyk::HashSrc), 6-byte records for the partition join; a prefilter is then keyed by hash and set by that pass
  const bool soa = hash_records_enabled() && std::is_same_v<H, int32_t> && g_key_hash == nullptr && w.size() >= 2 &&
                   bits >= 16 && bp.n_rows >= 16 && pp.n_rows >= 16;  // (>= 16: room for HashSrc's group reads)
  // a record join with integer keys: the prefilter is a key-range bitmap when the build keys' range fits
  const bool range_filter = use_bloom && !soa && std::is_integral_v<H>;
  hyk::RecOut<H, uint32_t> soa_outs[2];
  const hyk::RecOut<H, uint32_t> pass0_outs[2] = {aos_out<H, uint32_t>(bb.recA), aos_out<H, uint32_t>(pb.recA)};
  if (soa) {
    if (use_bloom) HY_HIP(hipMemsetAsync(bloom, 0, 4 * bloom_n, s));
    // the record passes after pass 0 ping-pong recA -> recB -> recA ...: the last one writes recB after an odd count
    const bool last_in_b = (w.size() - 1) % 2 == 1;
    soa_outs[0] = soa_out<H, uint32_t>(last_in_b ? bb.recB : bb.recA, bp.n_rows, bits, use_bloom ? bloom : nullptr,
                                       bloom_n);
    soa_outs[1] = soa_out<H, uint32_t>(direct ? static_cast<void*>(dbuf.out) : (last_in_b ? pb.recB : pb.recA),
                                       pp.n_rows, bits);
  }

  hyk::Rec<H>* recs[2] = {nullptr, nullptr};
  uint32_t* bounds[2] = {nullptr, nullptr};
  for (int side = 0; side < 2; ++side) {
    const SidePlan& p = side == 0 ? bp : pp;
    SideBufs<H>& b = side == 0 ? bb : pb;
    const char* tag = side == 0 ? "build" : "probe";
    const Common& cs = side == 0 ? cb : c;
    const hipStream_t st_s = side == 0 ? sb : s;
    const hyk::NextDigit nd = next_digit(w, 0, bits, b.digA);
    if (side == 1 && direct) {  // the probe side's direct passes (join_direct.hip)
      if constexpr (std::is_same_v<TP, H> && std::is_integral_v<H>) {
        const hyk::RecOut<H, uint32_t> lo = soa ? soa_outs[1] : aos_out<H, uint32_t>(dbuf.out);
        hy_status st = direct_side<hyk::OnProbe, TP, H>(dpl, dbuf, bits, prm->seed, c, s, lo, &bounds[1]);
        if (st != HY_OK) return st;
        recs[1] = dbuf.out;
      }
    } else if (blocks[side]) {  // pass 0 in row blocks and the record passes after it
      const bool pf = side == 1 && use_bloom;
      const hyk::Side sd = make_side(p, b, prm->seed, side == 1 && keep_nulls, p.ref_base, pf ? bloom : nullptr, bloom_n,
                                     soa, pf && range_filter ? filter_hdr : nullptr,
                                     pf && range_filter ? range_bitmap_words(bp.n_rows) : 0);
      const hyk::RecOut<H, uint32_t>* lo = soa ? &soa_outs[side] : nullptr;
      hy_status st = HY_ERR_UNSUPPORTED;
      if constexpr (i32)
        st = side == 0 ? blocked_side<hyk::OnBuild, TB, H>(p, b, bits, w, blocks[0], sd, cs, st_s, &recs[0], &bounds[0],
                                                           lo)
                       : blocked_side<hyk::OnProbe, TP, H>(p, b, bits, w, blocks[1], sd, cs, st_s, &recs[1], &bounds[1],
                                                           lo);
      if (st != HY_OK) return st;
    } else {
    hy_status st = side == 0
                       ? pass0_side<hyk::OnBuild, TB, H, uint32_t>(p, b, bits, w.empty() ? 0 : w[0], prm->seed, false,
                                                     p.ref_base, nd, cs, st_s, pass0_outs[0])
                       : pass0_side<hyk::OnProbe, TP, H, uint32_t>(p, b, bits, w.empty() ? 0 : w[0], prm->seed, keep_nulls,
                                                     p.ref_base, nd, cs, st_s, pass0_outs[1], use_bloom ? bloom : nullptr,
                                                     bloom_n, soa, range_filter ? filter_hdr : nullptr,
                                                     range_filter ? range_bitmap_words(bp.n_rows) : 0);
    if (st != HY_OK) return st;
    st = by_side(tag, [&](auto sdt) {
      return local_passes<decltype(sdt), H, uint32_t>(b, w, 1, bits, prm->seed, b.recA, b.recB, nd.bytes, b.digB,
                                                      b.segA, b.segB, w.empty() ? 1 : (1ull << w[0]), b.total,
                                                      p.n_rows, cs, st_s, &recs[side], &bounds[side],
                                                      soa ? &soa_outs[side] : nullptr);
    });
    if (st != HY_OK) return st;
    }
    if (side == 0 && use_bloom && !soa) {  // the probe side's prefilter over the build side's keys (its records)
      const uint64_t rw = range_filter ? range_bitmap_words(bp.n_rows) : 0;
      HY_HIP(hipMemsetAsync(filter_hdr, 0, sizeof(hyk::FilterHdr), s));
      KTimer kt_("prefilter_build", s, p.n_rows);
      if (range_filter)
        hipLaunchKernelGGL(hyk::filter_range<H>, dim3(static_cast<uint32_t>(std::min<uint64_t>(grid_for(p.n_rows, 256), 1024))),
                           dim3(256), 0, s, recs[0], b.total, filter_hdr);
      const uint32_t bmask = static_cast<uint32_t>(bloom_n - 1);
      if (fbk.blocks) {  // per LDS region: count, scan, scatter, set (the set also writes the words no key sets)
        const dim3 fbt(hyk::FB_THREADS);
        hipLaunchKernelGGL(hyk::filter_bucket_count<H>, dim3(fbk.blocks), fbt, 0, s, recs[0], b.total, filter_hdr, rw,
                           bloom_n, bmask, fb_hist, fb_count);
        HY_HIP(hipGetLastError());
        if (hy_status st = run_scan(fb_hist, fb_off, fbk.scan_len, c, s, fb_count + 1, fb_count, fbk.blocks); st != HY_OK)
          return st;
        hipLaunchKernelGGL(hyk::filter_bucket_scatter<H>, dim3(fbk.blocks), fbt, 0, s, recs[0], b.total, filter_hdr, rw,
                           bloom_n, bmask, fb_off, fb_items);
        HY_HIP(hipGetLastError());
        hipLaunchKernelGGL(hyk::filter_bucket_set<H>, dim3(fbk.bins), fbt, static_cast<size_t>(4u << fbk.shift), s,
                           filter_hdr, rw, bloom_n, fb_off, fb_count + 1, fbk.blocks, fb_items, bloom);
      } else {
        hipLaunchKernelGGL(hyk::filter_clear<H>, dim3(static_cast<uint32_t>(std::min<uint64_t>(grid_for(std::max(bloom_n, rw) / 4, 256), 4096))),
                           dim3(256), 0, s, filter_hdr, bloom, rw, bloom_n);
        hipLaunchKernelGGL(hyk::filter_set<H>, dim3(static_cast<uint32_t>(std::min<uint64_t>(grid_for(p.n_rows, 256), 4096))),
                           dim3(256), 0, s, recs[0], b.total, filter_hdr, bloom, rw, bmask);
      }
      kt_.done();
      HY_HIP(hipGetLastError());
    }
  }
  HY_HIP(join_back.join());  // the partition join waits for the build side
  // filtered sides emit RowIDs of their data table (the scan's PosLists dereferenced, write_output_columns)
  const hyk::RowMap bmap = bp.fuse ? make_map(bb.ref_row_begin, bp.ref_row_begin) : make_map(bb.row_begin, bp.row_begin);
  const hyk::RowMap pmap = pp.fuse ? make_map(pb.ref_row_begin, pp.ref_row_begin) : make_map(pb.row_begin, pp.row_begin);
  const bool probe_exact = !pp.filtered && !use_bloom;  // (a Bloom prefilter drops probe rows too)
  hy_status st = HY_OK;
  if (soa) {
    auto run_hash = [&](auto tag) {
      using HS = decltype(tag);
      return run_join_partitions<HS, uint32_t>(bounds[0], bounds[1], 1u << bits, HS{soa_outs[0].hk, soa_outs[0].pay},
                                               HS{soa_outs[1].hk, soa_outs[1].pay}, bmap, pmap, prm->mode, out_build,
                                               out_probe, out_capacity, partition_begin, partition_counts, result, c,
                                               s, bp.n_rows + pp.n_rows, pp.n_rows, probe_exact);
    };
    // records per lane and load (A/B, HY_HASH_GROUP): 1 (default) or 4
    st = knobs().hash_group == 4 ? run_hash(hyk::HashSrc<uint32_t, 4>{}) : run_hash(hyk::HashSrc<uint32_t, 1>{});
  } else {
    st = run_join_partitions<hyk::RecSrc<H, uint32_t>, uint32_t>(
        bounds[0], bounds[1], 1u << bits, hyk::RecSrc<H, uint32_t>{recs[0]}, hyk::RecSrc<H, uint32_t>{recs[1]}, bmap,
        pmap, prm->mode, out_build, out_probe, out_capacity, partition_begin, partition_counts, result, c, s,
        bp.n_rows + pp.n_rows, pp.n_rows, probe_exact);
  }
  if (direct) {
    if (capture_state().capturing) {  // (a prepared plan's replay reads the flag after the graph: finish_replay)
      capture_state().direct_overflow = dbuf.overflow;
    } else if (direct_overflow) {
      uint32_t f = 0;
      HY_HIP(hipMemcpyAsync(&f, dbuf.overflow, 4, hipMemcpyDeviceToHost, s));
      HY_HIP(hipStreamSynchronize(s));
      *direct_overflow = f != 0;
    }
  }
  return st;
}

template <typename TB, typename TP, typename H>
hy_status join_typed_any(const SidePlan& bp_in, const SidePlan& pp_in, const hy_join_params* prm, hy_row_id* out_build,
                         hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                         uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                         hipStream_t s) {
  const uint32_t bits = prm->radix_bits;
  {
    const auto w = digit_plan(bits, 0);
    const SidePlan b1 = one_tile_spans(bp_in), p1 = one_tile_spans(pp_in);
    if (onepass_ok(b1, w) && onepass_ok(p1, w) && workspace_bytes >= onepass_bytes<H>(b1, p1, bits)) {
      uint32_t overflow = 0;
      const hy_status st = join_typed_onepass<TB, TP, H>(b1, p1, prm, out_build, out_probe, out_capacity,
                                                         partition_begin, partition_counts, result, workspace,
                                                         workspace_bytes, s, &overflow);
      if (overflow == 0) return st;
      // a gapped region overflowed (or a look-back timed out): the two-read path below recomputes everything
    }
  }
  bool overflow = false;
  const hy_status st = join_typed_passes<TB, TP, H>(bp_in, pp_in, prm, out_build, out_probe, out_capacity,
                                                    partition_begin, partition_counts, result, workspace,
                                                    workspace_bytes, s, true, &overflow);
  if (!overflow || (st != HY_OK && st != HY_ERR_CAPACITY)) return st;
  // a direct region overflowed: the classic passes recompute everything (the workspace is carved differently, so
  // both sides' descriptors are staged again)
  direct_fell_back() = true;
  SidePlan b2 = bp_in, p2 = pp_in;
  b2.device_ready = p2.device_ready = false;
  return join_typed_passes<TB, TP, H>(b2, p2, prm, out_build, out_probe, out_capacity, partition_begin,
                                      partition_counts, result, workspace, workspace_bytes, s, false, nullptr);
}

// The join, then the fused scans' RowIDs (hy_join_filter.out_row_ids) of every side whose pass 0 wrote offsets.
template <typename TB, typename TP, typename H>
hy_status join_typed(const SidePlan& bp, const SidePlan& pp, const hy_join_params* prm, hy_row_id* out_build,
                     hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                     uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                     hipStream_t s) {
  scan_rows_written().clear();
  const hy_status st = join_typed_any<TB, TP, H>(bp, pp, prm, out_build, out_probe, out_capacity, partition_begin,
                                                 partition_counts, result, workspace, workspace_bytes, s);
  if (st != HY_OK && st != HY_ERR_CAPACITY) return st;
  for (const SidePlan* p : {&bp, &pp}) {
    if (!p->filtered || !p->scan_rows) continue;
    const auto& done = scan_rows_written();
    if (std::find(done.begin(), done.end(), p->scan_rows) != done.end()) continue;
    const hy_status e = hy_expand_chunk_row_ids(p->scan_out, p->scan_chunk_begin, nullptr,
                                                static_cast<uint32_t>(p->chunks.size()), p->scan_rows, s);
    if (e != HY_OK) return e;
  }
  return st;
}

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

// Only hashed types reachable through JoinHashTraits (hash_traits.hpp:9-42) are instantiated.
template <typename T, typename H>
constexpr bool reachable() {
  return (sizeof(H) >= sizeof(T) || std::is_floating_point_v<H>) &&
         !(std::is_floating_point_v<T> && !std::is_floating_point_v<H>);
}

// ---------------------------------------------------------------------------------------------------------------
// Distributed JoinHash: exchange records are Rec<H, hy_row_id> (16 bytes: key, global RowID).
// ---------------------------------------------------------------------------------------------------------------
inline uint32_t ceil_log2(uint32_t n) {
  uint32_t b = 0;
  while ((1u << b) < n) ++b;
  return b;
}

// Longest exclusive scan of the exchange partition's pass 0: one histogram row per first digit over the side's spans,
// plus the fused TableScan's match row when the side is filtered (part1_compact writes it, join.hip).
inline uint64_t exchange_scan_words(const SidePlan& p, const std::vector<uint32_t>& w) {
  const uint64_t rows = (1ull << w[0]) + (p.filtered ? 1 : 0);
  return std::max<uint64_t>(rows * std::max<uint64_t>(1, p.n_tiles1), 2);
}

template <typename H, typename P = hy_row_id>
size_t exchange_partition_bytes(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w) {
  Carver cv{nullptr, 0};
  SideBufs<H, P> b;
  SideSizes z = sizes_of(p, false);
  carve_side<H, P>(cv, z, bits, std::vector<uint32_t>(w.begin(), w.begin() + 1), 1, false, b);
  Common c;
  carve_common(cv, exchange_scan_words(p, w), bits, &c);
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

inline RecvPlan recv_plan(const uint64_t* counts, uint32_t n_senders, uint32_t nb, uint32_t digits) {
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
template <typename H, typename P = hy_row_id>
struct RecvBufs {
  SideBufs<H, P> b;
  uint32_t *seg_begin, *seg_end, *seg_stride, *seg_toff, *group_tiles, *group_out, *owner;
  uint64_t *seg_tile_begin, *seg_hbase, *group_hbase;
};

template <typename H, typename P = hy_row_id>
void carve_recv(Carver& cv, const RecvPlan& r, uint32_t bits, const std::vector<uint32_t>& w, uint32_t nb,
                uint32_t n_senders, RecvBufs<H, P>& rb) {
  SideSizes z;
  z.rows = r.rows;
  std::vector<uint32_t> tail(w.begin() + 1, w.end());
  if (tail.empty()) tail.push_back(0);
  carve_side<H, P>(cv, z, bits, tail, uint64_t(nb) * n_senders, true, rb.b);
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

template <typename H, typename P = hy_row_id>
hy_status recv_side(const char* tag, const RecvPlan& r, RecvBufs<H, P>& rb, const std::vector<uint32_t>& w,
                    uint32_t bits, uint32_t nb, uint32_t n_senders, uint32_t seed, const hyk::Rec<H, P>* in,
                    const Common& c, hipStream_t s, hyk::Rec<H, P>** recs, uint32_t** bounds) {
  auto up = [&](auto* dst, const auto& v) -> hy_status {
    if (!v.empty()) HY_STAGE(dst, v.data(), sizeof(v[0]) * v.size(), s);
    return HY_OK;
  };
  if (up(rb.seg_begin, r.seg_begin) || up(rb.seg_end, r.seg_end) || up(rb.seg_stride, r.seg_stride) ||
      up(rb.seg_toff, r.seg_toff) || up(rb.seg_tile_begin, r.seg_tile_begin) || up(rb.seg_hbase, r.seg_hbase) ||
      up(rb.group_hbase, r.group_hbase) || up(rb.group_tiles, r.group_tiles) || up(rb.group_out, r.group_out))
    return HY_ERR_DEVICE;
  HY_STAGE(rb.b.total, &r.rows, 8, s);
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
  return by_side(tag, [&](auto sdt) {
    using SD = decltype(sdt);
    hy_status st = record_pass<SD, H, P>(rb.b, sg, gr, nb, r.tiles, bits, shift, w1, seed, in, nullptr,
                                         hyk::NextDigit{nullptr, 0, 0}, aos_out<H, P>(rb.b.recA), rb.b.total,
                                         rb.b.segA, c, s, r.rows);
    if (st != HY_OK) return st;
    return local_passes<SD, H, P>(rb.b, w, 2, bits, seed, rb.b.recA, rb.b.recB, nullptr, nullptr, rb.b.segA,
                                  rb.b.segB, uint64_t(nb) << w1, rb.b.total, r.rows, c, s, recs, bounds);
  });
}

// Global chunk layouts of the two tables (row-index exchange records): device row_begin arrays of the RowMaps.
struct Layouts {
  std::vector<uint64_t> build_rows, probe_rows;  // row_begin (n_chunks + 1 each); empty for RowID records
};

inline std::vector<uint64_t> layout_rows(const uint32_t* sizes, uint32_t n) {
  std::vector<uint64_t> r(n + 1, 0);
  for (uint32_t i = 0; i < n; ++i) r[i + 1] = r[i] + sizes[i];
  return r;
}

template <typename H, typename P = hy_row_id>
size_t exchange_join_bytes(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits, const std::vector<uint32_t>& w,
                           uint32_t nb, uint32_t n_senders, const Layouts& lay = Layouts{}) {
  Carver cv{nullptr, 0};
  RecvBufs<H, P> a, b;
  carve_recv<H, P>(cv, rbp, bits, w, nb, n_senders, a);
  carve_recv<H, P>(cv, rpp, bits, w, nb, n_senders, b);
  cv.take<uint64_t>(lay.build_rows.size() + 1);
  cv.take<uint64_t>(lay.probe_rows.size() + 1);
  Common c;
  const uint64_t max_scan = std::max({rbp.hist_words * 2, rpp.hist_words * 2, (uint64_t(1) << bits) + 1,
                                      (rbp.rows + rpp.rows) / span2() * 256 + uint64_t(nb) * n_senders * 256});
  carve_common(cv, max_scan, bits, &c);
  return cv.used + 256;
}

template <typename H, typename P = hy_row_id>
hy_status exchange_partition_for_hashed(const SidePlan& p, int32_t value_type, const hy_join_params* params,
                                        int32_t keep_nulls, const std::vector<uint32_t>& w, void* out_records,
                                        uint64_t* bucket_counts, void* workspace, size_t workspace_bytes,
                                        hipStream_t s) {
  const uint32_t bits = params->radix_bits;
  const uint32_t T = 1u << w[0];
  return dispatch_type(value_type, [&](auto ttag) -> hy_status {
    using T_ = decltype(ttag);
    if constexpr (reachable<T_, H>()) {
      if (workspace_bytes < exchange_partition_bytes<H, P>(p, bits, w)) return fail(HY_ERR_WORKSPACE, "workspace");
      Carver cv{static_cast<char*>(workspace), workspace_bytes};
      SideBufs<H, P> b;
      carve_side<H, P>(cv, sizes_of(p, false), bits, std::vector<uint32_t>(w.begin(), w.begin() + 1), 1, false, b);
      Common c{};
      carve_common(cv, exchange_scan_words(p, w), bits, &c);
      if (!cv.ok) return fail(HY_ERR_WORKSPACE, "workspace");
      if (upload_side(p, b, s)) return HY_ERR_DEVICE;
      hy_status st2 = pass0_side<hyk::OnExchange, T_, H, P>(p, b, bits, w[0], params->seed, keep_nulls != 0, p.ref_base,
                                           hyk::NextDigit{nullptr, 0, 0}, c, s,
                                           aos_out<H, P>(static_cast<hyk::Rec<H, P>*>(out_records)));
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
}

template <typename H, typename P = hy_row_id>
hy_status exchange_join_for_hashed(const void* build_records, const void* probe_records, const RecvPlan& rbp,
                                   const RecvPlan& rpp, uint32_t n_senders, uint32_t n_buckets,
                                   const std::vector<uint32_t>& w, const hy_join_params* params, hy_row_id* out_build,
                                   hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                                   uint32_t* partition_counts, hy_join_result* result, void* workspace,
                                   size_t workspace_bytes, hipStream_t s, const Layouts& lay = Layouts{}) {
  const uint32_t bits = params->radix_bits;
  if (workspace_bytes < exchange_join_bytes<H, P>(rbp, rpp, bits, w, n_buckets, n_senders, lay))
    return fail(HY_ERR_WORKSPACE, "exchange join workspace too small");
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  RecvBufs<H, P> rb, rp;
  carve_recv<H, P>(cv, rbp, bits, w, n_buckets, n_senders, rb);
  carve_recv<H, P>(cv, rpp, bits, w, n_buckets, n_senders, rp);
  uint64_t* b_rows = cv.take<uint64_t>(lay.build_rows.size() + 1);
  uint64_t* p_rows = cv.take<uint64_t>(lay.probe_rows.size() + 1);
  Common c{};
  const uint64_t max_scan = std::max({rbp.hist_words * 2, rpp.hist_words * 2, (uint64_t(1) << bits) + 1,
                                      (rbp.rows + rpp.rows) / span2() * 256 + uint64_t(n_buckets) * n_senders * 256});
  carve_common(cv, max_scan, bits, &c);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "exchange join workspace too small");
  using R = hyk::Rec<H, P>;
  R* recs[2] = {nullptr, nullptr};
  uint32_t* bounds[2] = {nullptr, nullptr};
  hy_status st = recv_side<H, P>("build", rbp, rb, w, bits, n_buckets, n_senders, params->seed,
                                 static_cast<const R*>(build_records), c, s, &recs[0], &bounds[0]);
  if (st != HY_OK) return st;
  st = recv_side<H, P>("probe", rpp, rp, w, bits, n_buckets, n_senders, params->seed,
                       static_cast<const R*>(probe_records), c, s, &recs[1], &bounds[1]);
  if (st != HY_OK) return st;
  const uint32_t n_parts = n_buckets << (bits - w[0]);
  hyk::RowMap bmap{}, pmap{};
  if constexpr (std::is_same_v<P, uint32_t>) {  // global row indexes -> RowIDs of the global chunk layouts
    HY_STAGE(b_rows, lay.build_rows.data(), 8 * lay.build_rows.size(), s);
    HY_STAGE(p_rows, lay.probe_rows.data(), 8 * lay.probe_rows.size(), s);
    bmap = make_map(b_rows, lay.build_rows);
    pmap = make_map(p_rows, lay.probe_rows);
  }
  return run_join_partitions<hyk::RecSrc<H, P>, P>(bounds[0], bounds[1], n_parts, hyk::RecSrc<H, P>{recs[0]},
                                                   hyk::RecSrc<H, P>{recs[1]}, bmap, pmap, params->mode,
                                   out_build, out_probe, out_capacity, partition_begin, partition_counts, result, c, s,
                                   rbp.rows + rpp.rows, rpp.rows, true);
}

template <typename H>
hy_status join_for_hashed(const SidePlan& bp, const SidePlan& pp, int32_t build_type, int32_t probe_type,
                          const hy_join_params* params, hy_row_id* out_build, hy_row_id* out_probe,
                          uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,
                          hy_join_result* result, void* workspace, size_t workspace_bytes, hipStream_t s) {
  return dispatch_type(build_type, [&](auto btag) -> hy_status {
    using TB = decltype(btag);
    return dispatch_type(probe_type, [&](auto ptag) -> hy_status {
      using TP = decltype(ptag);
      if constexpr (reachable<TB, H>() && reachable<TP, H>()) {
        return join_typed<TB, TP, H>(bp, pp, params, out_build, out_probe, out_capacity, partition_begin,
                                     partition_counts, result, workspace, workspace_bytes, s);
      } else {
        return fail(HY_ERR_UNSUPPORTED, "hashed type not reachable from column types");
      }
    });
  });
}

// Per-hashed-type entry points (one translation unit each).
#define HYJ_DECLARE(SUFFIX, H)                                                                                      \
  hy_status join_##SUFFIX(const SidePlan& bp, const SidePlan& pp, int32_t build_type, int32_t probe_type,           \
                          const hy_join_params* params, hy_row_id* out_build, hy_row_id* out_probe,               \
                          uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,           \
                          hy_join_result* result, void* workspace, size_t workspace_bytes, hipStream_t s);    \
  size_t join_bytes_##SUFFIX(const SidePlan& bp, const SidePlan& pp, uint32_t bits);                               \
  size_t exchange_partition_bytes_##SUFFIX(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w);        \
  size_t exchange_join_bytes_##SUFFIX(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits,                      \
                                      const std::vector<uint32_t>& w, uint32_t nb, uint32_t n_senders);             \
  hy_status exchange_partition_##SUFFIX(const SidePlan& p, int32_t value_type, const hy_join_params* params,        \
                                        int32_t keep_nulls, const std::vector<uint32_t>& w, void* out_records,      \
                                        uint64_t* bucket_counts, void* workspace, size_t workspace_bytes,           \
                                        hipStream_t s);                                                             \
  hy_status exchange_join_##SUFFIX(const void* build_records, const void* probe_records, const RecvPlan& rbp,      \
                                   const RecvPlan& rpp, uint32_t n_senders, uint32_t n_buckets,                    \
                                   const std::vector<uint32_t>& w, const hy_join_params* params,                   \
                                   hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,              \
                                   uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,  \
                                   void* workspace, size_t workspace_bytes, hipStream_t s);                        \
  size_t exchange_partition_rows_bytes_##SUFFIX(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w);   \
  size_t exchange_join_rows_bytes_##SUFFIX(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits,                 \
                                           const std::vector<uint32_t>& w, uint32_t nb, uint32_t n_senders,         \
                                           const Layouts& lay);                                                     \
  hy_status exchange_partition_rows_##SUFFIX(const SidePlan& p, int32_t value_type, const hy_join_params* params,   \
                                             int32_t keep_nulls, const std::vector<uint32_t>& w, void* out_records, \
                                             uint64_t* bucket_counts, void* workspace, size_t workspace_bytes,      \
                                             hipStream_t s);                                                        \
  hy_status exchange_join_rows_##SUFFIX(const void* build_records, const void* probe_records, const RecvPlan& rbp, \
                                        const RecvPlan& rpp, uint32_t n_senders, uint32_t n_buckets,               \
                                        const std::vector<uint32_t>& w, const hy_join_params* params,              \
                                        hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,         \
                                        uint64_t* partition_begin, uint32_t* partition_counts,                     \
                                        hy_join_result* result, void* workspace, size_t workspace_bytes,           \
                                        hipStream_t s, const Layouts& lay);
HYJ_DECLARE(i32, int32_t)
HYJ_DECLARE(i64, int64_t)
HYJ_DECLARE(f32, float)
HYJ_DECLARE(f64, double)
#undef HYJ_DECLARE

#define HYJ_DEFINE(SUFFIX, H)                                                                                       \
  hy_status join_##SUFFIX(const SidePlan& bp, const SidePlan& pp, int32_t build_type, int32_t probe_type,           \
                          const hy_join_params* params, hy_row_id* out_build, hy_row_id* out_probe,               \
                          uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,           \
                          hy_join_result* result, void* workspace, size_t workspace_bytes, hipStream_t s) {       \
    return join_for_hashed<H>(bp, pp, build_type, probe_type, params, out_build, out_probe, out_capacity,         \
                              partition_begin, partition_counts, result, workspace, workspace_bytes, s);          \
  }                                                                                                                 \
  size_t join_bytes_##SUFFIX(const SidePlan& bp, const SidePlan& pp, uint32_t bits) {                               \
    return join_bytes<H>(bp, pp, bits);                                                                             \
  }                                                                                                                 \
  size_t exchange_partition_bytes_##SUFFIX(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w) {       \
    return exchange_partition_bytes<H>(p, bits, w);                                                                 \
  }                                                                                                                 \
  size_t exchange_join_bytes_##SUFFIX(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits,                      \
                                      const std::vector<uint32_t>& w, uint32_t nb, uint32_t n_senders) {            \
    return exchange_join_bytes<H>(rbp, rpp, bits, w, nb, n_senders);                                                \
  }                                                                                                                 \
  hy_status exchange_partition_##SUFFIX(const SidePlan& p, int32_t value_type, const hy_join_params* params,        \
                                        int32_t keep_nulls, const std::vector<uint32_t>& w, void* out_records,      \
                                        uint64_t* bucket_counts, void* workspace, size_t workspace_bytes,           \
                                        hipStream_t s) {                                                            \
    return exchange_partition_for_hashed<H>(p, value_type, params, keep_nulls, w, out_records, bucket_counts,       \
                                            workspace, workspace_bytes, s);                                         \
  }                                                                                                                 \
  hy_status exchange_join_##SUFFIX(const void* build_records, const void* probe_records, const RecvPlan& rbp,      \
                                   const RecvPlan& rpp, uint32_t n_senders, uint32_t n_buckets,                    \
                                   const std::vector<uint32_t>& w, const hy_join_params* params,                   \
                                   hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,              \
                                   uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,  \
                                   void* workspace, size_t workspace_bytes, hipStream_t s) {                        \
    return exchange_join_for_hashed<H>(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w, params,     \
                                       out_build, out_probe, out_capacity, partition_begin, partition_counts,      \
                                       result, workspace, workspace_bytes, s);                                      \
  }                                                                                                                 \
  size_t exchange_partition_rows_bytes_##SUFFIX(const SidePlan& p, uint32_t bits, const std::vector<uint32_t>& w) {  \
    return exchange_partition_bytes<H, uint32_t>(p, bits, w);                                                       \
  }                                                                                                                 \
  size_t exchange_join_rows_bytes_##SUFFIX(const RecvPlan& rbp, const RecvPlan& rpp, uint32_t bits,                 \
                                           const std::vector<uint32_t>& w, uint32_t nb, uint32_t n_senders,         \
                                           const Layouts& lay) {                                                    \
    return exchange_join_bytes<H, uint32_t>(rbp, rpp, bits, w, nb, n_senders, lay);                                 \
  }                                                                                                                 \
  hy_status exchange_partition_rows_##SUFFIX(const SidePlan& p, int32_t value_type, const hy_join_params* params,   \
                                             int32_t keep_nulls, const std::vector<uint32_t>& w, void* out_records, \
                                             uint64_t* bucket_counts, void* workspace, size_t workspace_bytes,      \
                                             hipStream_t s) {                                                       \
    return exchange_partition_for_hashed<H, uint32_t>(p, value_type, params, keep_nulls, w, out_records,            \
                                                      bucket_counts, workspace, workspace_bytes, s);                \
  }                                                                                                                 \
  hy_status exchange_join_rows_##SUFFIX(const void* build_records, const void* probe_records, const RecvPlan& rbp, \
                                        const RecvPlan& rpp, uint32_t n_senders, uint32_t n_buckets,               \
                                        const std::vector<uint32_t>& w, const hy_join_params* params,              \
                                        hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,         \
                                        uint64_t* partition_begin, uint32_t* partition_counts,                     \
                                        hy_join_result* result, void* workspace, size_t workspace_bytes,           \
                                        hipStream_t s, const Layouts& lay) {                                       \
    return exchange_join_for_hashed<H, uint32_t>(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w,   \
                                                 params, out_build, out_probe, out_capacity, partition_begin,      \
                                                 partition_counts, result, workspace, workspace_bytes, s, lay);    \
  }

}  // namespace hyj
