// agg_dense_stream: agg_dense_vec (aggregate_vec.hip) with its column loads taken off the critical path and its
// per-row work cut down - the TPC-H 1 shape (data input, TableScan fused as a dictionary id range, a few dictionary
// group codes, SUM / AVG over float columns and + - * chains of them). Reference: Projection::_on_execute
// (projection.cpp:39-87) materialising the SELECT list, then Aggregate (aggregate.cpp:133-249, 291-498) summing it;
// the fused predicate is SingleColumnTableScanImpl's dictionary rewrite (single_column_table_scan_impl.cpp:145-205).
//
// Round 3 measured agg_dense_vec latency-bound: each 256-row step issued its column loads and waited for them before
// any arithmetic (168 VGPRs, 3 waves per SIMD, waves stalled ~60 % of their cycles); prefetching the next step into
// registers spilled. Here:
//   * loads go straight to LDS (global_load_lds, no VGPR destination) one step ahead: a step reads its column bytes
//     and filter ids from the wave's stage, then issues the next step's loads into the same stage, then accumulates;
//     every LDS array is its own __shared__ object, so the compiler's wait before an LDS read covers only the
//     stage's DMA (the decoded values, decode tables and group table are read with the next step's loads in flight);
//   * a wave takes whole 4096-row tiles (16 steps of 256 rows, grid-stride over the tiles by wave): the tile's column
//     descriptors stay in registers for its steps, its dictionaries are read once into per-wave LDS decode tables
//     (group-by tables map a NULL id to the NULL code and are checked against the code domain once per tile);
//   * chains are FMA-form programs compiled by the host (StreamTerm: term = fma(x, a, b), then one uniform-branch
//     combine), decoded values are read once per step from LDS;
//   * group codes map to table entries through a per-wave LDS table, the rows of every entry are one-hot bits of
//     one word (counts by popcount, last rows by find-last-set);
//   * exactness per flush period as agg_dense_vec (the period's smallest exponent is its base, a wider spread than
//     LN_WINDOW discards the period and defers its steps): the largest magnitude by a float max3 (abs modifiers), the
//     smallest nonzero one by (bits << 1) - 1 and an integer min3; a NaN or infinity anywhere reaches every
//     accumulator of the lane (0 * inf) and is caught at the flush. Rows that take no part are never multiplied into
//     an entry; their values may widen the period's window (a discarded period is exact again in agg_dense_fused).
// Preconditions (host, plan_stream): agg_dense_vec's, plus: every DICT chunk of a loaded column has <= ST_DICT_MAX
// dictionary entries, the filter (if any) is a dictionary id range on every chunk, the stage layout fits, float sums
// are + - * chains, int32 sums are plain columns, group codes < 64.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int ST_WAVES = AGG_THREADS / WAVE;
constexpr int ST_STEPS = AGG_TILE / (WAVE * FQ_R);  // steps of a tile (16)
constexpr int ST_STAGE = 3072;                      // bytes of one step's column bytes + filter ids, per wave
constexpr int ST_DCOLS = 6;                         // dictionary-decoded loaded columns
constexpr int ST_VALS = 4;                          // loaded columns besides the group-by columns
constexpr int ST_DICT_MAX = 63;                     // dictionary entries (id 63 may then only be a NULL id)
constexpr int ST_PLIST = 64;                        // tiles recorded per period
constexpr int ST_CODES = 64;                        // group codes of the per-wave entry table
constexpr uint32_t ST_NO_SLOT = 0xFFFFFFFFu;

// A chain term: x = the loaded column's decoded value (int32 -> float with ST_CVT, 0 with ST_LIT), term = fma(x, a, b)
// (x, lit + x, lit - x, lit * x, x - lit, x * lit - one rounding each, as the reference's float functors), then
// running = combine(running, term).
enum : int32_t { ST_SET = 0, ST_ADD = 1, ST_SUB = 2, ST_RSUB = 3, ST_MUL = 4, ST_COMB = 7, ST_CVT = 8, ST_LIT = 16 };
enum : int32_t { ST_SUM_NONE = 0, ST_SUM_FLOAT = 1, ST_SUM_INT = 2 };
struct StreamTerm {
  float a, b;
  int32_t col;    // loaded column index (>= the group-by columns)
  int32_t flags;  // ST_SET..ST_MUL | ST_CVT | ST_LIT
};

// The plan of one launch (device memory, read through the constant address space).
struct StreamPlan {
  uint32_t col_off[LN_COLS];    // stage byte offset of loaded column li (256 rows x its widest chunk width)
  uint32_t dict_slot[LN_COLS];  // decode table of loaded column li (< ST_DCOLS), or ST_NO_SLOT
  uint32_t filt_off;            // stage byte offset of the filter ids
  uint32_t stage_bytes;         // one step's column bytes + filter ids (<= ST_STAGE)
  uint32_t n_dslots;            // decode tables in use
  int32_t sum_kind[LN_SUMS];    // ST_SUM_*
  int32_t sum_first[LN_SUMS], sum_len[LN_SUMS];
  StreamTerm terms[LN_TERMS + VEC_TERMS];
  // AggDesc's tile / chunk arrays (filled at launch): read through the plan, so that the loop re-reads them from the
  // scalar cache instead of holding ten pointer SGPRs
  const uint32_t* tile_chunk;
  const uint64_t* chunk_tile_begin;
  const uint32_t* chunk_size;
  const uint64_t* chunk_row_begin;
  const hy_scan_chunk* filter;
};

typedef __attribute__((address_space(3))) void st_lds_t;
typedef const __attribute__((address_space(1))) void st_g_t;

template <int SZ>
__device__ __forceinline__ void st_dma(const void* src, void* lds) {
  if constexpr (SZ == 16)
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 16, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 4, 0, 0);
}

// The lane id recomputed where it is used (asm volatile: not hoisted), so the loop keeps no lane-offset registers
// alive across a step - at this kernel's register budget they were the values spilled, and a spill reload waits for
// every LDS-DMA issued before it.
__device__ __forceinline__ uint32_t st_lane() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// The 256 rows [base, base + 256) of a column of `width`-byte elements into `lds` in row order: 4-byte pieces per lane
// for 1- and 2-byte ids, 16-byte pieces for 4-byte elements. At a chunk's end a lane's piece is clamped to the last
// aligned piece that holds a row of the chunk: an aligned piece holding one valid byte lies on a mapped page, and the
// rows past the end it repeats are inactive. (Only dword-sized LDS-DMA is used: measured on MI355X, the byte / short
// forms do not pack their lanes.)
__device__ __forceinline__ void st_load_column(const void* data, uint32_t width, uint32_t base, uint32_t size,
                                               void* lds) {
  const uint32_t lane = st_lane();
  const char* p = static_cast<const char*>(data);
  char* l = static_cast<char*>(lds);
  const uint64_t last = uint64_t(size - 1u) * width;  // byte offset of the chunk's last element
  const uint64_t b = uint64_t(base) * width;
  if (width == 4) {
    st_dma<16>(p + min(b + 16u * lane, last & ~uint64_t(15)), l);
  } else if (width == 2) {
    st_dma<4>(p + min(b + 4u * lane, last & ~uint64_t(3)), l);
    st_dma<4>(p + min(b + 256u + 4u * lane, last & ~uint64_t(3)), l + 256);
  } else {
    st_dma<4>(p + min(b + 4u * lane, last & ~uint64_t(3)), l);
  }
}

// A lane's 4 rows of a staged column (element width 1, 2 or 4), zero-extended.
__device__ __forceinline__ void st_read4(const unsigned char* col, uint32_t width, uint32_t (&v)[FQ_R]) {
  const uint32_t lane = st_lane();
  if (width == 1) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(col + 4u * lane);
#pragma unroll
    for (int k = 0; k < FQ_R; ++k) v[k] = (w >> (8 * k)) & 0xFFu;
  } else if (width == 2) {
    const uint2 w = *reinterpret_cast<const uint2*>(col + 8u * lane);
    v[0] = w.x & 0xFFFFu;
    v[1] = w.x >> 16;
    v[2] = w.y & 0xFFFFu;
    v[3] = w.y >> 16;
  } else {
    const uint4 w = *reinterpret_cast<const uint4*>(col + 16u * lane);
    v[0] = w.x;
    v[1] = w.y;
    v[2] = w.z;
    v[3] = w.w;
  }
}

// A tile's column descriptors (wave-uniform, kept in registers for the tile's steps): per loaded column its data and
// packed info (bits 0-2 element width, bit 3 dictionary, bits 8-15 dictionary size, bits 16-23 decode table slot).
// (Re-reading them from the scalar cache at every use measured slower: 7.97 against 7.12 ms at TPC-H 1 SF100.)
struct StreamCtx {
  uint32_t tile, c, size, base0;  // tile, chunk, chunk rows, the tile's first row in the chunk
  uint32_t n_steps;               // steps of the tile
  const void* data[VEC_COLS];
  uint32_t info[VEC_COLS];
  const void* fdata;              // the filter's ids, its id range and width
  uint32_t f_lo, f_span, f_neg, f_dsize, f_width;
  bool valid;
};
__device__ __forceinline__ uint32_t st_width(uint32_t info) { return info & 7u; }
__device__ __forceinline__ bool st_dict(uint32_t info) { return (info >> 3) & 1u; }
__device__ __forceinline__ uint32_t st_dsize(uint32_t info) { return (info >> 8) & 0xFFu; }

// Ends a flush period (vec_flush's rules) with the period's steps kept as (tile, step mask) pairs. emax: the
// largest magnitude as float bits; emin: the smallest nonzero magnitude as (bits << 1) - 1.
template <int NS, int NA>
__device__ __forceinline__ void st_flush(uint32_t H, uint32_t words, const LanePlan& lp,
                                         const ln_cptr<StreamPlan> P, unsigned long long* records,
                                         double (&acc)[LN_GROUPS][NA], uint32_t (&cnt)[LN_GROUPS],
                                         uint32_t (&lo)[LN_GROUPS], uint32_t (&hi)[LN_GROUPS],
                                         const int32_t (&tab)[LN_GROUPS], float (&emax)[NA], uint32_t (&emin)[NA],
                                         const uint2* plist, uint32_t& n_plist, uint32_t& n_period) {
  const int lane = __lane_id();
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  int32_t base[NA];
  bool exact = true;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    base[s] = 1;
    if (P->sum_kind[s] != ST_SUM_FLOAT) continue;
    bool nan = false;
#pragma unroll
    for (int j = 0; j < LN_GROUPS; ++j) nan = nan || acc[j][s] != acc[j][s];
    if (__ballot(nan) != 0ull) exact = false;
    const uint32_t hi_bits = wave_max_u(__float_as_uint(emax[s]));
    if (hi_bits == 0) continue;  // no nonzero value this period
    const int e_hi = static_cast<int>(hi_bits >> 23);
    const int e_lo = max(static_cast<int>((wave_min_u(emin[s]) + 1u) >> 24), 1);  // denormals: unit 2^-149
    base[s] = __builtin_amdgcn_readfirstlane(e_lo);
    if (e_hi >= 0xFF || e_hi - e_lo > LN_WINDOW || e_lo > LN_BASE_MAX) exact = false;
  }
  if (!exact) {  // discard the period: its steps go to agg_dense_fused
    for (uint32_t i = 0; i < n_plist; ++i) {
      const uint2 e = plist[i];
      if (static_cast<uint32_t>(lane) < ST_STEPS && ((e.y >> lane) & 1u)) {
        const uint32_t slot = atomicAdd(lp.n_deferred, 1u);
        lp.deferred[slot] = e.x * ST_STEPS + static_cast<uint32_t>(lane);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < LN_GROUPS; ++j) {
    if (tab[j] < 0) continue;
    unsigned long long* rec = records + static_cast<uint64_t>(tab[j]) * words;
    const unsigned long long rows = exact ? fq_wave_sum(cnt[j]) : 0ull;
    const uint32_t first = exact ? lo[j] : 0u;  // wave-uniform already
    const uint32_t last1 = exact ? wave_max_u(hi[j]) : 0u;
    cnt[j] = 0;
    lo[j] = 0xFFFFFFFFu;
    hi[j] = 0;
    if (rows && lane == 0) {
      atomicAdd(rec + H + AGG_HDR_ROWS, rows);
      atomicMin(rec + H + AGG_HDR_FIRST, static_cast<unsigned long long>(first));
      atomicMax(rec + H + AGG_HDR_LAST, static_cast<unsigned long long>(last1 - 1u));
      for (int f = 0; f < T->n_cnt; ++f) atomicAdd(rec + T->cnt_word[f], rows);  // non-NULL counts
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double a = acc[j][s];
      acc[j][s] = 0.0;
      const int32_t kind = P->sum_kind[s];
      if (!exact || kind == ST_SUM_NONE || __ballot(a != 0.0) == 0ull) continue;
      const int b = base[s];
      const double units = kind == ST_SUM_FLOAT ? ldexp(a, 150 - b) : a;
      const int64_t tot = static_cast<int64_t>(fq_wave_sum(static_cast<uint64_t>(static_cast<int64_t>(units))));
      if (lane == 0) {
        for (int q = 0; q < T->sum_nfn[s]; ++q) {
          if (kind == ST_SUM_FLOAT)
            fq_add_scaled(rec + T->sum_word[s][q] + 2, T->sum_limbs[s], tot, b - 1);
          else
            atomicAdd(rec + T->sum_word[s][q] + 1, static_cast<unsigned long long>(tot));
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    emax[s] = 0.f;
    emin[s] = 0xFFFFFFFFu;
  }
  n_period = 0;
  n_plist = 0;
}

template <int NS>
__global__ __launch_bounds__(AGG_THREADS) __attribute__((amdgpu_waves_per_eu(3))) void agg_dense_stream(
    AggDesc d, LanePlan lp, const StreamPlan* __restrict__ plan, unsigned long long* __restrict__ records) {
  constexpr int NA = NS > 0 ? NS : 1;
  constexpr int R = FQ_R;
  constexpr uint32_t NONE = LN_GROUPS;
  // every LDS array its own object (see the header); only the stage is written by LDS-DMA
  __shared__ __align__(16) unsigned char s_stage[ST_WAVES][ST_STAGE];
  __shared__ __align__(16) uint4 s_vals[ST_WAVES][ST_VALS][WAVE];
  __shared__ __align__(16) uint32_t s_dtab[ST_WAVES][ST_DCOLS][WAVE];
  __shared__ __align__(16) uint32_t s_entry[ST_WAVES][ST_CODES];  // group code -> table entry (NONE: not in it)
  __shared__ uint2 s_plist[ST_WAVES][ST_PLIST];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  // the kernel arguments' fields as locals: the lambdas below capture by reference, and a captured by-value kernel
  // argument would be copied to scratch
  const uint32_t H = d.n_gb;
  const uint32_t words = d.words;
  const uint64_t n_tiles = d.n_tiles;
  uint32_t* const error = d.error;
  const LanePlan lpv = lp;
  const int nl = lp.n_load;
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  const ln_cptr<StreamPlan> P = ln_const(plan);
  const ln_cptr<uint32_t> tile_chunk = ln_const(d.tile_chunk);
  const ln_cptr<uint64_t> chunk_tile_begin = ln_const(d.chunk_tile_begin);
  const ln_cptr<uint32_t> chunk_size = ln_const(d.chunk_size);
  const ln_cptr<uint64_t> chunk_row_begin = ln_const(d.chunk_row_begin);
  const ln_cptr<hy_scan_chunk> filt = ln_const(d.filter);
  const bool filtered = d.filter != nullptr;
  unsigned char* const stage = &s_stage[w][0];
  uint4* const vals = &s_vals[w][0][0];
  uint32_t* const dtab = &s_dtab[w][0][0];
  uint32_t* const entry = &s_entry[w][0];
  uint2* const plist = &s_plist[w][0];

  double acc[LN_GROUPS][NA];
  uint32_t cnt[LN_GROUPS], lo[LN_GROUPS], hi[LN_GROUPS];  // per lane: rows, last row + 1; lo: wave's first row
  int32_t tab[LN_GROUPS];
  float emax[NA];
  uint32_t emin[NA];
#pragma unroll
  for (int j = 0; j < LN_GROUPS; ++j) {
    tab[j] = -1;
    cnt[j] = 0;
    lo[j] = 0xFFFFFFFFu;
    hi[j] = 0;
#pragma unroll
    for (int s = 0; s < NA; ++s) acc[j][s] = 0.0;
  }
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    emax[s] = 0.f;
    emin[s] = 0xFFFFFFFFu;
  }
  entry[st_lane()] = NONE;
  uint32_t n_period = 0, n_plist = 0;

  const uint32_t GW = gridDim.x * ST_WAVES;
  auto load_ctx = [&](uint32_t tile) __attribute__((always_inline)) -> StreamCtx {
    StreamCtx x{};
    x.valid = tile < n_tiles;
    if (!x.valid) return x;
    x.tile = tile;
    x.c = tile_chunk[tile];
    x.size = chunk_size[x.c];
    x.base0 = static_cast<uint32_t>(tile - chunk_tile_begin[x.c]) * AGG_TILE;
    x.n_steps = min(static_cast<uint32_t>(ST_STEPS), (x.size - x.base0 + WAVE * R - 1) / (WAVE * R));
#pragma unroll
    for (int li = 0; li < VEC_COLS; ++li) {
      if (li >= nl) break;
      const auto& ch = ln_const(T->load_chunks[li])[x.c];
      const bool dict = ch.kind == HY_COL_DICT;
      x.data[li] = ch.data;
      x.info[li] = (dict ? static_cast<uint32_t>(ch.vid_width) : 4u) | (dict ? 8u : 0u) |
                   (dict ? (ch.dictionary_size << 8) : 0u) | ((P->dict_slot[li] & 0xFFu) << 16);
    }
    if (filtered) {
      const auto& f = filt[x.c];
      const IdRange fr = id_range(f.op, f.search_vid, f.column.dictionary_size);
      x.fdata = f.column.data;
      x.f_lo = fr.lo;
      x.f_span = fr.span;
      x.f_neg = fr.neg;
      x.f_dsize = fr.dsize;
      x.f_width = static_cast<uint32_t>(f.column.vid_width);
    }
    return x;
  };
  // a step's column bytes and filter ids into the stage
  auto issue = [&](const StreamCtx& x, uint32_t h) __attribute__((always_inline)) {
    if (!x.valid) return;
    const uint32_t base = x.base0 + h * (WAVE * R);
#pragma unroll
    for (int li = 0; li < VEC_COLS; ++li) {
      if (li >= nl) break;
      st_load_column(x.data[li], st_width(x.info[li]), base, x.size, stage + P->col_off[li]);
    }
    if (filtered) st_load_column(x.fdata, x.f_width, base, x.size, stage + P->filt_off);
  };

  StreamCtx ctx = load_ctx(blockIdx.x * ST_WAVES + static_cast<uint32_t>(w));
  uint32_t h = 0;
  issue(ctx, 0);
  bool period_full = false;  // the period reached LN_FLUSH_STEPS steps or ST_PLIST tiles: flush before the next step
  // one flush site (st_flush is large): the loop runs once more with no step for the final flush
  for (;;) {
    const bool done = !ctx.valid;
    const uint32_t tile = ctx.tile, step = h;
    const uint32_t base = ctx.base0 + h * (WAVE * R);
    const uint32_t first = base + st_lane() * R;
    uint32_t act = 0, vnull = 0, g[R] = {0, 0, 0, 0};
    uint32_t rowv = 0;
    if (!done) {
      // this step's loads (issued one step ago) have landed in the stage. Explicit: the compiler's own LDS-DMA
      // tracking does not see a DMA issued in the previous loop iteration (measured: without this wait the stage was
      // read before its loads completed)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (h == 0) {  // the tile's decode tables (plain loads: one wait per tile)
#pragma unroll
        for (int li = 0; li < VEC_COLS; ++li) {
          if (li >= nl) break;
          const uint32_t info = ctx.info[li];
          const uint32_t k = (info >> 16) & 0xFFu;
          if (k == 0xFFu || !st_dict(info) || st_dsize(info) == 0) continue;
          const auto& ch = ln_const(T->load_chunks[li])[ctx.c];
          uint32_t v = ln_load_word(reinterpret_cast<uintptr_t>(ch.dictionary),
                                    4u * min(st_lane(), st_dsize(info) - 1u));
          if (static_cast<uint32_t>(li) < H) {  // group codes: a NULL id maps to the NULL code; codes must be < domain
            const uint32_t domain = T->gb_domain[li];
            const bool ent = st_lane() < st_dsize(info);
            if (__ballot(ent && v >= domain) != 0ull && st_lane() == 0) atomicOr(error, 2u);
            v = ent ? min(v, domain) : domain;
          }
          dtab[k * WAVE + st_lane()] = v;
        }
      }
      rowv = static_cast<uint32_t>(chunk_row_begin[ctx.c]) + first;
      // (A) everything read from the stage: the filter's matches, the group codes, the other columns decoded into
      // the wave's value area
      act = base + WAVE * R <= ctx.size ? 0xFu : 0u;
      if (!act) {
#pragma unroll
        for (int k = 0; k < R; ++k) act |= static_cast<uint32_t>(first + k < ctx.size) << k;
      }
      if (filtered) {
        uint32_t ids[R];
        st_read4(stage + P->filt_off, ctx.f_width, ids);
        const IdRange fr{ctx.f_lo, ctx.f_span, ctx.f_neg, ctx.f_dsize, true};
#pragma unroll
        for (int k = 0; k < R; ++k) act &= ~(static_cast<uint32_t>(!id_in_range(fr, ids[k])) << k);
      }
      bool bad_code = false;
#pragma unroll
      for (int li = 0; li < VEC_COLS; ++li) {
        if (li >= nl) break;
        const uint32_t info = ctx.info[li];
        const bool dict = st_dict(info);
        const bool gb = static_cast<uint32_t>(li) < H;
        uint32_t v[R];
        st_read4(stage + P->col_off[li], st_width(info), v);
        if (dict) {
          const uint32_t* tb = dtab + ((info >> 16) & 0xFFu) * WAVE;
          const uint32_t ds = st_dsize(info);
#pragma unroll
          for (int k = 0; k < R; ++k) {
            if (!gb) vnull |= static_cast<uint32_t>(v[k] >= ds) << k;  // (group-by tables map NULL ids themselves)
            v[k] = tb[min(v[k], static_cast<uint32_t>(ST_DICT_MAX))];
          }
        }
        if (gb) {
          const uint32_t domain = T->gb_domain[li], stride = T->gb_stride[li];
          if (!dict) {  // value codes: checked per row
#pragma unroll
            for (int k = 0; k < R; ++k) {
              bad_code = bad_code || (v[k] >= domain && ((act >> k) & 1u));
              v[k] = min(v[k], domain);
            }
          }
#pragma unroll
          for (int k = 0; k < R; ++k) g[k] += v[k] * stride;
        } else {
          vals[(li - static_cast<int>(H)) * WAVE + st_lane()] = make_uint4(v[0], v[1], v[2], v[3]);
        }
      }
      if (__ballot(bad_code) != 0ull && st_lane() == 0) atomicOr(error, 2u);
      // every LDS read of the stage has returned before the next step's loads may overwrite it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (h + 1 < ctx.n_steps) {
        ++h;
      } else {
        ctx = load_ctx(ctx.tile + GW);
        h = 0;
      }
      issue(ctx, h);
    }
    const bool active = !done && __ballot(act != 0) != 0ull;
    const uint32_t step_id = tile * ST_STEPS + step;
    // (B) group codes -> table entries; codes the table lacks take free entries, or the period ends first
    uint32_t e[R];
    bool unmapped = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const bool a = (act >> k) & 1u;
      e[k] = a ? entry[min(g[k], static_cast<uint32_t>(ST_CODES - 1))] : NONE;
      unmapped = unmapped || (a && e[k] == NONE);
    }
    const bool remap = active && __ballot(unmapped) != 0ull;
    uint64_t present = 0, need = 0;
    bool refill = false;
    if (remap) {
      uint64_t mine = 0;
#pragma unroll
      for (int k = 0; k < R; ++k) mine |= ((act >> k) & 1u) ? (1ull << (g[k] & 63u)) : 0ull;
      present = ln_uniform64(wave_or64(mine));
      uint64_t have = 0;
      int free_slots = 0;
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) {
        if (tab[j] >= 0) have |= 1ull << tab[j];
        else ++free_slots;
      }
      need = present & ~have;
      refill = __popcll(need) > free_slots;
    }
    if (done || period_full || refill)
      st_flush<NS, NA>(H, words, lpv, P, records, acc, cnt, lo, hi, tab, emax, emin, plist, n_plist, n_period);
    period_full = false;
    if (done) break;
    if (!active) continue;
    if (remap) {
      if (refill) {
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) {
          if (tab[j] >= 0 && st_lane() == 0) entry[tab[j]] = NONE;
          tab[j] = -1;
        }
        need = present;
      }
      if (__popcll(need) > LN_GROUPS) {
        ln_defer(lpv, step_id);
        continue;
      }
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) {
        if (tab[j] < 0 && need) {
          tab[j] = __builtin_ctzll(need);
          need &= need - 1;
          if (st_lane() == 0) entry[tab[j]] = static_cast<uint32_t>(j);
        }
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        e[k] = NONE;
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j)
          e[k] = ((act >> k) & 1u) && g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];
      }
    }
    // NULLs in the other loaded columns send the step to agg_dense_fused
    if (__ballot((vnull & act) != 0) != 0ull) {
      ln_defer(lpv, step_id);
      continue;
    }
    // the rows of every entry as one-hot bits: bit 4 * e + k (entries past the table land above bit 15)
    uint32_t onehot = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) onehot |= 1u << (e[k] * 4u + static_cast<uint32_t>(k));
    // the FMA multipliers: m[k][j] = 1 when row k of the lane is in entry j (a register pair each, shared by the sums)
    double m[R][LN_GROUPS];
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) m[k][j] = (onehot >> (4 * j + k)) & 1u ? 1.0 : 0.0;
    // (C) per sum: its chain over the decoded values, then (D) its accumulation acc[j][s] += m[k][j] * x (exact when
    // the period checks out at its flush) - one sum's values live at a time
#pragma unroll
    for (int sn = 0; sn < NS; ++sn) {
      const int32_t kind = P->sum_kind[sn];
      if (kind == ST_SUM_NONE) continue;
      const int t0 = P->sum_first[sn], tn = P->sum_len[sn];
      float rf[R] = {0.f, 0.f, 0.f, 0.f};
      uint32_t ri[R] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < VEC_TERMS; ++t) {
        if (t >= tn) break;
        const StreamTerm tm{P->terms[t0 + t].a, P->terms[t0 + t].b, P->terms[t0 + t].col, P->terms[t0 + t].flags};
        float x[R] = {0.f, 0.f, 0.f, 0.f};
        if (!(tm.flags & ST_LIT)) {
          const uint4 q = vals[(tm.col - static_cast<int>(H)) * WAVE + st_lane()];
          const uint32_t qs[R] = {q.x, q.y, q.z, q.w};
          if (kind == ST_SUM_INT) {  // a plain int32 column: its bits as they are
#pragma unroll
            for (int k = 0; k < R; ++k) ri[k] = qs[k];
            break;
          }
#pragma unroll
          for (int k = 0; k < R; ++k)
            x[k] = (tm.flags & ST_CVT) ? static_cast<float>(static_cast<int32_t>(qs[k])) : __uint_as_float(qs[k]);
        }
        float tv[R];
#pragma unroll
        for (int k = 0; k < R; ++k) tv[k] = __builtin_fmaf(x[k], tm.a, tm.b);
        switch (tm.flags & ST_COMB) {  // uniform branches (each arm kept: no speculation of all four)
          case ST_SET:
#pragma unroll
            for (int k = 0; k < R; ++k) rf[k] = tv[k];
            break;
          case ST_ADD:
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < R; ++k) rf[k] = rf[k] + tv[k];
            break;
          case ST_SUB:
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < R; ++k) rf[k] = rf[k] - tv[k];
            break;
          case ST_RSUB:
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < R; ++k) rf[k] = tv[k] - rf[k];
            break;
          default:
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < R; ++k) rf[k] = rf[k] * tv[k];
            break;
        }
      }
      if (kind == ST_SUM_FLOAT) {  // the period's magnitude range (exactness, see the header)
        emax[sn] = fmaxf(emax[sn], fmaxf(fmaxf(fabsf(rf[0]), fabsf(rf[1])), fmaxf(fabsf(rf[2]), fabsf(rf[3]))));
#pragma unroll
        for (int k = 0; k < R; ++k) emin[sn] = min(emin[sn], (__float_as_uint(rf[k]) << 1) - 1u);  // zero: no effect
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const double xv = kind == ST_SUM_INT ? static_cast<double>(static_cast<int32_t>(ri[k]))
                                             : static_cast<double>(rf[k]);
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) acc[j][sn] = __builtin_fma(m[k][j], xv, acc[j][sn]);
      }
    }
#pragma unroll
    for (int j = 0; j < LN_GROUPS; ++j) {
      const uint32_t mb = (onehot >> (4 * j)) & 0xFu;  // this lane's rows of entry j
      cnt[j] += static_cast<uint32_t>(__popc(mb));
      hi[j] = mb ? rowv + static_cast<uint32_t>(31 - __builtin_clz(mb)) + 1u : hi[j];
      // the period's first row of entry j: wave-uniform, reduced once - when the entry first has rows
      if (lo[j] == 0xFFFFFFFFu && __ballot(mb != 0) != 0ull)
        lo[j] = __builtin_amdgcn_readfirstlane(
            wave_min_u(mb ? rowv + static_cast<uint32_t>(__builtin_ctz(mb)) : 0xFFFFFFFFu));
    }
    // the period's steps as (tile, step mask) pairs
    if (n_plist == 0 || plist[n_plist - 1].x != tile) {
      if (st_lane() == 0) plist[n_plist] = make_uint2(tile, 1u << step);
      ++n_plist;
    } else if (st_lane() == 0) {
      plist[n_plist - 1].y |= 1u << step;
    }
    period_full = ++n_period >= LN_FLUSH_STEPS || n_plist >= ST_PLIST;
  }
}

}  // namespace hyk
