// agg_dense_stream: agg_dense_vec (aggregate_vec.hip) with its column loads taken off the critical path - the TPC-H 1
// shape (data input, TableScan fused as a dictionary id range, a few dictionary group codes, SUM / AVG over float
// columns and + - * chains of them). Reference: Projection::_on_execute (projection.cpp:39-87) materialising the
// SELECT list, then Aggregate (aggregate.cpp:133-249, 291-498) summing it; the fused predicate is
// SingleColumnTableScanImpl's dictionary rewrite (single_column_table_scan_impl.cpp:145-205).
//
// Round 3 measured agg_dense_vec latency-bound: each 256-row step issued its column loads and waited for them before
// any arithmetic (168 VGPRs, 3 waves per SIMD, waves stalled ~60 % of their cycles); prefetching the next step into
// registers spilled. Here the loads go straight to LDS (global_load_lds, no VGPR destination), one step ahead:
//   * work unit: a wave takes whole 4096-row tiles (16 steps of 256 rows, grid-stride over the tiles by wave), so the
//     step sequence of a wave is known in advance and a tile's dictionaries are read once;
//   * two stage slots per wave, separate __shared__ objects, the loop unrolled by two: while a wave computes the step
//     in one slot, the next step's columns and filter ids stream into the other.
//     The compiler's wait before an LDS read covers only LDS-DMA writes into the same object, so the read of one slot
//     waits for that slot's loads and leaves the other slot's in flight;
//   * a row's 4 consecutive rows per lane come from one LDS read per column (the stage holds each column's bytes in
//     row order: 16-byte DMA per lane for 4-byte columns, 4-byte DMA for narrower ids of full steps; a step at a
//     chunk's end loads element-wise with clamped rows);
//   * dictionary ids are decoded through per-wave LDS tables, filled at a tile's first step by plain loads (one wait
//     per tile that also drains the next step's loads); group-by tables map a NULL id to the NULL code and are
//     checked against the code domain once per tile;
//   * accumulation, exactness per flush period and deferral to agg_dense_fused are agg_dense_vec's (vec_flush's
//     rules); a discarded period's steps are kept as (tile, step mask) pairs.
// Preconditions (host, plan_stream): agg_dense_vec's, plus: every DICT chunk of a loaded column has <= ST_DICT_MAX
// dictionary entries, the filter (if any) is a dictionary id range on every chunk, the stage layout fits.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int ST_WAVES = AGG_THREADS / WAVE;
constexpr int ST_STEPS = AGG_TILE / (WAVE * FQ_R);  // steps of a tile (16)
constexpr int ST_STAGE = 4096;                      // bytes of one step's column bytes + filter ids, per wave
constexpr int ST_DCOLS = 6;                         // dictionary-decoded loaded columns
constexpr int ST_VALS = 6;                          // loaded columns besides the group-by columns
constexpr int ST_DICT_MAX = 63;                     // dictionary entries (id 63 may then only be a NULL id)
constexpr int ST_PLIST = 64;                        // tiles recorded per period
constexpr uint32_t ST_NO_SLOT = 0xFFFFFFFFu;

// The stage layout of a plan (device memory, read through the constant address space).
struct StreamLayout {
  uint32_t col_off[LN_COLS];   // stage byte offset of loaded column li (256 rows x its widest chunk width)
  uint32_t dict_slot[LN_COLS]; // decode table of loaded column li (< ST_DCOLS), or ST_NO_SLOT
  uint32_t filt_off;           // stage byte offset of the filter ids
};

typedef __attribute__((address_space(3))) void st_lds_t;
typedef const __attribute__((address_space(1))) void st_g_t;

template <int SZ>
__device__ __forceinline__ void st_dma(const void* src, void* lds) {
  if constexpr (SZ == 16)
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 16, 0, 0);
  else if constexpr (SZ == 4)
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 4, 0, 0);
  else if constexpr (SZ == 2)
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 2, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((st_g_t*)src, (st_lds_t*)lds, 1, 0, 0);
}

// The lane id recomputed where it is used (asm volatile: not hoisted), so the loop keeps no lane-offset registers
// alive across a step - at this kernel's register budget they were the values spilled, and a spill reload here waits
// for every LDS-DMA issued before it.
__device__ __forceinline__ uint32_t st_lane() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// The 256 rows [base, base + 256) of a column of `width`-byte elements into `lds` in row order: 4-byte pieces per lane
// for 1- and 2-byte ids, 16-byte pieces for 4-byte elements. At a chunk's end a lane's piece is clamped to the last
// aligned piece that holds a row of the chunk: an aligned piece holding one valid byte lies on a mapped page, and the
// rows past the end it repeats are inactive. (Only dword-sized LDS-DMA is used: the byte / short forms are not relied
// on to pack their lanes.)
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
  const uint32_t lane = __lane_id();
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

// One step of a wave's sequence (wave-uniform).
struct StreamStep {
  uint32_t tile, c, base, size, h;
  bool valid, first;  // first: the tile's first step (fills the decode tables)
};

// Ends a flush period (vec_flush's rules) with the period's steps kept as (tile, step mask) pairs.
template <int NS, int NA>
__device__ __forceinline__ void st_flush(uint32_t H, uint32_t words, const LanePlan& lp, unsigned long long* records,
                                         double (&acc)[LN_GROUPS][NA], uint32_t (&cnt)[LN_GROUPS],
                                         uint32_t (&lo)[LN_GROUPS], uint32_t (&hi)[LN_GROUPS],
                                         const int32_t (&tab)[LN_GROUPS], uint32_t (&emax)[NA], uint32_t (&emin)[NA],
                                         const uint2* plist, uint32_t& n_plist, uint32_t& n_period) {
  const int lane = __lane_id();
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  int32_t base[NA];
  bool exact = true;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    base[s] = 1;
    if (T->sum_kind[s] != LN_SUM_FLOAT) continue;
    const uint32_t hi_bits = wave_max_u(emax[s]);
    if (hi_bits == 0) continue;  // no nonzero value this period
    const int e_hi = static_cast<int>(hi_bits >> 23);
    const int e_lo = max(static_cast<int>((wave_min_u(emin[s]) + 1u) >> 23), 1);  // denormals: unit 2^-149
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
      const int32_t kind = T->sum_kind[s];
      if (!exact || kind == LN_SUM_CHECK || __ballot(a != 0.0) == 0ull) continue;
      const int b = base[s];
      const double units = kind == LN_SUM_FLOAT ? ldexp(a, 150 - b) : a;
      const int64_t tot = static_cast<int64_t>(fq_wave_sum(static_cast<uint64_t>(static_cast<int64_t>(units))));
      if (lane == 0) {
        for (int q = 0; q < T->sum_nfn[s]; ++q) {
          if (kind == LN_SUM_FLOAT)
            fq_add_scaled(rec + T->sum_word[s][q] + 2, T->sum_limbs[s], tot, b - 1);
          else
            atomicAdd(rec + T->sum_word[s][q] + 1, static_cast<unsigned long long>(tot));
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    emax[s] = 0;
    emin[s] = 0xFFFFFFFFu;
  }
  n_period = 0;
  n_plist = 0;
}

template <int NS, bool ALLF>
__global__ __launch_bounds__(AGG_THREADS) __attribute__((amdgpu_waves_per_eu(3))) void agg_dense_stream(
    AggDesc d, LanePlan lp, const StreamLayout* __restrict__ layout, unsigned long long* __restrict__ records) {
  constexpr int NA = NS > 0 ? NS : 1;
  constexpr int R = FQ_R;
  // every LDS array its own object (see the header): the stage, the decoded values, the decode tables, the period's
  // steps - only the stage is written by LDS-DMA
  __shared__ __align__(16) unsigned char s_stage[ST_WAVES][ST_STAGE];
  __shared__ __align__(16) uint4 s_vals[ST_WAVES][ST_VALS][WAVE];
  __shared__ __align__(16) uint32_t s_dtab[ST_WAVES][ST_DCOLS][WAVE];
  __shared__ uint2 s_plist[ST_WAVES][ST_PLIST];
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  // the kernel arguments' fields as locals: the lambdas below capture by reference, and a captured by-value kernel
  // argument would be copied to scratch
  const uint32_t H = d.n_gb;
  const uint32_t words = d.words;
  const uint64_t n_tiles = d.n_tiles;
  uint32_t* const error = d.error;
  const LanePlan lpv = lp;
  const int nl = lp.n_load;
  const ln_cptr<LaneTables> T0 = ln_const(lp.t);
  const ln_cptr<LnTerm> terms0 = ln_const(lp.terms);
  const ln_cptr<StreamLayout> L0 = ln_const(layout);
  const ln_cptr<uint32_t> tile_chunk = ln_const(d.tile_chunk);
  const ln_cptr<uint64_t> chunk_tile_begin = ln_const(d.chunk_tile_begin);
  const ln_cptr<uint32_t> chunk_size = ln_const(d.chunk_size);
  const ln_cptr<uint64_t> chunk_row_begin = ln_const(d.chunk_row_begin);
  const ln_cptr<hy_scan_chunk> filt = ln_const(d.filter);
  const bool filtered = d.filter != nullptr;
  unsigned char* const stage = &s_stage[w][0];
  uint4* const vals = &s_vals[w][0][0];
  uint32_t* const dtab = &s_dtab[w][0][0];
  uint2* const plist = &s_plist[w][0];

  double acc[LN_GROUPS][NA];
  uint32_t cnt[LN_GROUPS], lo[LN_GROUPS], hi[LN_GROUPS];  // per lane: rows, last row + 1; lo: wave's first row
  int32_t tab[LN_GROUPS];
  uint32_t emax[NA], emin[NA];
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
    emax[s] = 0;
    emin[s] = 0xFFFFFFFFu;
  }
  uint32_t n_period = 0, n_plist = 0;

  const uint32_t GW = gridDim.x * ST_WAVES;
  auto tile_step = [&](uint32_t tile) __attribute__((always_inline)) -> StreamStep {  // a tile's first step
    StreamStep s{};
    s.valid = tile < n_tiles;
    if (!s.valid) return s;
    s.tile = tile;
    s.c = tile_chunk[tile];
    s.base = static_cast<uint32_t>(tile - chunk_tile_begin[s.c]) * AGG_TILE;
    s.size = chunk_size[s.c];
    s.h = 0;
    s.first = true;
    return s;
  };
  // a step's column bytes and filter ids into the stage
  auto issue = [&](const StreamStep& s, ln_cptr<LaneTables> T, ln_cptr<StreamLayout> L) __attribute__((always_inline)) {
    if (!s.valid) return;
#pragma unroll 1
    for (int li = 0; li < nl; ++li) {
      const auto& ch = ln_const(T->load_chunks[li])[s.c];
      const uint32_t width = ch.kind == HY_COL_DICT ? static_cast<uint32_t>(ch.vid_width) : 4u;
      st_load_column(ch.data, width, s.base, s.size, stage + L->col_off[li]);
    }
    if (filtered) {
      const auto& f = filt[s.c];
      st_load_column(f.column.data, static_cast<uint32_t>(f.column.vid_width), s.base, s.size, stage + L->filt_off);
    }
  };

  StreamStep cur = tile_step(blockIdx.x * ST_WAVES + static_cast<uint32_t>(w));
  issue(cur, T0, L0);
  bool period_full = false;  // the period reached LN_FLUSH_STEPS steps or ST_PLIST tiles: flush before the next step
  // one flush site (st_flush is large): the loop runs once more with no step for the final flush
  for (;;) {
    // the plan's tables re-read every step through an opaque zero offset: hoisted out of the loop, their ~100
    // loop-invariant scalars would be kept in SGPRs and spill (to VGPR lanes and scratch)
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const ln_cptr<LaneTables> T = T0 + z;
    const ln_cptr<LnTerm> terms = terms0 + z;
    const ln_cptr<StreamLayout> L = L0 + z;
    const bool done = !cur.valid;
    const StreamStep s = cur;
    uint32_t act = 0, vnull = 0;
    uint32_t g[R] = {0, 0, 0, 0};
    const uint32_t first = s.base + static_cast<uint32_t>(st_lane()) * R;
    if (!done) {
      StreamStep nxt;
      if (s.h + 1 < ST_STEPS && s.base + WAVE * R < s.size) {
        nxt = s;
        nxt.base += WAVE * R;
        nxt.h += 1;
        nxt.first = false;
      } else {
        nxt = tile_step(s.tile + GW);
      }
      const uint32_t c = s.c;
      if (s.first) {  // the tile's decode tables (plain loads: one wait per tile)
#pragma unroll 1
        for (int li = 0; li < nl; ++li) {
          const uint32_t k = L->dict_slot[li];
          const auto& ch = ln_const(T->load_chunks[li])[c];
          if (k == ST_NO_SLOT || ch.kind != HY_COL_DICT || ch.dictionary_size == 0) continue;
          uint32_t v = ln_load_word(reinterpret_cast<uintptr_t>(ch.dictionary),
                                    4u * min(static_cast<uint32_t>(st_lane()), ch.dictionary_size - 1u));
          if (static_cast<uint32_t>(li) < H) {  // group codes: a NULL id maps to the NULL code; codes must be < domain
            const uint32_t domain = T->gb_domain[li];
            const bool entry = static_cast<uint32_t>(st_lane()) < ch.dictionary_size;
            if (__ballot(entry && v >= domain) != 0ull && st_lane() == 0) atomicOr(error, 2u);
            v = entry ? min(v, domain) : domain;
          }
          dtab[k * WAVE + st_lane()] = v;
        }
      }
      // (A) everything read from the stage: the filter's matches, the group codes, the other columns decoded into
      // the wave's value area; then the next step's loads go out while this step is accumulated
#pragma unroll
      for (int k = 0; k < R; ++k) act |= static_cast<uint32_t>(first + k < s.size) << k;
      if (filtered) {
        const auto& f = filt[c];
        const IdRange fr = id_range(f.op, f.search_vid, f.column.dictionary_size);
        uint32_t ids[R];
        st_read4(stage + L->filt_off, static_cast<uint32_t>(f.column.vid_width), ids);
#pragma unroll
        for (int k = 0; k < R; ++k) act &= ~(static_cast<uint32_t>(!id_in_range(fr, ids[k])) << k);
      }
      bool bad_code = false;
#pragma unroll 1
      for (int li = 0; li < nl; ++li) {
        const auto& ch = ln_const(T->load_chunks[li])[c];
        const bool dict = ch.kind == HY_COL_DICT;
        const bool gb = static_cast<uint32_t>(li) < H;
        uint32_t v[R];
        st_read4(stage + L->col_off[li], dict ? static_cast<uint32_t>(ch.vid_width) : 4u, v);
        if (dict) {
          const uint32_t* tb = dtab + L->dict_slot[li] * WAVE;
          const uint32_t ds = ch.dictionary_size;
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
      // every LDS read of the stage has returned before the next step's loads may overwrite it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(nxt, T, L);
      cur = nxt;
      if (__ballot(bad_code) != 0ull && st_lane() == 0) atomicOr(error, 2u);
    }
    const bool active = !done && __ballot(act != 0) != 0ull;
    const uint32_t step_id = s.tile * ST_STEPS + s.h;
    // (B) group codes -> table entries; codes the table lacks take free entries, or the period ends first
#pragma unroll
    for (int k = 0; k < R; ++k) g[k] = ((act >> k) & 1u) ? g[k] : LN_NO_ROW;
    uint32_t e[R];
    bool unmapped = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      e[k] = LN_GROUPS;
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) e[k] = g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];
      unmapped = unmapped || (((act >> k) & 1u) && e[k] == LN_GROUPS);
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
    if (done || period_full || refill) {
      st_flush<NS, NA>(H, words, lpv, records, acc, cnt, lo, hi, tab, emax, emin, plist, n_plist, n_period);
      period_full = false;
    }
    if (done) break;
    if (!active) continue;
    if (remap) {
      if (refill) {
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) tab[j] = -1;
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
        }
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        e[k] = LN_GROUPS;
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j)
          e[k] = g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];
      }
    }
    // NULLs in the other loaded columns send the step to agg_dense_fused
    if (__ballot((vnull & act) != 0) != 0ull) {
      ln_defer(lpv, step_id);
      continue;
    }
    // (C) chains over the decoded values (agg_dense_vec's LnTerm programs)
    uint32_t r[NA][R];
#pragma unroll
    for (int sn = 0; sn < NS; ++sn) {
#pragma unroll
      for (int k = 0; k < R; ++k) r[sn][k] = 0;
      const int32_t skind = T->sum_kind[sn];
      if (skind == LN_SUM_CHECK) continue;
      const bool fl = ALLF || T->sum_float[sn] != 0;
      const int t0 = T->sum_first[sn], tn = T->sum_len[sn];
      int32_t kind[VEC_TERMS], op[VEC_TERMS], col[VEC_TERMS], cvt[VEC_TERMS], comb[VEC_TERMS], rev[VEC_TERMS];
      uint32_t lit[VEC_TERMS];
#pragma unroll
      for (int t = 0; t < VEC_TERMS; ++t) {  // (terms past the chain are valid memory: the host pads the table)
        kind[t] = terms[t0 + t].kind;
        op[t] = terms[t0 + t].op;
        col[t] = terms[t0 + t].col;
        lit[t] = terms[t0 + t].lit;
        cvt[t] = terms[t0 + t].cvt;
        comb[t] = terms[t0 + t].comb;
        rev[t] = terms[t0 + t].rev;
      }
#pragma unroll
      for (int t = 0; t < VEC_TERMS; ++t) {
        if (t >= tn) break;
        uint32_t x[R];
        if (kind[t] == LN_TERM_LIT) {
#pragma unroll
          for (int k = 0; k < R; ++k) x[k] = lit[t];
        } else {
          const uint4 q = vals[(col[t] - static_cast<int>(H)) * WAVE + st_lane()];
          x[0] = q.x;
          x[1] = q.y;
          x[2] = q.z;
          x[3] = q.w;
          if (cvt[t]) {
#pragma unroll
            for (int k = 0; k < R; ++k) x[k] = __float_as_uint(static_cast<float>(static_cast<int32_t>(x[k])));
          }
          if (kind[t] != LN_TERM_COL) {
            uint32_t l[R];
#pragma unroll
            for (int k = 0; k < R; ++k) l[k] = lit[t];
            if (kind[t] == LN_TERM_LIT_COL) ln_apply(op[t], fl, l, x, x);
            else ln_apply(op[t], fl, x, l, x);
          }
        }
        if (t == 0) {
#pragma unroll
          for (int k = 0; k < R; ++k) r[sn][k] = x[k];
        } else if (rev[t]) {
          ln_apply(comb[t], fl, x, r[sn], r[sn]);
        } else {
          ln_apply(comb[t], fl, r[sn], x, r[sn]);
        }
      }
#pragma unroll
      for (int k = 0; k < R; ++k) r[sn][k] = ((act >> k) & 1u) ? r[sn][k] : 0u;
      if (ALLF || skind == LN_SUM_FLOAT) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const uint32_t ax = r[sn][k] & 0x7FFFFFFFu;
          emax[sn] = max(emax[sn], ax);
          emin[sn] = min(emin[sn], ax - 1u);  // a zero wraps to 0xFFFFFFFF: no effect
        }
      }
    }
    // (D) accumulate: acc[j][s] += (row in entry j) * x; exact when the period checks out at its flush
#pragma unroll
    for (int k = 0; k < R; ++k) {
      double xv[NA];
#pragma unroll
      for (int sn = 0; sn < NS; ++sn) {
        if (ALLF)
          xv[sn] = static_cast<double>(__uint_as_float(r[sn][k]));
        else
          xv[sn] = T->sum_kind[sn] == LN_SUM_FLOAT ? static_cast<double>(__uint_as_float(r[sn][k]))
                                                   : static_cast<double>(static_cast<int32_t>(r[sn][k]));
      }
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) {
        const double m = e[k] == static_cast<uint32_t>(j) ? 1.0 : 0.0;
#pragma unroll
        for (int sn = 0; sn < NS; ++sn) acc[j][sn] = __builtin_fma(m, xv[sn], acc[j][sn]);
      }
    }
    const uint32_t rowv = static_cast<uint32_t>(chunk_row_begin[s.c]) + first;
#pragma unroll
    for (int j = 0; j < LN_GROUPS; ++j) {
      uint32_t mb = 0;
#pragma unroll
      for (int k = 0; k < R; ++k) mb |= static_cast<uint32_t>(e[k] == static_cast<uint32_t>(j)) << k;
      cnt[j] += static_cast<uint32_t>(__popc(mb));
      hi[j] = mb ? rowv + static_cast<uint32_t>(31 - __builtin_clz(mb)) + 1u : hi[j];
      // the period's first row of entry j: wave-uniform, reduced once - when the entry first has rows
      if (lo[j] == 0xFFFFFFFFu && __ballot(mb != 0) != 0ull)
        lo[j] = __builtin_amdgcn_readfirstlane(
            wave_min_u(mb ? rowv + static_cast<uint32_t>(__builtin_ctz(mb)) : 0xFFFFFFFFu));
    }
    // the period's steps as (tile, step mask) pairs
    if (n_plist == 0 || plist[n_plist - 1].x != s.tile) {
      if (st_lane() == 0) plist[n_plist] = make_uint2(s.tile, 1u << s.h);
      ++n_plist;
    } else if (st_lane() == 0) {
      plist[n_plist - 1].y |= 1u << s.h;
    }
    period_full = ++n_period >= LN_FLUSH_STEPS || n_plist >= ST_PLIST;
  }
}

}  // namespace hyk
