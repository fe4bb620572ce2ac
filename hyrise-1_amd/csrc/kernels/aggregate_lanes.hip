// agg_dense_lanes: the dense Aggregate with its Projection fused in, accumulating per lane - TPC-H 1's shape (a few
// groups from dictionary codes; SUM / AVG of float columns and of arithmetic expressions over them; COUNT) over a
// TableScan's output. Reference: Projection::_on_execute (projection.cpp:39-87) materialising
// l_extendedprice * (1 - l_discount) etc., then Aggregate (aggregate.cpp:133-249, 291-498) summing sequentially.
//
// agg_dense_fused reduces every aggregate of every group across the wave on every 256-row step (~6k wave instructions
// per step): ALU-bound at ~4% of the HBM roofline. Here each lane keeps its own exact fixed-point partial sums and the
// wave reduces them only when it flushes (every LN_FLUSH_STEPS steps and at the end):
//   * group table: a wave accumulates LN_GROUPS group codes at once (wave-uniform table; Q1 has 4 groups). A step
//     with codes outside the table claims free entries; a full table is flushed and refilled.
//   * sums: one per distinct SUM / AVG input (SUM(x) and AVG(x) share it), evaluated from the loaded columns as a
//     chain of terms (see LnTerm; the host compiles the expression programs) in the reference's calc type.
//   * exactness: a lane accumulates in a double. Every float value v = m * 2^(e - 150) (24-bit m) of a sum has its
//     biased exponent e in [base, base + LN_WINDOW] (per-wave, per-sum base), so it is an integer multiple of
//     2^(base - 150) below 2^(24 + LN_WINDOW) units; 2048 rows per lane keep every partial sum below 2^53 units, so
//     each double addition is exact. The flush scales a lane's sum to its exact integer (< 2^53), sums the lanes as
//     int64 and folds the total into the group record's limbs at bit base - 1 - the same exact fixed-point sum as
//     every other path, rounded once on the host. int32 sums: < 2^42 per lane, exact in a double too.
//   * anything else - NULLs, non-finite or denormal values, exponents outside the window even after a re-base, a
//     step whose rows reference several chunks, more than LN_GROUPS codes in one step - sends the whole step to a
//     list that agg_dense_fused (list mode) processes afterwards. Record words combine by ADD / MIN / MAX, so the
//     split is exact.
// Roofline: HBM (RowIDs + the columns' bytes per row); ~80 VALU per row-slot keeps the ALU below the memory time.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int LN_GROUPS = 4;         // group codes a wave accumulates at once
constexpr int LN_SUMS = 8;           // distinct summed / checked inputs
constexpr int LN_COLS = 8;           // columns loaded per step (group-by columns first)
constexpr int LN_TERMS = 32;         // chain terms over all sums
constexpr int LN_WINDOW = 18;        // 0 <= e - base <= LN_WINDOW: a value is < 2^(24 + 18) units of 2^(base - 150)
constexpr int LN_HEAD = 4;           // a new base leaves room for exponents up to 4 above the step's largest
constexpr int LN_BASE_MAX = 200;     // fold pieces (base - 1 + 31 + 59 bits) stay inside the 9 float limbs
constexpr int LN_FLUSH_STEPS = 512;  // 4 rows per lane per step: <= 2048 rows, partial sums < 2^(42 + 11) units
constexpr int LN_DICT_CACHE = 64;    // dictionary entries of a loaded column kept in the wave's LDS (TPC-H 1: <= 50)

enum : int32_t { LN_TERM_COL = 0, LN_TERM_LIT = 1, LN_TERM_LIT_COL = 2, LN_TERM_COL_LIT = 3 };
enum : int32_t { LN_SUM_INT = 0, LN_SUM_FLOAT = 1, LN_SUM_CHECK = 2 };

// One term of a sum's chain. Term value: the loaded column (converted int32 -> float when cvt), a literal, or
// literal `op` column / column `op` literal (op: + - *). The chain's running value starts at term 0; term t > 0 joins it as
// running = running comb term (rev = 0) or running = term comb running (rev = 1). Every operation computes in the
// chain's type (float or int32), as the reference's ExpressionEvaluator does for 4-byte operands.
struct LnTerm {
  int32_t kind;
  int32_t op;
  int32_t col;   // loaded column index (>= the number of group-by columns)
  uint32_t lit;  // literal bits, already in the chain's type
  int32_t cvt;
  int32_t comb;
  int32_t rev;
  int32_t pad;
};

// Per-input tables of the plan, in device memory (indexed at run time by the flush; a runtime index into a kernel
// argument would make the compiler copy the argument to scratch).
constexpr int LN_SUM_FNS = 2;  // aggregates sharing one input (SUM(x) and AVG(x))
struct LaneTables {
  int32_t n_load, n_sums;                        // as LanePlan (host bookkeeping)
  const hy_column_chunk* load_chunks[LN_COLS];   // each loaded column's chunk descriptors
  uint32_t gb_domain[FQ_MAX_GB];                 // group-by columns: code domain and mixed-radix stride
  uint32_t gb_stride[FQ_MAX_GB];
  int32_t sum_kind[LN_SUMS];                     // LN_SUM_*
  int32_t sum_float[LN_SUMS];                    // the chain computes in float
  int32_t sum_first[LN_SUMS];                    // first term
  int32_t sum_len[LN_SUMS];
  int32_t sum_nfn[LN_SUMS];                      // SUM / AVG aggregates over this input
  uint32_t sum_word[LN_SUMS][LN_SUM_FNS];        // their first record words
  int32_t sum_limbs[LN_SUMS];                    // float: limbs of their accumulators
  int32_t n_cnt;                                 // aggregates with a column: their non-NULL count words
  uint32_t cnt_word[AGG_MAX_AGGREGATES];
};

struct LanePlan {
  int32_t n_load;                 // loaded columns; [0, n_gb) are the group-by columns
  int32_t n_sums;
  const LaneTables* t;            // device
  const LnTerm* terms;            // device
  uint32_t* deferred;             // device: step ids (FQ_STEPS_PER_TILE numbering) for agg_dense_fused
  uint32_t* n_deferred;
};

// Per-wave LDS of agg_dense_lanes: the step's loaded values (read by the chains at run-time column indices), the
// flush's staging of one group's lane partial sums, and the per-group rows / first / last row (updated by lane 0).
struct LnHeader {
  unsigned long long rows, first, last, pad;  // rows: unused (the lanes count them)
};
__host__ __device__ inline size_t ln_wave_lds(int n_store, int n_sums) {
  return size_t(n_store) * WAVE * 16 + size_t(n_sums) * WAVE * 8 + LN_GROUPS * sizeof(LnHeader) + LN_SUMS * 4 +
         size_t(LN_COLS) * LN_DICT_CACHE * 4;
}

// Chain operations. The term kind / op are wave-uniform: each case is a branch over the step's FQ_R rows (as selects
// the compiler would evaluate every operation for every row). + - * only (the host leaves / and % to
// agg_dense_fused); int32 wraps like the reference's functors.
#pragma clang fp contract(off)
__device__ __forceinline__ void ln_apply(int32_t op, bool fl, const uint32_t (&a)[FQ_R], const uint32_t (&b)[FQ_R],
                                         uint32_t (&o)[FQ_R]) {
  if (fl) {
    if (op == HY_EXPR_ADD) {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = __float_as_uint(__uint_as_float(a[k]) + __uint_as_float(b[k]));
    } else if (op == HY_EXPR_SUB) {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = __float_as_uint(__uint_as_float(a[k]) - __uint_as_float(b[k]));
    } else {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = __float_as_uint(__uint_as_float(a[k]) * __uint_as_float(b[k]));
    }
  } else {
    if (op == HY_EXPR_ADD) {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = a[k] + b[k];
    } else if (op == HY_EXPR_SUB) {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = a[k] - b[k];
    } else {
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) o[k] = a[k] * b[k];
    }
  }
}

// Read-only, wave-uniform data (the plan's tables and terms, the chunk descriptors) read through the constant address
// space: scalar loads. Through a generic pointer the compiler cannot rule out the kernel's own stores and emits
// vector loads with VGPR address arithmetic (~170 loads per step).
template <class X>
using ln_cptr = const __attribute__((address_space(4))) X*;
template <class X>
__device__ __forceinline__ ln_cptr<X> ln_const(const X* p) {
  return (ln_cptr<X>)(p);
}

// Column data in the global address space: global loads with a uniform (SGPR) base and 32-bit lane offsets instead
// of flat loads with 64-bit VGPR addresses.
using ln_gword = const __attribute__((address_space(1))) uint32_t*;
__device__ __forceinline__ uint32_t ln_load_word(uintptr_t base, uint32_t byte_off) {
  return *reinterpret_cast<ln_gword>(base + byte_off);
}
// Element `i` of a 1-, 2- or 4-byte wide array (wave-uniform width), zero-extended.
__device__ __forceinline__ uint32_t ln_load_elem(uintptr_t base, uint32_t i, uint32_t width) {
  if (width == 1) return *reinterpret_cast<const __attribute__((address_space(1))) uint8_t*>(base + i);
  if (width == 2) return *reinterpret_cast<const __attribute__((address_space(1))) uint16_t*>(base + 2ull * i);
  return *reinterpret_cast<ln_gword>(base + 4ull * i);
}

__device__ __forceinline__ uint64_t ln_uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void ln_defer(const LanePlan& lp, uint32_t step_id) {
  if (__lane_id() == 0) lp.deferred[atomicAdd(lp.n_deferred, 1u)] = step_id;
}

constexpr uint32_t LN_NO_ROW = 0xFFFFFFFEu;  // group code of inactive rows: matches no table entry (empty = -1)

// Folds a wave's lane partial sums and its per-entry rows / first / last into the group records; keeps the table.
template <int NS, int NA>
__device__ __forceinline__ void ln_flush(const AggDesc& d, const LanePlan& lp, unsigned long long* records,
                                         double (&acc)[LN_GROUPS][NA], uint32_t (&cnt)[LN_GROUPS],
                                         const int32_t (&tab)[LN_GROUPS], const int32_t (&fbase)[NA], double* stage,
                                         LnHeader* hdr, int32_t* sbase, uint32_t* first_set, uint32_t* since) {
  const int lane = __lane_id();
  const uint32_t H = d.n_gb;
  const uint32_t words = d.words;
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) sbase[s] = fbase[s];
  }
#pragma unroll
  for (int j = 0; j < LN_GROUPS; ++j) {
    if (tab[j] < 0) continue;
    unsigned long long* rec = records + static_cast<uint64_t>(tab[j]) * words;
    const unsigned long long rows = fq_wave_sum(cnt[j]);
    cnt[j] = 0;
    if (lane == 0) {
      const LnHeader hd = hdr[j];
      if (rows) {
        atomicAdd(rec + H + AGG_HDR_ROWS, rows);
        atomicMin(rec + H + AGG_HDR_FIRST, hd.first);
        atomicMax(rec + H + AGG_HDR_LAST, hd.last);
        for (int f = 0; f < T->n_cnt; ++f) atomicAdd(rec + T->cnt_word[f], rows);  // non-NULL counts
      }
      hdr[j] = LnHeader{0, ~0ull, 0, 0};
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      stage[s * WAVE + lane] = acc[j][s];
      acc[j][s] = 0.0;
    }
#pragma unroll 1
    for (int s = 0; s < NS; ++s) {
      const int32_t kind = T->sum_kind[s];
      const double a = stage[s * WAVE + lane];
      if (kind == LN_SUM_CHECK || __ballot(a != 0.0) == 0ull) continue;
      const int base = __builtin_amdgcn_readfirstlane(sbase[s]);
      // the lane's exact integer: float sums in units of 2^(base - 150), int32 sums as they are (|x| < 2^53)
      const double units = kind == LN_SUM_FLOAT ? ldexp(a, 150 - base) : a;
      const int64_t tot = static_cast<int64_t>(fq_wave_sum(static_cast<uint64_t>(static_cast<int64_t>(units))));
      if (lane == 0) {
        for (int q = 0; q < T->sum_nfn[s]; ++q) {
          if (kind == LN_SUM_FLOAT)
            fq_add_scaled(rec + T->sum_word[s][q] + 2, T->sum_limbs[s], tot, base - 1);
          else
            atomicAdd(rec + T->sum_word[s][q] + 1, static_cast<unsigned long long>(tot));
        }
      }
    }
  }
  *first_set = 0;
  *since = 0;
}

// The float sums' windows for the step's chain values: a sum without a base takes one from this step (largest
// exponent + LN_HEAD - LN_WINDOW); returns false if some nonzero value lies outside its sum's window. *hard: the
// base would pass LN_BASE_MAX.
template <int NS, int NA>
__device__ __forceinline__ bool ln_window_ok(const LanePlan& lp, const uint32_t (&r)[NA][FQ_R], uint32_t act,
                                             int32_t (&fbase)[NA], bool* hard) {
  bool ok = true;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (ln_const(lp.t)->sum_kind[s] != LN_SUM_FLOAT) continue;
    if (fbase[s] < 0) {
      uint32_t em = 0;
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) {
        const uint32_t ax = r[s][k] & 0x7FFFFFFFu;
        if (((act >> k) & 1u) && ax < 0x7F800000u) em = max(em, ax >> 23);
      }
      const int E = __builtin_amdgcn_readfirstlane(wave_max_i(static_cast<int>(em)));
      const int b = max(E + LN_HEAD - LN_WINDOW, 1);
      if (E > 0 && b <= LN_BASE_MAX) fbase[s] = b;
      else if (E > 0) *hard = true;  // values too large for the limbs' fold range
    }
    const uint32_t lo = static_cast<uint32_t>(fbase[s] < 0 ? 0 : fbase[s]) << 23;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < FQ_R; ++k) {
      const uint32_t ax = r[s][k] & 0x7FFFFFFFu;
      // nonzero and exponent outside [base, base + LN_WINDOW] (non-finite values and denormals included)
      if (((act >> k) & 1u) && ax != 0 && (fbase[s] < 0 || ax - lo >= ((LN_WINDOW + 1u) << 23))) bad = true;
    }
    if (__ballot(bad) != 0ull) ok = false;
  }
  return ok;
}

// PF: the next step's RowIDs are prefetched (8 more VGPRs). Round 2 measured 3 waves per SIMD (<= 168 VGPRs) best
// without it (4 spills, 2 left too little latency hiding); with the prefetch and the LDS dictionaries a step has one
// dependent global round trip instead of three, so the prefetching instance runs at 2 waves per SIMD (HY_AGG_PREFETCH
// picks it; tools measure both).
// VEC (data input, no PosList): a lane's FQ_R rows of a step are consecutive (base + lane * FQ_R + k) instead of
// strided by the wave (base + k * WAVE + lane), so every column is read with ONE vector load per lane and step (a
// dword of four u8 ids, a dwordx2 of u16 ids, a dwordx4 of 4-byte values; the host checked 16-byte alignment) instead
// of FQ_R single-element loads. A step still covers the same 256 rows, so deferred steps are unchanged.
template <int NS, bool PF, bool VEC>
__global__ __launch_bounds__(AGG_THREADS) __attribute__((amdgpu_waves_per_eu(PF ? 2 : 3))) void agg_dense_lanes(
    AggDesc d, LanePlan lp, unsigned long long* __restrict__ records) {
  constexpr int NA = NS > 0 ? NS : 1;
  extern __shared__ __align__(16) unsigned char s_lanes[];
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);  // wave-uniform: steps branch on scalars
  const uint32_t H = d.n_gb;
  const int n_store = lp.n_load - static_cast<int>(H);
  unsigned char* wl = s_lanes + static_cast<size_t>(w) * ln_wave_lds(n_store, NS);
  uint4* vals = reinterpret_cast<uint4*>(wl);                        // [stored column][lane]
  double* stage = reinterpret_cast<double*>(vals + n_store * WAVE);  // [sum][lane]
  LnHeader* hdr = reinterpret_cast<LnHeader*>(stage + NS * WAVE);    // [table entry]
  int32_t* sbase = reinterpret_cast<int32_t*>(hdr + LN_GROUPS);       // [sum]
  uint32_t* dcache = reinterpret_cast<uint32_t*>(sbase + LN_SUMS);     // [loaded column][dictionary entry]
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  const ln_cptr<LnTerm> terms = ln_const(lp.terms);
  if (lane < LN_GROUPS) hdr[lane] = LnHeader{0, ~0ull, 0, 0};

  double acc[LN_GROUPS][NA];
  uint32_t cnt[LN_GROUPS];  // the lane's rows per table entry
  int32_t tab[LN_GROUPS];
  int32_t fbase[NA];
  uint32_t first_set = 0;   // bit j: hdr[j].first holds the flush period's first row of entry j
#pragma unroll
  for (int j = 0; j < LN_GROUPS; ++j) {
    tab[j] = -1;
    cnt[j] = 0;
#pragma unroll
    for (int s = 0; s < NA; ++s) acc[j][s] = 0.0;
  }
#pragma unroll
  for (int s = 0; s < NA; ++s) fbase[s] = -1;
  uint32_t since = 0;
  // The (referenced) chunk whose small dictionaries sit in dcache, and which loaded columns they are (bit li): a
  // dictionary decode is then an LDS read instead of a dependent global load per row.
  uint32_t cached_cc = 0xFFFFFFFFu, cached = 0;

  for (uint64_t tile = blockIdx.x; tile < d.n_tiles; tile += gridDim.x) {
    const uint32_t c = agg_tile_chunk(d, tile);
    const uint32_t size = d.chunk_size[c];
    const uint32_t span = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE + w * AGG_WAVE_SPAN;
    const uint64_t row0 = d.chunk_row_begin[c];
    const uintptr_t pl = d.n_pos_groups ? reinterpret_cast<uintptr_t>(ln_const(d.pos_lists)[c]) : 0;
    // RowIDs of the next step, loaded during the current one (after its column loads, so waiting for those does not
    // wait for these)
    unsigned long long next_rid[FQ_R];
    bool have_next = false;  // a deferred step (continue below) leaves no prefetch for its successor
    for (int h = 0; h < AGG_ITEMS / FQ_R; ++h) {
      const uint32_t base = span + h * FQ_R * WAVE;
      if (base >= size) break;  // wave-uniform
      const uint32_t step_id = static_cast<uint32_t>(tile) * FQ_STEPS_PER_TILE + w * (AGG_ITEMS / FQ_R) + h;
      constexpr uint32_t STR = VEC ? 1u : static_cast<uint32_t>(WAVE);  // row step between a lane's items
      const uint32_t first = VEC ? base + lane * FQ_R : base + lane;
      const bool full = VEC && first + FQ_R <= size;                      // the lane's items all in the chunk
      uint32_t act = 0;
#pragma unroll
      for (int k = 0; k < FQ_R; ++k)
        if (first + k * STR < size) act |= 1u << k;
      // row offsets inside the (single) chunk the step's rows live in
      uint32_t off[FQ_R];
      uint32_t cc = c;
      const bool prefetch = PF && d.n_pos_groups && h + 1 < AGG_ITEMS / FQ_R && base + FQ_R * WAVE < size;
      if (!VEC && d.n_pos_groups) {
        hy_row_id rid[FQ_R];
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) {
          unsigned long long q;
          if (!have_next) {
            const uint32_t i = min(base + k * WAVE + lane, size - 1);
            q = *reinterpret_cast<const __attribute__((address_space(1))) unsigned long long*>(pl + 8ull * i);
          } else {
            q = next_rid[k];
          }
          rid[k] = hy_row_id{static_cast<uint32_t>(q), static_cast<uint32_t>(q >> 32)};
        }
        have_next = false;
        cc = __builtin_amdgcn_readfirstlane(rid[0].chunk_id);
        bool same = true;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) {
          if ((act >> k) & 1u) same = same && rid[k].chunk_id == cc && rid[k].chunk_offset != 0xFFFFFFFFu;
          off[k] = ((act >> k) & 1u) ? rid[k].chunk_offset : 0u;
        }
        if (__ballot(!same) != 0ull || cc == 0xFFFFFFFFu) {
          ln_defer(lp, step_id);
          continue;
        }
      } else {
        if (d.filter != nullptr) act &= agg_filter_mask<FQ_R, STR>(d, c, first);  // fused TableScan
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) off[k] = ((act >> k) & 1u) ? first + k * STR : 0u;
      }
      // the chunk's small dictionaries into the wave's LDS (once per chunk change)
      if (cc != cached_cc) {
        cached = 0;
#pragma unroll 1
        for (int li = 0; li < LN_COLS; ++li) {
          if (li >= lp.n_load) break;
          const auto& ch = ln_const(T->load_chunks[li])[cc];
          if (ch.kind == HY_COL_DICT && ch.dictionary_size <= LN_DICT_CACHE) {
            if (static_cast<uint32_t>(lane) < ch.dictionary_size)
              dcache[li * LN_DICT_CACHE + lane] =
                  ln_load_word(reinterpret_cast<uintptr_t>(ch.dictionary), static_cast<uint32_t>(lane) * 4u);
            cached |= 1u << li;
          }
        }
        cached_cc = cc;
      }
      // loads: every column's value / vid first (one batch in flight), then vids -> dictionary values
      uint32_t raw[LN_COLS][FQ_R];
#pragma unroll
      for (int li = 0; li < LN_COLS; ++li) {
        if (li >= lp.n_load) break;
        const auto& ch = ln_const(T->load_chunks[li])[cc];
        const uint32_t wb = ch.kind == HY_COL_DICT ? static_cast<uint32_t>(ch.vid_width) : 4u;
        const uintptr_t p0 = reinterpret_cast<uintptr_t>(ch.data);
        if (full) {
          vec_load_ids<FQ_R>(ch.data, wb, first, raw[li]);
        } else {
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) raw[li][k] = ln_load_elem(p0, off[k], wb);
        }
      }
      if (prefetch) {  // the next step's RowIDs, behind this step's column loads
        have_next = true;
        const uint32_t nb = base + FQ_R * WAVE;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) {
          const uint32_t i = min(nb + k * WAVE + lane, size - 1);
          next_rid[k] = *reinterpret_cast<const __attribute__((address_space(1))) unsigned long long*>(pl + 8ull * i);
        }
      }
      uint32_t g[FQ_R] = {0, 0, 0, 0};
      uint32_t nulls = 0;  // rows with a NULL in a non-group-by column
      bool bad_code = false;
#pragma unroll
      for (int li = 0; li < LN_COLS; ++li) {
        if (li >= lp.n_load) break;
        const auto& ch = ln_const(T->load_chunks[li])[cc];
        const bool dict = ch.kind == HY_COL_DICT;
        uint32_t v[FQ_R];
        uint32_t nl = 0;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) v[k] = raw[li][k];
        if (dict && ((cached >> li) & 1u)) {
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) {
            const bool isnull = v[k] >= ch.dictionary_size;
            if (isnull) nl |= 1u << k;
            v[k] = dcache[li * LN_DICT_CACHE + (isnull ? 0u : v[k])];
          }
        } else if (dict) {
          const uintptr_t dv = reinterpret_cast<uintptr_t>(ch.dictionary);
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) {
            const bool isnull = v[k] >= ch.dictionary_size;
            if (isnull) nl |= 1u << k;
            v[k] = ln_load_word(dv, (isnull ? 0u : v[k]) * 4u);
          }
        } else if (ch.nulls != nullptr) {  // nullable value column: its NULL flag bytes
          const uintptr_t n0 = reinterpret_cast<uintptr_t>(ch.nulls);
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            if (ln_load_elem(n0, off[k], 1)) nl |= 1u << k;
        }
        if (li < FQ_MAX_GB && static_cast<uint32_t>(li) < H) {
          const uint32_t domain = T->gb_domain[li < FQ_MAX_GB ? li : 0];
          const uint32_t stride = T->gb_stride[li < FQ_MAX_GB ? li : 0];
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) {
            uint32_t code = domain;
            if (!((nl >> k) & 1u)) {
              code = v[k];
              if (code >= domain) {
                bad_code = bad_code || ((act >> k) & 1u);
                code = domain;
              }
            }
            g[k] += code * stride;
          }
        } else {
          nulls |= nl;
          vals[(li - static_cast<int>(H)) * WAVE + lane] = make_uint4(v[0], v[1], v[2], v[3]);
        }
      }
      if (bad_code) atomicOr(d.error, 2u);
#pragma unroll
      for (int k = 0; k < FQ_R; ++k)
        if (!((act >> k) & 1u)) g[k] = LN_NO_ROW;
      if (__ballot((nulls & act) != 0) != 0ull) {
        ln_defer(lp, step_id);
        continue;
      }
      // group table: every row's code must have an entry
      {
        uint32_t mapped = 0;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k)
#pragma unroll
          for (int j = 0; j < LN_GROUPS; ++j)
            if (g[k] == static_cast<uint32_t>(tab[j])) mapped |= 1u << k;
        if (__ballot((act & ~mapped) != 0) != 0ull) {
          uint64_t mine = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            if ((act >> k) & 1u) mine |= 1ull << (g[k] & 63u);
          const uint64_t present = ln_uniform64(wave_or64(mine));
          uint64_t have = 0;
          int free_slots = 0;
#pragma unroll
          for (int j = 0; j < LN_GROUPS; ++j) {
            if (tab[j] >= 0) have |= 1ull << tab[j];
            else ++free_slots;
          }
          uint64_t need = present & ~have;
          if (__popcll(need) > free_slots) {  // flush and refill
            ln_flush<NS, NA>(d, lp, records, acc, cnt, tab, fbase, stage, hdr, sbase, &first_set, &since);
#pragma unroll
            for (int j = 0; j < LN_GROUPS; ++j) tab[j] = -1;
            need = present;
          }
          if (__popcll(need) > LN_GROUPS) {
            ln_defer(lp, step_id);
            continue;
          }
#pragma unroll
          for (int j = 0; j < LN_GROUPS; ++j) {
            if (tab[j] < 0 && need) {
              tab[j] = __builtin_ctzll(need);
              need &= need - 1;
            }
          }
        }
      }
      // sums: chain values of the step's rows
      uint32_t r[NA][FQ_R];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bool fl = T->sum_float[s] != 0;
        const int t0 = T->sum_first[s], tn = T->sum_len[s];
#pragma unroll 1
        for (int t = 0; t < tn; ++t) {
          LnTerm tm;  // field by field (a constant-address-space struct has no copy constructor)
          tm.kind = terms[t0 + t].kind;
          tm.op = terms[t0 + t].op;
          tm.col = terms[t0 + t].col;
          tm.lit = terms[t0 + t].lit;
          tm.cvt = terms[t0 + t].cvt;
          tm.comb = terms[t0 + t].comb;
          tm.rev = terms[t0 + t].rev;
          uint32_t x[FQ_R];
          if (tm.kind == LN_TERM_LIT) {
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) x[k] = tm.lit;
          } else {
            const uint4 q = vals[(tm.col - static_cast<int>(H)) * WAVE + lane];
            x[0] = q.x;
            x[1] = q.y;
            x[2] = q.z;
            x[3] = q.w;
            if (tm.cvt) {
#pragma unroll
              for (int k = 0; k < FQ_R; ++k) x[k] = __float_as_uint(static_cast<float>(static_cast<int32_t>(x[k])));
            }
            if (tm.kind != LN_TERM_COL) {
              uint32_t l[FQ_R];
#pragma unroll
              for (int k = 0; k < FQ_R; ++k) l[k] = tm.lit;
              if (tm.kind == LN_TERM_LIT_COL) ln_apply(tm.op, fl, l, x, x);
              else ln_apply(tm.op, fl, x, l, x);
            }
          }
          if (t == 0) {
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) r[s][k] = x[k];
          } else if (tm.rev) {
            ln_apply(tm.comb, fl, x, r[s], r[s]);
          } else {
            ln_apply(tm.comb, fl, r[s], x, r[s]);
          }
        }
      }
      bool hard = false;
      if (!ln_window_ok<NS, NA>(lp, r, act, fbase, &hard) && !hard) {
        // re-base: flush, drop the bases and take them from this step
        ln_flush<NS, NA>(d, lp, records, acc, cnt, tab, fbase, stage, hdr, sbase, &first_set, &since);
#pragma unroll
        for (int s = 0; s < NA; ++s) fbase[s] = -1;
        if (!ln_window_ok<NS, NA>(lp, r, act, fbase, &hard)) hard = true;
      }
      if (hard) {
        ln_defer(lp, step_id);
        continue;
      }
      // accumulate: acc[j][s] = fma(m, x, acc[j][s]) with m = 1.0 for the rows of entry j, else 0.0 - exactly the
      // (exact, see above) sum, without a branch per entry; the lane's row counts likewise
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) {
        double xv[NA];
#pragma unroll
        for (int s = 0; s < NS; ++s)
          xv[s] = T->sum_float[s] ? static_cast<double>(__uint_as_float(r[s][k]))
                                  : static_cast<double>(static_cast<int32_t>(r[s][k]));
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) {
          const bool in = g[k] == static_cast<uint32_t>(tab[j]);  // empty entries (-1) match no row
          const double m = static_cast<double>(static_cast<uint32_t>(in));  // (a select would become select + add)
          cnt[j] += in ? 1u : 0u;
#pragma unroll
          for (int s = 0; s < NS; ++s) acc[j][s] = __builtin_fma(m, xv[s], acc[j][s]);
        }
      }
      // first row (once per flush period) and last row per entry; lane 0 keeps them in LDS
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) {
        if (tab[j] < 0) continue;
        if constexpr (VEC) {  // row of (lane, k) = base + lane * FQ_R + k
          uint32_t mine = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) mine |= static_cast<uint32_t>(g[k] == static_cast<uint32_t>(tab[j])) << k;
          const uint64_t anyb = __ballot(mine != 0);
          if (anyb == 0) continue;
          const uint64_t rb = row0 + base;
          const int ll = 63 - __builtin_clzll(anyb);
          const uint32_t ml = static_cast<uint32_t>(__shfl(static_cast<int>(mine), ll));
          if (lane == 0)
            atomicMax(&hdr[j].last, static_cast<unsigned long long>(rb + ll * FQ_R + 31 - __builtin_clz(ml)));
          if (!((first_set >> j) & 1u)) {
            const int lf = __builtin_ctzll(anyb);
            const uint32_t mf = static_cast<uint32_t>(__shfl(static_cast<int>(mine), lf));
            if (lane == 0) atomicMin(&hdr[j].first, static_cast<unsigned long long>(rb + lf * FQ_R + __builtin_ctz(mf)));
            first_set |= 1u << j;
          }
          continue;
        }
        uint64_t mk[FQ_R];
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) mk[k] = __ballot(g[k] == static_cast<uint32_t>(tab[j]));
        if ((mk[0] | mk[1] | mk[2] | mk[3]) == 0) continue;
        const uint64_t rb = row0 + base;
        const int kl = mk[3] ? 3 : mk[2] ? 2 : mk[1] ? 1 : 0;
        const uint64_t ml = mk[3] ? mk[3] : mk[2] ? mk[2] : mk[1] ? mk[1] : mk[0];
        const uint64_t ls = rb + kl * WAVE + 63 - __builtin_clzll(ml);
        if (lane == 0) atomicMax(&hdr[j].last, static_cast<unsigned long long>(ls));
        if (!((first_set >> j) & 1u)) {
          const int kf = mk[0] ? 0 : mk[1] ? 1 : mk[2] ? 2 : 3;
          const uint64_t mf = mk[0] ? mk[0] : mk[1] ? mk[1] : mk[2] ? mk[2] : mk[3];
          if (lane == 0) atomicMin(&hdr[j].first, static_cast<unsigned long long>(rb + kf * WAVE + __builtin_ctzll(mf)));
          first_set |= 1u << j;
        }
      }
      if (++since >= LN_FLUSH_STEPS) ln_flush<NS, NA>(d, lp, records, acc, cnt, tab, fbase, stage, hdr, sbase, &first_set, &since);
    }
  }
  ln_flush<NS, NA>(d, lp, records, acc, cnt, tab, fbase, stage, hdr, sbase, &first_set, &since);
}

}  // namespace hyk
