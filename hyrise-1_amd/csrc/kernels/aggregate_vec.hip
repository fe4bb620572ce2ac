// agg_dense_vec: agg_dense_lanes (aggregate_lanes.hip) for a DATA input - the TPC-H 1 shape with its TableScan fused
// in (hy_agg_input.filter) - restructured for instruction count. Reference: Projection::_on_execute
// (projection.cpp:39-87) materialising the SELECT list, then Aggregate (aggregate.cpp:133-249, 291-498) summing it.
//
// Measured on MI355X (round 3, PMC): agg_dense_lanes issues ~940 VALU + ~800 SALU instructions per 256-row step and is
// issue-bound, not memory-bound (0.7 TB/s). Here:
//   * a lane's 4 rows of a step are consecutive (base + 4 * lane + k): one vector load per column and step; the wave
//     index is made wave-uniform (readfirstlane) so step bounds are scalar branches, not exec-mask bookkeeping;
//   * the fused scan's dictionary predicate is an id range per chunk (one subtract / compare / xor per row);
//   * columns are decoded in a rolled loop into the wave's LDS (small code, few live registers);
//   * exactness is checked per flush PERIOD instead of per step: every lane keeps, per float sum, the largest and the
//     smallest nonzero magnitude it accumulated (two integer max / min on the float bits per value). At the flush the
//     wave takes the smallest exponent E_lo as the period's base: each value is then an integer multiple of
//     2^(E_lo - 150), and if the largest exponent E_hi <= E_lo + LN_WINDOW every lane's double partial sum of <= 2048
//     values stayed below 2^53 units - every addition was exact, and the sum folds into the group record's limbs as an
//     exact integer. A period that breaks this (a wider spread, non-finite values, exponents past LN_BASE_MAX) is
//     discarded - its partial sums, rows and first / last rows are dropped - and its steps (their ids are kept in LDS)
//     are deferred to agg_dense_fused, like steps with NULL inputs or more than LN_GROUPS groups.
//   * first / last rows are tracked per lane (reduced at the flush).
// Preconditions (host, plan_lanes): data input; every loaded column chunk 16-byte aligned, DICT (any width) or 4-byte
// VALUE without NULL flags; the table's rows < 2^32.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int VEC_TERMS = 4;  // terms per sum's chain (longer chains: agg_dense_lanes)
constexpr int VEC_COLS = 7;   // loaded columns (more: agg_dense_lanes)
constexpr uint32_t VEC_NO_DICT = 0xFFFFFFFFu;

// Per-wave LDS of agg_dense_vec: the stored columns of a step (agg_dense_lanes' layout), the flush staging, the
// small dictionaries, then the ids of the period's accumulated steps.
__host__ __device__ inline size_t vec_wave_lds(int n_store, int n_sums) {
  return ln_wave_lds(n_store, n_sums) + LN_FLUSH_STEPS * 4;
}

__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
  return static_cast<uint32_t>(wave_max_i(static_cast<int>(v ^ 0x80000000u))) ^ 0x80000000u;
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
  return static_cast<uint32_t>(wave_min_i(static_cast<int>(v ^ 0x80000000u))) ^ 0x80000000u;
}

// Ends a flush period: checks its exactness (see the header), then folds the lanes' partial sums, rows and first /
// last rows into the group records - or, if the period is not exact, defers its steps instead. Resets the period.
template <int NS, int NA>
__device__ __forceinline__ void vec_flush(const AggDesc& d, const LanePlan& lp, unsigned long long* records,
                                          double (&acc)[LN_GROUPS][NA], uint32_t (&cnt)[LN_GROUPS],
                                          uint32_t (&lo)[LN_GROUPS], uint32_t (&hi)[LN_GROUPS],
                                          const int32_t (&tab)[LN_GROUPS], uint32_t (&emax)[NA], uint32_t (&emin)[NA],
                                          double* stage, uint32_t* plist, uint32_t& n_period) {
  const int lane = __lane_id();
  const uint32_t H = d.n_gb;
  const uint32_t words = d.words;
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
    for (uint32_t i = static_cast<uint32_t>(lane); i < n_period; i += WAVE) {
      const uint32_t slot = atomicAdd(lp.n_deferred, 1u);
      lp.deferred[slot] = plist[i];
    }
  }
#pragma unroll
  for (int j = 0; j < LN_GROUPS; ++j) {
    if (tab[j] < 0) continue;
    unsigned long long* rec = records + static_cast<uint64_t>(tab[j]) * words;
    const unsigned long long rows = exact ? fq_wave_sum(cnt[j]) : 0ull;
    const uint32_t first = exact ? wave_min_u(lo[j]) : 0u;
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
      stage[s * WAVE + lane] = acc[j][s];
      acc[j][s] = 0.0;
    }
    if (!exact) continue;
#pragma unroll 1
    for (int s = 0; s < NS; ++s) {
      const int32_t kind = T->sum_kind[s];
      const double a = stage[s * WAVE + lane];
      if (kind == LN_SUM_CHECK || __ballot(a != 0.0) == 0ull) continue;
      const int b = __builtin_amdgcn_readfirstlane(base[s < NA ? s : 0]);
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
}

// ALLF: every sum is a float sum (TPC-H 1): no per-value choice between the float and the int32 conversion.
template <int NS, bool ALLF>
__global__ __launch_bounds__(AGG_THREADS) __attribute__((amdgpu_waves_per_eu(3))) void agg_dense_vec(
    AggDesc d, LanePlan lp, unsigned long long* __restrict__ records) {
  constexpr int NA = NS > 0 ? NS : 1;
  constexpr int R = FQ_R;
  extern __shared__ __align__(16) unsigned char s_lanes[];
  const int lane = __lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);  // wave-uniform: steps branch on scalars
  const uint32_t H = d.n_gb;
  const int nl = lp.n_load;
  const int n_store = nl - static_cast<int>(H);
  unsigned char* wl = s_lanes + static_cast<size_t>(w) * vec_wave_lds(n_store, NS);
  uint4* vals = reinterpret_cast<uint4*>(wl);                        // [stored column][lane]
  double* stage = reinterpret_cast<double*>(vals + n_store * WAVE);  // [sum][lane]
  // (agg_dense_lanes' per-entry headers and base slots follow the staging area; unused here)
  uint32_t* dcache = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(stage + NS * WAVE) +
                                                 LN_GROUPS * sizeof(LnHeader) + LN_SUMS * 4);  // [column][entry]
  uint32_t* plist = dcache + LN_COLS * LN_DICT_CACHE;  // ids of the period's accumulated steps
  const ln_cptr<LaneTables> T = ln_const(lp.t);
  const ln_cptr<LnTerm> terms = ln_const(lp.terms);

  double acc[LN_GROUPS][NA];
  uint32_t cnt[LN_GROUPS], lo[LN_GROUPS], hi[LN_GROUPS];  // per lane: rows, first row, last row + 1 (period)
  int32_t tab[LN_GROUPS];
  uint32_t emax[NA], emin[NA];  // per lane and float sum: largest magnitude bits, smallest nonzero magnitude bits - 1
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
  uint32_t n_period = 0;  // accumulated steps of the period (<= LN_FLUSH_STEPS)
  uint32_t cached_c = 0xFFFFFFFFu;
  // the fused scan's predicate on the current chunk: 0 none (every row), 1 dictionary id range, 2 generic
  uint32_t f_mode = 0, f_width = 1;
  uintptr_t f_data = 0;
  IdRange f_r{};

  for (uint64_t tile = blockIdx.x; tile < d.n_tiles; tile += gridDim.x) {
    const uint32_t c = agg_tile_chunk(d, tile);
    const uint32_t size = d.chunk_size[c];
    const uint32_t span = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE + w * AGG_WAVE_SPAN;
    const uint32_t row0 = static_cast<uint32_t>(d.chunk_row_begin[c]);
    if (c != cached_c) {  // the chunk's small dictionaries into the wave's LDS, its predicate's form
#pragma unroll 1
      for (int li = 0; li < nl; ++li) {
        const auto& ch = ln_const(T->load_chunks[li])[c];
        if (ch.kind == HY_COL_DICT && ch.dictionary_size <= LN_DICT_CACHE &&
            static_cast<uint32_t>(lane) < ch.dictionary_size)
          dcache[li * LN_DICT_CACHE + lane] =
              ln_load_word(reinterpret_cast<uintptr_t>(ch.dictionary), static_cast<uint32_t>(lane) * 4u);
      }
      if (d.filter != nullptr) {
        const auto& f = ln_const(d.filter)[c];
        f_mode = 2;
        if (f.column.kind == HY_COL_DICT) {
          f_r = id_range(f.op, f.search_vid, f.column.dictionary_size);
          if (f_r.range) {
            f_mode = 1;
            f_data = reinterpret_cast<uintptr_t>(f.column.data);
            f_width = static_cast<uint32_t>(f.column.vid_width);
          }
        }
      }
      cached_c = c;
    }
#pragma unroll 1
    for (int h = 0; h < AGG_ITEMS / R; ++h) {
      const uint32_t base = span + h * R * WAVE;
      if (base >= size) break;  // wave-uniform
      const uint32_t step_id = static_cast<uint32_t>(tile) * FQ_STEPS_PER_TILE + w * (AGG_ITEMS / R) + h;
      const uint32_t first = base + static_cast<uint32_t>(lane) * R;
      const bool full = base + R * WAVE <= size;  // wave-uniform
      uint32_t act = 0;
#pragma unroll
      for (int k = 0; k < R; ++k) act |= static_cast<uint32_t>(first + k < size) << k;
      // (0) every column's ids / values of the step in flight at once (the descriptors are scalar loads of one
      // batch), before anything waits on them
      uint32_t raw[VEC_COLS][R];
      uint32_t cdsize[VEC_COLS];  // dictionary size (ids >= it: NULL), VEC_NO_DICT for a value chunk
#pragma unroll
      for (int li = 0; li < VEC_COLS; ++li) {
        if (li >= nl) break;
        const auto& ch = ln_const(T->load_chunks[li])[c];
        const bool dict = ch.kind == HY_COL_DICT;
        const uint32_t width = dict ? static_cast<uint32_t>(ch.vid_width) : 4u;
        cdsize[li] = dict ? ch.dictionary_size : VEC_NO_DICT;
        if (full)
          vec_load_ids<R>(ch.data, width, first, raw[li]);
        else
          elem_load_ids<R>(ch.data, width, first, size, raw[li]);
      }
      if (f_mode == 1) {  // fused TableScan, dictionary predicate: one vector load of the ids, a range test per row
        uint32_t ids[R];
        if (full)
          vec_load_ids<R>(reinterpret_cast<const void*>(f_data), f_width, first, ids);
        else
          elem_load_ids<R>(reinterpret_cast<const void*>(f_data), f_width, first, size, ids);
#pragma unroll
        for (int k = 0; k < R; ++k) act &= ~(static_cast<uint32_t>(!id_in_range(f_r, ids[k])) << k);
      } else if (f_mode == 2) {
        act &= agg_filter_mask<R, 1>(d, c, first);
      }
      if (__ballot(act != 0) == 0ull) continue;
      // decode: dictionary ids -> values (LDS cache of small dictionaries, else a gather); nl: NULL ids
      auto decode = [&](int li, uint32_t (&v)[R]) -> uint32_t {
        uint32_t nl_ = 0;
        if (cdsize[li] != VEC_NO_DICT) {
          const bool cached = cdsize[li] <= LN_DICT_CACHE;
          const uintptr_t dv = cached ? 0 : reinterpret_cast<uintptr_t>(ln_const(T->load_chunks[li])[c].dictionary);
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const bool isnull = v[k] >= cdsize[li];
            nl_ |= static_cast<uint32_t>(isnull) << k;
            const uint32_t id = isnull ? 0u : v[k];
            v[k] = cached ? dcache[li * LN_DICT_CACHE + id] : ln_load_word(dv, id * 4u);
          }
        }
        return nl_;
      };
      // (1) group codes -> table entries (a refill may end the period)
      uint32_t g[R] = {0, 0, 0, 0};
      bool bad_code = false;
#pragma unroll
      for (int li = 0; li < FQ_MAX_GB; ++li) {
        if (static_cast<uint32_t>(li) >= H) break;
        const uint32_t gn = decode(li, raw[li]);
        const uint32_t domain = T->gb_domain[li], stride = T->gb_stride[li];
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const bool isnull = (gn >> k) & 1u;
          const bool out = !isnull && raw[li][k] >= domain;
          bad_code = bad_code || (out && ((act >> k) & 1u));
          g[k] += ((isnull || out) ? domain : raw[li][k]) * stride;
        }
      }
      if (bad_code) atomicOr(d.error, 2u);
#pragma unroll
      for (int k = 0; k < R; ++k) g[k] = ((act >> k) & 1u) ? g[k] : LN_NO_ROW;
      uint32_t e[R];  // table entry of each row (LN_GROUPS: none / inactive)
      bool unmapped = false;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        e[k] = LN_GROUPS;
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) e[k] = g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];
        unmapped = unmapped || (((act >> k) & 1u) && e[k] == LN_GROUPS);
      }
      if (__ballot(unmapped) != 0ull) {  // new group codes: free entries, or flush and refill
        uint64_t mine = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) mine |= ((act >> k) & 1u) ? (1ull << (g[k] & 63u)) : 0ull;
        const uint64_t present = ln_uniform64(wave_or64(mine));
        uint64_t have = 0;
        int free_slots = 0;
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) {
          if (tab[j] >= 0) have |= 1ull << tab[j];
          else ++free_slots;
        }
        uint64_t need = present & ~have;
        if (__popcll(need) > free_slots) {
          vec_flush<NS, NA>(d, lp, records, acc, cnt, lo, hi, tab, emax, emin, stage, plist, n_period);
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
#pragma unroll
        for (int k = 0; k < R; ++k) {
          e[k] = LN_GROUPS;
#pragma unroll
          for (int j = 0; j < LN_GROUPS; ++j)
            e[k] = g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];
        }
      }
      // (2) the other loaded columns, decoded, into the wave's LDS (the chains read them by column index)
      uint32_t vnull = 0;  // rows with a NULL in a non-group-by column
#pragma unroll
      for (int li = 0; li < VEC_COLS; ++li) {
        if (li >= nl) break;
        if (static_cast<uint32_t>(li) < H) continue;
        vnull |= decode(li, raw[li]);
        vals[(li - static_cast<int>(H)) * WAVE + lane] = make_uint4(raw[li][0], raw[li][1], raw[li][2], raw[li][3]);
      }
      if (__ballot((vnull & act) != 0) != 0ull) {
        ln_defer(lp, step_id);
        continue;
      }
      // (3) chains (agg_dense_lanes' LnTerm programs, at most VEC_TERMS terms per sum: all of a sum's term fields are
      // read in one batch of scalar loads, not one dependent round trip per field); COUNT-only inputs need no value
      uint32_t r[NA][R];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
#pragma unroll
        for (int k = 0; k < R; ++k) r[s][k] = 0;
        const int32_t skind = T->sum_kind[s];
        if (skind == LN_SUM_CHECK) continue;
        const bool fl = ALLF || T->sum_float[s] != 0;
        const int t0 = T->sum_first[s], tn = T->sum_len[s];
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
            const uint4 q = vals[(col[t] - static_cast<int>(H)) * WAVE + lane];
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
            for (int k = 0; k < R; ++k) r[s][k] = x[k];
          } else if (rev[t]) {
            ln_apply(comb[t], fl, x, r[s], r[s]);
          } else {
            ln_apply(comb[t], fl, r[s], x, r[s]);
          }
        }
        // rows that take no part count as 0 (a filtered-out row's value - even non-finite - never reaches the sums)
#pragma unroll
        for (int k = 0; k < R; ++k) r[s][k] = ((act >> k) & 1u) ? r[s][k] : 0u;
        if (ALLF || skind == LN_SUM_FLOAT) {  // the period's magnitude range (exactness, see the header)
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const uint32_t ax = r[s][k] & 0x7FFFFFFFu;
            emax[s] = max(emax[s], ax);
            emin[s] = min(emin[s], ax - 1u);  // a zero wraps to 0xFFFFFFFF: no effect
          }
        }
      }
      // (4) accumulate: acc[j][s] += (row in entry j) * x; exact when the period checks out at its flush
#pragma unroll
      for (int k = 0; k < R; ++k) {
        double xv[NA];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if (ALLF)
            xv[s] = static_cast<double>(__uint_as_float(r[s][k]));
          else
            xv[s] = T->sum_kind[s] == LN_SUM_FLOAT ? static_cast<double>(__uint_as_float(r[s][k]))
                                                   : static_cast<double>(static_cast<int32_t>(r[s][k]));
        }
#pragma unroll
        for (int j = 0; j < LN_GROUPS; ++j) {
          const double m = e[k] == static_cast<uint32_t>(j) ? 1.0 : 0.0;
#pragma unroll
          for (int s = 0; s < NS; ++s) acc[j][s] = __builtin_fma(m, xv[s], acc[j][s]);
        }
      }
      // rows, first / last rows per lane: a lane's rows only grow (tiles and steps are taken in row order)
      const uint32_t rowv = row0 + first;
#pragma unroll
      for (int j = 0; j < LN_GROUPS; ++j) {
        uint32_t mb = 0;  // this lane's rows of entry j
#pragma unroll
        for (int k = 0; k < R; ++k) mb |= static_cast<uint32_t>(e[k] == static_cast<uint32_t>(j)) << k;
        cnt[j] += static_cast<uint32_t>(__popc(mb));
        hi[j] = mb ? rowv + static_cast<uint32_t>(31 - __builtin_clz(mb)) + 1u : hi[j];
        lo[j] = (lo[j] == 0xFFFFFFFFu && mb) ? rowv + static_cast<uint32_t>(__builtin_ctz(mb)) : lo[j];
      }
      if (lane == 0) plist[n_period] = step_id;
      if (++n_period >= LN_FLUSH_STEPS)
        vec_flush<NS, NA>(d, lp, records, acc, cnt, lo, hi, tab, emax, emin, stage, plist, n_period);
    }
  }
  vec_flush<NS, NA>(d, lp, records, acc, cnt, lo, hi, tab, emax, emin, stage, plist, n_period);
}

}  // namespace hyk
