// agg_dense_fused: the dense Aggregate with its Projection fused in - TPC-H 1's shape (a handful of groups from
// dictionary codes, SUM / AVG of float columns and of arithmetic expressions over them, COUNT, over a TableScan's
// output). Reference: Projection::_on_execute (projection.cpp:39-87) materialising l_extendedprice * (1 - l_discount)
// etc., then Aggregate (aggregate.cpp:133-249, 291-498) summing sequentially.
//
// Per step a wave takes 256 consecutive input rows of one chunk (4 per lane, coalesced per k), loads the RowIDs, then
// every needed 4-byte column once into "slots" (one batched load per row and column: RowID -> value or vid ->
// dictionary; the referenced chunk's descriptor is wave-uniform for a scan output, per lane otherwise), evaluates the
// expression columns from the slots in registers, and folds each aggregate per group present in the step:
//   * float SUM / AVG: exact. The step's values of the aggregate share an exponent window: with E the largest
//     exponent, every value with exponent >= E - 31 is an integer multiple of 2^(E - 31 - 150) below 2^55, so a wave's
//     masked sum of them is an exact int64, added into the group's limbs (3 pieces) with LDS atomics. Rarer values
//     (smaller exponents, or steps near the float range's top) are added per row as exact limb pieces (float_parts).
//     Either way the record holds the exact sum, rounded once on the host: the same result as every other path.
//   * int32 SUM / AVG: int64 sums; MIN / MAX: order-preserving bits; COUNT: popcounts.
// Roofline: HBM (the RowIDs, the column bytes and vids per row); the window keeps the per-row ALU to a few dozen
// instructions, so the kernel is bound by memory latency / bandwidth rather than by exact summation.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

constexpr int FQ_R = 4;         // rows per lane per step
constexpr int FQ_SLOTS = 8;     // 4-byte value slots per step (plain columns + expressions)
constexpr int FQ_DEPTH = 4;     // expression stack depth
constexpr int FQ_MAX_GB = 4;    // group-by columns

// Expression op of the fused kernel (host-compiled from hy_expr_node; every value is 4 bytes): COLUMN pushes slot
// `arg`; VALUE pushes the literal bits `lit` (NULL when `arg` != 0); arithmetic pops b, a, converts the operands
// flagged in `arg` (bit 0: a, bit 1: b) from int32 to float, and computes in `calc` (int32 or float), which is also
// the result type: for 4-byte operand types std::common_type and expression_common_type agree.
struct FqOp {
  int32_t kind;   // HY_EXPR_*
  int32_t calc;   // HY_TYPE_INT32 / HY_TYPE_FLOAT (arithmetic)
  int32_t arg;
  uint32_t lit;
};

struct FusedPlan {
  int32_t n_slots;
  int32_t slot_col[FQ_SLOTS];   // plain slot: input column index (a 4-byte, non-expression column); else -1
  int32_t slot_prog[FQ_SLOTS];  // expression slot: first node in progs; else -1
  int32_t slot_nodes[FQ_SLOTS];
  int32_t slot_type[FQ_SLOTS];
  int32_t fn_slot[AGG_MAX_AGGREGATES];  // slot of each aggregate's column, -1 for COUNT(*)
  const FqOp* progs;            // device: the expressions' ops
};

// Value bits of one 4-byte column at (chunk descriptor, offset); false for NULL.
__device__ __forceinline__ bool fq_load_one(const hy_column_chunk& ch, uint32_t off, uint32_t* v) {
  if (ch.kind == HY_COL_DICT) {
    uint32_t vid;
    if (ch.vid_width == 1)
      vid = static_cast<const uint8_t*>(ch.data)[off];
    else if (ch.vid_width == 2)
      vid = static_cast<const uint16_t*>(ch.data)[off];
    else
      vid = static_cast<const uint32_t*>(ch.data)[off];
    if (vid >= ch.dictionary_size) return false;
    *v = static_cast<const uint32_t*>(ch.dictionary)[vid];
    return true;
  }
  if (ch.nulls != nullptr && ch.nulls[off]) return false;
  *v = static_cast<const uint32_t*>(ch.data)[off];
  return true;
}

// Values of a plain 4-byte column for the step's FQ_R rows of this lane; returns the non-NULL mask.
__device__ __forceinline__ uint32_t fq_load(const AggCol& col, uint32_t c, uint32_t base, uint32_t act, bool uniform,
                                            uint32_t cc, const hy_row_id (&rid)[FQ_R], uint32_t (&v)[FQ_R]) {
  const int lane = __lane_id();
  uint32_t ok = 0;
  if (col.pos_group < 0 || uniform) {
    const hy_column_chunk& ch = col.chunks[col.pos_group < 0 ? c : cc];  // wave-uniform descriptor
#pragma unroll
    for (int k = 0; k < FQ_R; ++k) {
      v[k] = 0;
      const uint32_t off = col.pos_group < 0 ? base + k * WAVE + lane : rid[k].chunk_offset;
      if (((act >> k) & 1u) && (col.pos_group < 0 || off != 0xFFFFFFFFu) && fq_load_one(ch, off, &v[k]))
        ok |= 1u << k;
    }
    return ok;
  }
#pragma unroll
  for (int k = 0; k < FQ_R; ++k) {  // rows of several referenced chunks: each row through its own descriptor
    v[k] = 0;
    if (((act >> k) & 1u) && rid[k].chunk_offset != 0xFFFFFFFFu &&
        fq_load_one(col.chunks[rid[k].chunk_id], rid[k].chunk_offset, &v[k]))
      ok |= 1u << k;
  }
  return ok;
}

// Slot s of value array `vals` at row k, by unrolled selection (keeps the arrays in registers).
__device__ __forceinline__ uint32_t fq_pick(const uint32_t (&vals)[FQ_SLOTS][FQ_R], int s, int k) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < FQ_SLOTS; ++j)
#pragma unroll
    for (int q = 0; q < FQ_R; ++q)
      if (j == s && q == k) r = vals[j][q];
  return r;
}

__device__ __forceinline__ uint32_t fq_pick_mask(const uint32_t (&m)[FQ_SLOTS], int s) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < FQ_SLOTS; ++j)
    if (j == s) r = m[j];
  return r;
}

// Wave reductions through DPP (row_shr within 16-lane rows, then row_bcast 15 / 31): VALU-only, the total lands in
// lane 63 and is read back as a wave-uniform value - no LDS permutes. 64-bit values travel as two 32-bit halves.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t fq_dpp64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(v), CTRL, ROW_MASK, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(v >> 32), CTRL, ROW_MASK, 0xf, false);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t fq_wave_sum(uint64_t v) {
  v += fq_dpp64<0x111, 0xf>(v);  // row_shr:1
  v += fq_dpp64<0x112, 0xf>(v);  // row_shr:2
  v += fq_dpp64<0x114, 0xf>(v);  // row_shr:4
  v += fq_dpp64<0x118, 0xf>(v);  // row_shr:8
  v += fq_dpp64<0x142, 0xa>(v);  // row_bcast:15
  v += fq_dpp64<0x143, 0xc>(v);  // row_bcast:31
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 63);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), 63);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// min / max of unsigned 64-bit values (identity `id` in lanes without a value)
template <bool MAX>
__device__ __forceinline__ uint64_t fq_wave_ext(uint64_t v, uint64_t id) {
  auto step = [&](uint64_t o) { v = MAX ? (o > v ? o : v) : (o < v ? o : v); };
  auto dpp = [&](auto tag) {
    constexpr int C = decltype(tag)::value;
    const uint32_t lo = __builtin_amdgcn_update_dpp(static_cast<uint32_t>(id), static_cast<uint32_t>(v), C, 0xf, 0xf,
                                                    false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(static_cast<uint32_t>(id >> 32), static_cast<uint32_t>(v >> 32), C,
                                                    0xf, 0xf, false);
    return (static_cast<uint64_t>(hi) << 32) | lo;
  };
  step(dpp(std::integral_constant<int, 0x111>{}));
  step(dpp(std::integral_constant<int, 0x112>{}));
  step(dpp(std::integral_constant<int, 0x114>{}));
  step(dpp(std::integral_constant<int, 0x118>{}));
  step(dpp(std::integral_constant<int, 0x142>{}));
  step(dpp(std::integral_constant<int, 0x143>{}));
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 63);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), 63);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Number of set bits (rows) over the step: k-th bit of every lane's mask, counted with ballots (scalar only).
__device__ __forceinline__ uint32_t fq_count(uint32_t m) {
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < FQ_R; ++k) n += __popcll(__ballot((m >> k) & 1u));
  return n;
}

// Adds the signed integer S * 2^p (p = bit position above limb 0's least significant bit) to a record's limbs.
__device__ __forceinline__ void fq_add_scaled(unsigned long long* limbs, int n_limbs, int64_t S, int p) {
  if (S == 0) return;
  const bool neg = S < 0;
  const unsigned __int128 u = static_cast<unsigned __int128>(neg ? 0ull - static_cast<uint64_t>(S)
                                                                  : static_cast<uint64_t>(S))
                              << (p & 31);
  const int i = p >> 5;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int64_t piece = static_cast<int64_t>(static_cast<uint32_t>(u >> (32 * q)));
    if (piece && i + q < n_limbs) atomicAdd(limbs + i + q, static_cast<unsigned long long>(neg ? -piece : piece));
  }
}

// One step of a wave: the FQ_R * WAVE rows [base, base + FQ_R * WAVE) of input chunk c (base < the chunk's size),
// folded into the workgroup's LDS records.
__device__ __forceinline__ void fused_step(const AggDesc& d, const FusedPlan& fp, unsigned long long* s_recf,
                                           uint32_t c, uint32_t base) {
  const uint32_t words = d.words;
  const int lane = __lane_id();
  const uint32_t H = d.n_gb;
  const uint32_t size = d.chunk_size[c];
  const uint64_t row0 = d.chunk_row_begin[c];
  {
    {
      uint32_t act = 0;
#pragma unroll
      for (int k = 0; k < FQ_R; ++k)
        if (base + k * WAVE + lane < size) act |= 1u << k;
      if (d.filter != nullptr && d.n_pos_groups == 0) act &= agg_filter_mask<FQ_R>(d, c, base + __lane_id());  // fused TableScan
      hy_row_id rid[FQ_R];
      bool uniform = true;
      uint32_t cc = 0;
      if (d.n_pos_groups) {
        const hy_row_id* pl = d.pos_lists[c];
#pragma unroll
        for (int k = 0; k < FQ_R; ++k)
          rid[k] = ((act >> k) & 1u) ? pl[base + k * WAVE + lane] : hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu};
        cc = __builtin_amdgcn_readfirstlane(rid[0].chunk_id);
        bool same = true;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k)
          if ((act >> k) & 1u) same = same && rid[k].chunk_id == cc;
        uniform = __ballot(!same) == 0ull && cc != 0xFFFFFFFFu;  // all-NULL RowIDs: per-lane path (skips them)
      }
      // group index of every row
      uint32_t g[FQ_R];
#pragma unroll
      for (int k = 0; k < FQ_R; ++k) g[k] = 0;
      for (uint32_t j = 0; j < H; ++j) {
        const AggCol& col = d.cols[d.gb[j]];
        uint32_t v[FQ_R];
        const uint32_t ok = fq_load(col, c, base, act, uniform, cc, rid, v);
        bool bad = false;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) {
          uint32_t code = col.domain;
          if ((ok >> k) & 1u) {
            code = v[k];
            if (code >= col.domain) {
              bad = true;
              code = col.domain;
            }
          }
          g[k] += code * col.stride;
        }
        if (bad) atomicOr(d.error, 2u);
      }
      // slots: plain columns loaded once, expressions evaluated from them
      uint32_t vals[FQ_SLOTS][FQ_R];
      uint32_t okm[FQ_SLOTS];
#pragma unroll
      for (int s = 0; s < FQ_SLOTS; ++s) {
        okm[s] = 0;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) vals[s][k] = 0;
      }
      for (int s = 0; s < fp.n_slots; ++s) {  // one copy of the load code; the result goes in by selection
        if (fp.slot_col[s] < 0) continue;
        uint32_t v[FQ_R];
        const uint32_t ok = fq_load(d.cols[fp.slot_col[s]], c, base, act, uniform, cc, rid, v);
#pragma unroll
        for (int j = 0; j < FQ_SLOTS; ++j)
          if (j == s) {
            okm[j] = ok;
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) vals[j][k] = v[k];
          }
      }
      for (int s = 0; s < fp.n_slots; ++s) {  // expressions: evaluated op by op for the step's FQ_R rows at once
        if (fp.slot_prog[s] < 0) continue;
        const FqOp* prog = fp.progs + fp.slot_prog[s];
        const int n_ops = fp.slot_nodes[s];
        uint32_t sv[FQ_DEPTH][FQ_R];
        uint32_t sn[FQ_DEPTH];  // NULL mask (bit k) of each stack entry
#pragma unroll
        for (int j = 0; j < FQ_DEPTH; ++j) {
          sn[j] = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) sv[j][k] = 0;
        }
        int sp = 0;
        for (int i = 0; i < n_ops; ++i) {
          const FqOp op = prog[i];
          uint32_t r[FQ_R];
          uint32_t rn = 0;
          if (op.kind == HY_EXPR_COLUMN) {
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) r[k] = fq_pick(vals, op.arg, k);
            rn = ~fq_pick_mask(okm, op.arg) & ((1u << FQ_R) - 1);
          } else if (op.kind == HY_EXPR_VALUE) {
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) r[k] = op.lit;
            rn = op.arg ? (1u << FQ_R) - 1 : 0u;
          } else {
            uint32_t a[FQ_R], b[FQ_R];
            uint32_t an = 0, bn = 0;
#pragma unroll
            for (int j = 0; j < FQ_DEPTH; ++j) {
              if (j == sp - 2) {
                an = sn[j];
#pragma unroll
                for (int k = 0; k < FQ_R; ++k) a[k] = sv[j][k];
              }
              if (j == sp - 1) {
                bn = sn[j];
#pragma unroll
                for (int k = 0; k < FQ_R; ++k) b[k] = sv[j][k];
              }
            }
            sp -= 2;
            rn = an | bn;
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) {
              r[k] = 0;
              if ((rn >> k) & 1u) continue;
              if (op.calc == HY_TYPE_FLOAT) {
                const float x = (op.arg & 1) ? static_cast<float>(static_cast<int32_t>(a[k])) : __uint_as_float(a[k]);
                const float y = (op.arg & 2) ? static_cast<float>(static_cast<int32_t>(b[k])) : __uint_as_float(b[k]);
                float z = 0.f;
                switch (op.kind) {
                  case HY_EXPR_ADD: z = x + y; break;
                  case HY_EXPR_SUB: z = x - y; break;
                  case HY_EXPR_MUL: z = x * y; break;
                  case HY_EXPR_DIV:
                    if (y == 0.f) rn |= 1u << k;
                    else z = x / y;
                    break;
                  default:
                    if (y == 0.f) rn |= 1u << k;
                    else z = fmodf(x, y);
                    break;
                }
                r[k] = __float_as_uint(z);
              } else {
                const int32_t x = static_cast<int32_t>(a[k]), y = static_cast<int32_t>(b[k]);
                int32_t z = 0;
                switch (op.kind) {  // two's complement wrap like the reference's int functors
                  case HY_EXPR_ADD: z = static_cast<int32_t>(static_cast<uint32_t>(x) + static_cast<uint32_t>(y)); break;
                  case HY_EXPR_SUB: z = static_cast<int32_t>(static_cast<uint32_t>(x) - static_cast<uint32_t>(y)); break;
                  case HY_EXPR_MUL: z = static_cast<int32_t>(static_cast<uint32_t>(x) * static_cast<uint32_t>(y)); break;
                  case HY_EXPR_DIV:
                    if (y == 0) rn |= 1u << k;
                    else z = x / y;
                    break;
                  default:
                    if (y == 0) rn |= 1u << k;
                    else z = x % y;
                    break;
                }
                r[k] = static_cast<uint32_t>(z);
              }
            }
          }
#pragma unroll
          for (int j = 0; j < FQ_DEPTH; ++j)
            if (j == sp) {
              sn[j] = rn;
#pragma unroll
              for (int k = 0; k < FQ_R; ++k) sv[j][k] = r[k];
            }
          ++sp;
        }
#pragma unroll
        for (int j = 0; j < FQ_SLOTS; ++j)
          if (j == s) {
            okm[j] = act & ~sn[0];
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) vals[j][k] = sv[0][k];
          }
      }
      // groups present in the step
      uint64_t mine = 0;
#pragma unroll
      for (int k = 0; k < FQ_R; ++k)
        if ((act >> k) & 1u) mine |= 1ull << g[k];
      const uint64_t groups = wave_or64(mine);
      for (uint64_t pg = groups; pg;) {  // header words, from ballots: row k * 64 + lane of the step
        const uint32_t gg = static_cast<uint32_t>(__builtin_ctzll(pg));
        pg &= pg - 1;
        uint32_t rows = 0;
        uint64_t first = ~0ull, last = 0;
#pragma unroll
        for (int k = 0; k < FQ_R; ++k) {
          const uint64_t m = __ballot(((act >> k) & 1u) && g[k] == gg);
          if (m) {
            rows += __popcll(m);
            const uint64_t r0 = row0 + base + k * WAVE;
            first = min(first, r0 + __builtin_ctzll(m));
            last = max(last, r0 + 63 - __builtin_clzll(m));
          }
        }
        if (lane == 0) {
          unsigned long long* rec = s_recf + gg * words;
          atomicAdd(rec + H + AGG_HDR_ROWS, static_cast<unsigned long long>(rows));
          atomicMin(rec + H + AGG_HDR_FIRST, static_cast<unsigned long long>(first));
          atomicMax(rec + H + AGG_HDR_LAST, static_cast<unsigned long long>(last));
        }
      }
      for (uint32_t f = 0; f < d.n_fns; ++f) {
        const AggFn fn = d.fns[f];
        const int s = fp.fn_slot[f];
        if (s < 0) continue;  // COUNT(*) = rows
        uint32_t v[FQ_R];
        uint32_t ok = 0;
#pragma unroll
        for (int j = 0; j < FQ_SLOTS; ++j)
          if (j == s) {
            ok = okm[j];
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) v[k] = vals[j][k];
          }
        const int32_t type = fp.slot_type[s];
        const bool is_float = fn.limbs != 0;
        // per-row contributions (computed once, summed per group below)
        int64_t contrib[FQ_R];
        uint32_t rowwise = 0;  // float rows outside the step's window: exact pieces per row
        uint32_t special = 0;  // non-finite flags of row k at bits [4k, 4k + 3)
        int E = 0;
        if (is_float && (fn.function == HY_AGG_SUM || fn.function == HY_AGG_AVG)) {
          int em = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) {
            const uint32_t e = (v[k] >> 23) & 0xFFu;
            if (((ok >> k) & 1u) && e != 0xFFu) em = max(em, static_cast<int>(e == 0 ? 1 : e));
          }
          E = wave_max_i(em);
          const int wbase = max(E - 31, 1);
#pragma unroll
          for (int k = 0; k < FQ_R; ++k) {
            contrib[k] = 0;
            if (!((ok >> k) & 1u)) continue;
            const uint32_t b = v[k];
            const uint32_t e = (b >> 23) & 0xFFu;
            uint32_t m = b & 0x7FFFFFu;
            if (e == 0xFFu) {
              special |= (m ? 4u : ((b >> 31) ? 2u : 1u)) << (4 * k);
              continue;
            }
            if (e) m |= 0x800000u;
            const int ee = e == 0 ? 1 : static_cast<int>(e);
            if (m == 0) continue;
            if (ee < wbase || E > 230) {
              rowwise |= 1u << k;
              continue;
            }
            const int64_t mag = static_cast<int64_t>(static_cast<uint64_t>(m) << (ee - wbase));
            contrib[k] = (b >> 31) ? -mag : mag;
          }
        } else {
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            contrib[k] = ((ok >> k) & 1u) ? int_value(v[k], type) : 0;
        }
        for (uint64_t pg = groups; pg;) {
          const uint32_t gg = static_cast<uint32_t>(__builtin_ctzll(pg));
          pg &= pg - 1;
          uint32_t inm = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            if (((ok >> k) & 1u) && g[k] == gg) inm |= 1u << k;
          const uint32_t cnt = fq_count(inm);
          unsigned long long* rec = s_recf + gg * words;
          if (lane == 0 && cnt) atomicAdd(rec + fn.word, static_cast<unsigned long long>(cnt));
          if (cnt == 0 || fn.function == HY_AGG_COUNT) continue;
          if (fn.function == HY_AGG_MIN || fn.function == HY_AGG_MAX) {
            const bool is_min = fn.function == HY_AGG_MIN;
            uint64_t r = is_min ? ~0ull : 0ull;
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) {
              if ((inm >> k) & 1u) {
                const uint64_t ob = ordered_bits(v[k], type);
                r = is_min ? (ob < r ? ob : r) : (ob > r ? ob : r);
              }
            }
            r = is_min ? fq_wave_ext<false>(r, ~0ull) : fq_wave_ext<true>(r, 0ull);
            if (lane == 0) {
              if (is_min)
                atomicMin(rec + fn.word + 1, static_cast<unsigned long long>(r));
              else
                atomicMax(rec + fn.word + 1, static_cast<unsigned long long>(r));
            }
            continue;
          }
          int64_t sum = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            if (((inm >> k) & 1u) && !((rowwise >> k) & 1u)) sum += contrib[k];
          sum = static_cast<int64_t>(fq_wave_sum(static_cast<uint64_t>(sum)));
          if (!is_float) {
            if (lane == 0 && sum) atomicAdd(rec + fn.word + 1, static_cast<unsigned long long>(sum));
            continue;
          }
          uint32_t spg = 0;
#pragma unroll
          for (int k = 0; k < FQ_R; ++k)
            if ((inm >> k) & 1u) spg |= (special >> (4 * k)) & 7u;
          const uint32_t sp = __ballot(spg != 0) ? static_cast<uint32_t>(wave_or64(static_cast<uint64_t>(spg))) : 0u;
          if (lane == 0) {
            if (sp) atomicOr(rec + fn.word + 1, static_cast<unsigned long long>(sp));
            // the window's unit is 2^(wbase - 150) = limb 0's unit (2^-149) times 2^(wbase - 1)
            fq_add_scaled(rec + fn.word + 2, fn.limbs, sum, max(E - 31, 1) - 1);
          }
          const uint32_t rw = inm & rowwise;
          if (rw) {
#pragma unroll
            for (int k = 0; k < FQ_R; ++k) {
              if (!((rw >> k) & 1u)) continue;
              int i0 = 0;
              int64_t part[3] = {0, 0, 0};
              uint32_t spc = 0;
              const int np = float_parts(v[k], HY_TYPE_FLOAT, &i0, part, &spc);
              for (int q = 0; q < np; ++q)
                if (part[q]) atomicAdd(rec + fn.word + 2 + i0 + q, static_cast<unsigned long long>(part[q]));
            }
          }
        }
      }
    }
  }
}

// Step id of the deferred-step lists (agg_dense_lanes): tile * 16 + wave * 4 + step of the wave's span.
constexpr int FQ_STEPS_PER_TILE = (AGG_THREADS / WAVE) * (AGG_ITEMS / FQ_R);

// Every step of the input (steps == nullptr), or only the n_steps[0] steps listed in `steps` (the ones
// agg_dense_lanes deferred), spread over the grid's waves.
__global__ __launch_bounds__(AGG_THREADS) void agg_dense_fused(AggDesc d, FusedPlan fp, uint32_t n_groups,
                                                              unsigned long long* __restrict__ records,
                                                              const uint32_t* __restrict__ steps,
                                                              const uint32_t* __restrict__ n_steps) {
  extern __shared__ unsigned long long s_recf[];
  const uint32_t words = d.words;
  const uint32_t n_words = n_groups * words;
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) s_recf[i] = word_init(d.word_op[i % words]);
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  if (steps == nullptr) {
    for (uint64_t tile = blockIdx.x; tile < d.n_tiles; tile += gridDim.x) {
      const uint32_t c = agg_tile_chunk(d, tile);
      const uint32_t size = d.chunk_size[c];
      const uint32_t span = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE + w * AGG_WAVE_SPAN;
      for (int h = 0; h < AGG_ITEMS / FQ_R; ++h) {
        const uint32_t base = span + h * FQ_R * WAVE;
        if (base >= size) break;  // wave-uniform
        fused_step(d, fp, s_recf, c, base);
      }
    }
  } else {
    const uint32_t n = *n_steps;
    const uint32_t waves = gridDim.x * (AGG_THREADS / WAVE);
    for (uint32_t i = blockIdx.x * (AGG_THREADS / WAVE) + w; i < n; i += waves) {
      const uint32_t id = steps[i];
      const uint64_t tile = id / FQ_STEPS_PER_TILE;
      const uint32_t r = id % FQ_STEPS_PER_TILE;
      const uint32_t c = agg_tile_chunk(d, tile);
      const uint32_t base = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * AGG_TILE +
                            (r / (AGG_ITEMS / FQ_R)) * AGG_WAVE_SPAN + (r % (AGG_ITEMS / FQ_R)) * FQ_R * WAVE;
      fused_step(d, fp, s_recf, c, base);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n_words; i += AGG_THREADS) {
    const int32_t op = d.word_op[i % words];
    word_apply(records + i, op, s_recf[i]);
  }
}

}  // namespace hyk
