// Projection kernel for gfx950: evaluates arithmetic expressions (postfix programs of hy_expr_node) per input row and
// writes their result columns (values + NULL flags) for all chunks of the input in one launch.
//
// Reference: Projection::_on_execute (src/lib/operators/projection.cpp:39-87) evaluates every expression per chunk
// with ExpressionEvaluator; arithmetic is Functor<std::common_type_t<A, B>>(a, b) assigned to the expression's
// data type (expression_functors.hpp:104-180), NULL if an operand is NULL (_evaluate_default_null_logic,
// expression_evaluator.cpp:795-830) and, for / and %, if the divisor is 0.
//
// Layout: one tile of the input's global rows per workgroup (tiles cross chunk boundaries, so many small chunks such
// as a join output's partitions keep every lane busy), `items` rows per lane (row = tile base + k * 256 + thread; up
// to 16, fewer for small inputs so that the grid still covers the CUs), so the result store is coalesced per wave. Columns are read through the Aggregate's column model
// (value / dictionary chunks, or referenced chunks through PosList groups). The program is interpreted with a
// per-lane value stack; its control flow is uniform (the same program for every row), so there is no divergence.
// Roofline: HBM (the read column bytes + result bytes per row).
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace hyk {

struct ExprProgram {
  hy_expr_node nodes[HY_EXPR_MAX_NODES];
  uint32_t n_nodes;
  int32_t out_type;
};

// Value bits of `bits` (type `from`) converted to type `to` (C++ arithmetic conversions).
__device__ __forceinline__ uint64_t expr_convert(uint64_t bits, int32_t from, int32_t to) {
  if (from == to) return bits;
  int64_t i = 0;
  double dv = 0;
  float fv = 0;
  bool is_int = false, is_float = false;
  switch (from) {
    case HY_TYPE_INT32:
      i = static_cast<int32_t>(static_cast<uint32_t>(bits));
      is_int = true;
      break;
    case HY_TYPE_INT64:
      i = static_cast<int64_t>(bits);
      is_int = true;
      break;
    case HY_TYPE_FLOAT: {
      const uint32_t b = static_cast<uint32_t>(bits);
      __builtin_memcpy(&fv, &b, 4);
      is_float = true;
      break;
    }
    default:
      __builtin_memcpy(&dv, &bits, 8);
      break;
  }
  switch (to) {
    case HY_TYPE_INT32: {
      const int32_t v = is_int ? static_cast<int32_t>(i) : is_float ? static_cast<int32_t>(fv) : static_cast<int32_t>(dv);
      return static_cast<uint32_t>(v);
    }
    case HY_TYPE_INT64: {
      const int64_t v = is_int ? i : is_float ? static_cast<int64_t>(fv) : static_cast<int64_t>(dv);
      return static_cast<uint64_t>(v);
    }
    case HY_TYPE_FLOAT: {
      const float v = is_int ? static_cast<float>(i) : is_float ? fv : static_cast<float>(dv);
      uint32_t b;
      __builtin_memcpy(&b, &v, 4);
      return b;
    }
    default: {
      const double v = is_int ? static_cast<double>(i) : is_float ? static_cast<double>(fv) : dv;
      uint64_t b;
      __builtin_memcpy(&b, &v, 8);
      return b;
    }
  }
}

template <typename T>
__device__ __forceinline__ T expr_as(uint64_t bits) {
  T v;
  if constexpr (sizeof(T) == 4) {
    const uint32_t b = static_cast<uint32_t>(bits);
    __builtin_memcpy(&v, &b, 4);
  } else {
    __builtin_memcpy(&v, &bits, 8);
  }
  return v;
}

template <typename T>
__device__ __forceinline__ uint64_t expr_bits(T v) {
  if constexpr (sizeof(T) == 4) {
    uint32_t b;
    __builtin_memcpy(&b, &v, 4);
    return b;
  } else {
    uint64_t b;
    __builtin_memcpy(&b, &v, 8);
    return b;
  }
}

template <typename T>
__device__ __forceinline__ uint64_t expr_arith_t(int32_t op, uint64_t a_bits, uint64_t b_bits, bool* null) {
  const T a = expr_as<T>(a_bits), b = expr_as<T>(b_bits);
  T r{};
  switch (op) {
    case HY_EXPR_ADD:
      r = a + b;
      break;
    case HY_EXPR_SUB:
      r = a - b;
      break;
    case HY_EXPR_MUL:
      r = a * b;
      break;
    case HY_EXPR_DIV:
      if (b == T(0)) *null = true;
      else r = a / b;
      break;
    default:  // HY_EXPR_MOD: % for integrals, fmod for floats
      if (b == T(0)) {
        *null = true;
      } else {
        if constexpr (std::is_integral_v<T>)
          r = a % b;
        else
          r = fmod(a, b);
      }
      break;
  }
  return expr_bits<T>(r);
}

__device__ __forceinline__ uint64_t expr_arith(int32_t op, int32_t calc, uint64_t a, uint64_t b, bool* null) {
  switch (calc) {
    case HY_TYPE_INT32:
      return expr_arith_t<int32_t>(op, a, b, null);
    case HY_TYPE_INT64:
      return expr_arith_t<int64_t>(op, a, b, null);
    case HY_TYPE_FLOAT:
      return expr_arith_t<float>(op, a, b, null);
    default:
      return expr_arith_t<double>(op, a, b, null);
  }
}


// One output column of a projection launch: the program (device copy) and where its values / NULL flags go.
struct ProjOut {
  const ExprProgram* prog;
  void* values;
  uint8_t* nulls;  // may be null
};

// Every program of the launch over every row (hy_projection_multi: the reference's Projection evaluates all its
// expressions per chunk, projection.cpp:52-85): the row's chunk (LDS window), its RowIDs and the programs' column
// reads are shared by the programs instead of repeated per launch.
__global__ __launch_bounds__(AGG_THREADS) void projection_kernel(AggDesc d, const ProjOut* __restrict__ outs,
                                                                uint32_t n_outs, uint64_t total_rows, uint32_t items) {
  __shared__ ChunkWinLds s_win;
  const uint64_t tile_row0 = static_cast<uint64_t>(blockIdx.x) * AGG_THREADS * items;
  const ChunkWin win =
      chunk_window(d, tile_row0, min(total_rows, tile_row0 + static_cast<uint64_t>(AGG_THREADS) * items), s_win);
#pragma unroll 1
  for (uint32_t k = 0; k < items; ++k) {
    const uint64_t row = tile_row0 + static_cast<uint64_t>(k) * AGG_THREADS + threadIdx.x;
    if (row >= total_rows) break;
    uint32_t off;
    const uint32_t c = win_chunk(d, win, s_win, tile_row0, row, &off);
    RowRefs refs;
    if (d.n_pos_groups) load_refs(d, c, off, &refs);
#pragma unroll 1
    for (uint32_t o = 0; o < n_outs; ++o) {
      const ProjOut po = outs[o];
      const ExprProgram& prog = *po.prog;
      // value stack in registers: every slot access is an unrolled compare against the (uniform) stack pointer, so
      // the arrays are never indexed dynamically (which would place them in scratch memory)
      uint64_t val[HY_EXPR_MAX_DEPTH];
      bool nul[HY_EXPR_MAX_DEPTH];
      int32_t typ[HY_EXPR_MAX_DEPTH];
      auto push = [&](int sp, uint64_t v, bool n, int32_t t) {
#pragma unroll
        for (int j = 0; j < HY_EXPR_MAX_DEPTH; ++j)
          if (j == sp) {
            val[j] = v;
            nul[j] = n;
            typ[j] = t;
          }
      };
      auto peek = [&](int sp, uint64_t* v, bool* n, int32_t* t) {
#pragma unroll
        for (int j = 0; j < HY_EXPR_MAX_DEPTH; ++j)
          if (j == sp) {
            *v = val[j];
            *n = nul[j];
            *t = typ[j];
          }
      };
      int sp = 0;
      const uint32_t n_nodes = prog.n_nodes;
      for (uint32_t i = 0; i < n_nodes; ++i) {
        const hy_expr_node nd = prog.nodes[i];
        if (nd.kind == HY_EXPR_COLUMN) {
          uint64_t bits = 0;
          const bool ok = read_col(d, d.cols[nd.column], c, off, refs, &bits);
          push(sp++, bits, !ok, nd.type);
        } else if (nd.kind == HY_EXPR_VALUE) {
          push(sp++, nd.value, nd.type == 0, nd.type);
        } else {
          uint64_t a = 0, b = 0;
          bool na = true, nb = true;
          int32_t ta = 0, tb = 0;
          peek(sp - 1, &b, &nb, &tb);
          peek(sp - 2, &a, &na, &ta);
          sp -= 2;
          bool null = na || nb || ta == 0 || tb == 0;
          uint64_t r = 0;
          if (!null) {
            r = expr_arith(nd.kind, nd.calc_type, expr_convert(a, ta, nd.calc_type), expr_convert(b, tb, nd.calc_type),
                           &null);
            r = expr_convert(r, nd.calc_type, nd.type);
          }
          push(sp++, null ? 0 : r, null, nd.type);
        }
      }
      const uint64_t r = val[0];
      if (is_wide(prog.out_type))
        static_cast<uint64_t*>(po.values)[row] = r;
      else
        static_cast<uint32_t*>(po.values)[row] = static_cast<uint32_t>(r);
      if (po.nulls != nullptr) po.nulls[row] = nul[0] ? 1 : 0;
    }
  }
}

}  // namespace hyk
