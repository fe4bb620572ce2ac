// C-ABI implementation of the Aggregate entry points (include/hyrise_amd.h): record layout, workspace carving,
// dense / hash path selection and the launches of kernels/aggregate.hip. Host helpers round exact limb sums.
#include <hip/hip_runtime.h>

#include <unordered_map>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "capi_common.hpp"
#include "../kernels/aggregate.hip"
#include "../kernels/projection.hip"
#include "../kernels/aggregate_fused.hip"
#include "../kernels/aggregate_lanes.hip"
#include "../kernels/aggregate_vec.hip"
#include "../kernels/aggregate_stream.hip"
#include "agg_jit.hpp"

using namespace hyc;

namespace {

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Validates a postfix program over the plain (non-expression) columns of `in` and copies it into *out.
hy_status validate_program(const hy_agg_input* in, const hy_expr_node* program, uint32_t n_nodes,
                           hyk::ExprProgram* out, int* max_depth = nullptr) {
  if (!program || n_nodes == 0 || n_nodes > HY_EXPR_MAX_NODES) return fail(HY_ERR_INVALID_ARGUMENT, "program size");
  *out = hyk::ExprProgram{};
  int depth = 0, deepest = 0;
  for (uint32_t i = 0; i < n_nodes; ++i) {
    const hy_expr_node& nd = program[i];
    out->nodes[i] = nd;
    const bool typed = nd.type >= HY_TYPE_INT32 && nd.type <= HY_TYPE_DOUBLE;
    switch (nd.kind) {
      case HY_EXPR_COLUMN:
        if (nd.column < 0 || nd.column >= static_cast<int32_t>(in->n_columns))
          return fail(HY_ERR_INVALID_ARGUMENT, "expression column");
        if (in->columns[nd.column].n_nodes) return fail(HY_ERR_INVALID_ARGUMENT, "expression over an expression");
        if (nd.type != in->columns[nd.column].value_type) return fail(HY_ERR_INVALID_ARGUMENT, "column node type");
        ++depth;
        break;
      case HY_EXPR_VALUE:
        if (!typed && nd.type != 0) return fail(HY_ERR_INVALID_ARGUMENT, "literal type");
        ++depth;
        break;
      case HY_EXPR_ADD:
      case HY_EXPR_SUB:
      case HY_EXPR_MUL:
      case HY_EXPR_DIV:
      case HY_EXPR_MOD:
        if (depth < 2) return fail(HY_ERR_INVALID_ARGUMENT, "expression stack underflow");
        if (!typed || nd.calc_type < HY_TYPE_INT32 || nd.calc_type > HY_TYPE_DOUBLE)
          return fail(HY_ERR_INVALID_ARGUMENT, "arithmetic node types");
        --depth;
        break;
      default:
        return fail(HY_ERR_INVALID_ARGUMENT, "expression node kind");
    }
    if (depth > HY_EXPR_MAX_DEPTH) return fail(HY_ERR_UNSUPPORTED, "expression deeper than HY_EXPR_MAX_DEPTH");
    deepest = std::max(deepest, depth);
  }
  if (depth != 1) return fail(HY_ERR_INVALID_ARGUMENT, "program does not leave one value");
  out->n_nodes = n_nodes;
  out->out_type = program[n_nodes - 1].type;
  if (out->out_type == 0) return fail(HY_ERR_UNSUPPORTED, "an all-NULL expression has no column type");
  if (max_depth) *max_depth = deepest;
  return HY_OK;
}

inline bool four_bytes(int32_t t) { return t == HY_TYPE_INT32 || t == HY_TYPE_FLOAT; }

struct AggPlan {
  hyk::AggDesc d{};
  std::vector<int32_t> word_op;
  hy_agg_layout layout{};
  uint64_t rows = 0;
  uint64_t n_tiles = 0;
  uint32_t dense_groups = 0;  // > 0: dense path
  uint64_t cap = 0, dcap = 0;
  uint64_t max_groups = 0;
  bool distinct = false;
  std::vector<uint32_t> expr_cols;         // input columns that are expressions
  std::vector<hyk::ExprProgram> exprs;     // their programs (same order)
  bool fused = false;                      // agg_dense_fused (expressions evaluated in the kernel)
  bool materialize = false;                // else: expression columns materialised first (projection kernel)
  hyk::FusedPlan fp{};
  std::vector<hyk::FqOp> fused_nodes;      // fp.progs on the host
  bool lanes = false;                      // agg_dense_lanes first, agg_dense_fused over the steps it defers
  hyk::LaneTables lt{};                    // agg_dense_lanes' tables (copied to the workspace)
  std::vector<hyk::LnTerm> lane_terms;     // lp.terms on the host
  std::vector<int32_t> lane_cols;          // input column of each loaded column
  bool lanes_vec = false;                  // agg_dense_lanes<.., VEC>: data input, 16-byte aligned column chunks
  bool dense_vec = false;                  // agg_dense_vec instead (its preconditions hold; the default then)
  bool dense_stream = false;               // agg_dense_stream instead (its preconditions hold; the default then)
  hyk::StreamPlan stream_plan{};           // its stage layout and FMA-form chains
  bool dense_jit = false;                  // the stream plan compiled into its own kernel (hyrise_amd_agg_jit.cpp)
  hyjit::Shape jit_shape{};
};

// agg_dense_fused applies: the dense path; at most one PosList group; int32 group-by columns; every aggregate over a
// 4-byte plain column or a 4-byte expression of 4-byte plain columns (stack <= FQ_DEPTH); <= FQ_SLOTS slots; no
// COUNT(DISTINCT). HY_AGG_FUSED=0 disables it (tests compare the paths).
void plan_fused(const hy_agg_input* in, const hy_agg_params* p, AggPlan* plan) {
  if (const char* e = std::getenv("HY_AGG_FUSED"))
    if (std::atoi(e) == 0) return;
  if (!plan->dense_groups || plan->distinct || in->n_pos_groups > 1 || p->n_groupby > hyk::FQ_MAX_GB) return;
  for (uint32_t j = 0; j < p->n_groupby; ++j) {
    const auto& c = in->columns[p->groupby[j]];
    if (c.n_nodes || c.value_type != HY_TYPE_INT32) return;
  }
  auto& fp = plan->fp;
  fp = hyk::FusedPlan{};
  std::vector<int32_t> slot_of(in->n_columns, -1);
  auto plain_slot = [&](uint32_t col) -> int32_t {
    if (slot_of[col] >= 0) return slot_of[col];
    if (fp.n_slots >= hyk::FQ_SLOTS || !four_bytes(in->columns[col].value_type)) return -1;
    const int32_t sl = fp.n_slots++;
    fp.slot_col[sl] = static_cast<int32_t>(col);
    fp.slot_prog[sl] = -1;
    fp.slot_type[sl] = in->columns[col].value_type;
    return slot_of[col] = sl;
  };
  std::vector<int32_t> expr_slot(in->n_columns, -1);
  for (uint32_t a = 0; a < p->n_aggregates; ++a) {
    const auto& def = p->aggregates[a];
    fp.fn_slot[a] = -1;
    if (def.column < 0) continue;
    const auto& c = in->columns[def.column];
    if (!four_bytes(c.value_type)) return;
    if (!c.n_nodes) {
      if ((fp.fn_slot[a] = plain_slot(def.column)) < 0) return;
      continue;
    }
    if (expr_slot[def.column] < 0) {
      int depth = 0;
      hyk::ExprProgram prog;
      if (validate_program(in, c.program, c.n_nodes, &prog, &depth) != HY_OK || depth > hyk::FQ_DEPTH) return;
      // compile to FqOps: every value 4 bytes; the stack's types are tracked here, so the kernel only converts the
      // operands flagged per op
      std::vector<hyk::FqOp> nodes;
      std::vector<int32_t> types;  // 0 = NULL literal
      for (uint32_t i = 0; i < c.n_nodes; ++i) {
        const hy_expr_node& nd = c.program[i];
        hyk::FqOp op{nd.kind, 0, 0, 0};
        if (nd.kind == HY_EXPR_COLUMN) {
          if (!four_bytes(nd.type) || (op.arg = plain_slot(static_cast<uint32_t>(nd.column))) < 0) return;
          types.push_back(nd.type);
        } else if (nd.kind == HY_EXPR_VALUE) {
          if (nd.type != 0 && !four_bytes(nd.type)) return;
          op.arg = nd.type == 0 ? 1 : 0;
          op.lit = static_cast<uint32_t>(nd.value);
          types.push_back(nd.type);
        } else {
          if (!four_bytes(nd.calc_type) || nd.type != nd.calc_type) return;
          const int32_t tb = types.back();
          types.pop_back();
          const int32_t ta = types.back();
          types.pop_back();
          op.calc = nd.calc_type;
          if (nd.calc_type == HY_TYPE_FLOAT) op.arg = (ta == HY_TYPE_INT32 ? 1 : 0) | (tb == HY_TYPE_INT32 ? 2 : 0);
          else if (ta == HY_TYPE_FLOAT || tb == HY_TYPE_FLOAT) return;  // float operand of an int32 op
          types.push_back(nd.type);
        }
        nodes.push_back(op);
      }
      if (fp.n_slots >= hyk::FQ_SLOTS) return;
      const int32_t sl = fp.n_slots++;
      fp.slot_col[sl] = -1;
      fp.slot_prog[sl] = static_cast<int32_t>(plan->fused_nodes.size());
      fp.slot_nodes[sl] = static_cast<int32_t>(nodes.size());
      fp.slot_type[sl] = c.value_type;
      plan->fused_nodes.insert(plan->fused_nodes.end(), nodes.begin(), nodes.end());
      expr_slot[def.column] = sl;
    }
    fp.fn_slot[a] = expr_slot[def.column];
  }
  for (uint32_t a = 0; a < p->n_aggregates; ++a)  // float sums use the float limb layout only
    if (plan->d.fns[a].limbs && plan->d.fns[a].limbs != hyk::FLOAT_LIMBS) return;
  plan->fused = true;
}

// agg_dense_stream (aggregate_stream.hip) takes what agg_dense_vec takes when, in addition, every DICT chunk of a
// loaded column has <= ST_DICT_MAX entries (decoded through the wave's LDS tables), at most ST_DCOLS loaded columns have
// DICT chunks, at most ST_VALS loaded columns besides the group-by columns, the filter (if any) is a dictionary id range
// on every chunk, the tile ids fit the step numbering and one step's column bytes (256 rows x each column's widest
// chunk width) fit the stage, float sums are + - * chains (compiled to FMA-form terms), int32 sums plain columns and
// the group codes < ST_CODES. HY_AGG_STREAM=0: agg_dense_vec.
void plan_stream(const hy_agg_input* in, AggPlan* plan) {
  plan->dense_stream = false;
  if (!plan->dense_vec) return;
  if (const char* e = std::getenv("HY_AGG_STREAM"))
    if (std::atoi(e) == 0) return;
  if (plan->n_tiles >= (1ull << 28)) return;
  if (plan->lt.n_load - static_cast<int32_t>(plan->d.n_gb) > hyk::ST_VALS) return;
  hyk::StreamPlan L{};
  uint32_t off = 0, slots = 0;
  for (size_t li = 0; li < plan->lane_cols.size(); ++li) {
    const auto& col = in->columns[plan->lane_cols[li]];
    uint32_t width = 1;
    bool dict = false;
    for (uint32_t k = 0; k < col.n_chunks; ++k) {
      const auto& ch = col.chunks[k];
      if (ch.size == 0) continue;
      if (ch.kind == HY_COL_DICT) {
        if (ch.dictionary_size > hyk::ST_DICT_MAX) return;
        dict = true;
        width = std::max<uint32_t>(width, static_cast<uint32_t>(ch.vid_width));
      } else {
        width = 4;
      }
    }
    L.col_off[li] = off;
    off += 256u * width;
    L.dict_slot[li] = hyk::ST_NO_SLOT;
    if (dict) {
      if (slots >= static_cast<uint32_t>(hyk::ST_DCOLS)) return;
      L.dict_slot[li] = slots++;
    }
  }
  if (in->filter) {
    uint32_t width = 1;
    for (uint32_t k = 0; k < in->n_chunks; ++k) {
      const auto& f = in->filter[k];
      if (f.column.size == 0) continue;
      if (f.column.kind != HY_COL_DICT) return;
      switch (f.op) {
        case HY_OP_EQ: case HY_OP_NE: case HY_OP_LT: case HY_OP_LE: case HY_OP_GT: case HY_OP_GE:
        case HY_OP_ALL: case HY_OP_IS_NOT_NULL: case HY_OP_NONE:
          break;
        default:
          return;  // no id-range form (VID_SET, ...)
      }
      width = std::max<uint32_t>(width, static_cast<uint32_t>(f.column.vid_width));
    }
    L.filt_off = off;
    off += 256u * width;
  }
  if (off > static_cast<uint32_t>(hyk::ST_STAGE)) return;
  L.stage_bytes = off;
  L.n_dslots = slots;
  // the sums: float chains as FMA-form terms (hyk::StreamTerm), int32 sums of plain columns, COUNT-only inputs
  const auto& lt = plan->lt;
  for (int32_t q = 0; q < lt.n_sums; ++q) {
    L.sum_first[q] = lt.sum_first[q];
    L.sum_len[q] = lt.sum_len[q];
    if (lt.sum_kind[q] == hyk::LN_SUM_CHECK) {
      L.sum_kind[q] = hyk::ST_SUM_NONE;
      continue;
    }
    if (lt.sum_kind[q] == hyk::LN_SUM_INT) {
      const auto& t = plan->lane_terms[lt.sum_first[q]];
      if (lt.sum_len[q] != 1 || t.kind != hyk::LN_TERM_COL || t.cvt) return;  // int32 chains: agg_dense_vec
      L.sum_kind[q] = hyk::ST_SUM_INT;
      L.terms[lt.sum_first[q]] = hyk::StreamTerm{1.f, -0.f, t.col, hyk::ST_SET};
      continue;
    }
    L.sum_kind[q] = hyk::ST_SUM_FLOAT;
    for (int32_t i = 0; i < lt.sum_len[q]; ++i) {
      const hyk::LnTerm& t = plan->lane_terms[lt.sum_first[q] + i];
      float lit;
      std::memcpy(&lit, &t.lit, 4);
      hyk::StreamTerm o{1.f, -0.f, t.col, t.cvt ? hyk::ST_CVT : 0};
      // term = fma(x, a, b): one rounding, as x, lit + x, lit - x, lit * x, x - lit, x * lit compute
      switch (t.kind) {
        case hyk::LN_TERM_COL:
          break;
        case hyk::LN_TERM_LIT:
          o = hyk::StreamTerm{0.f, lit, 0, hyk::ST_LIT};
          break;
        case hyk::LN_TERM_LIT_COL:
        case hyk::LN_TERM_COL_LIT:
          if (t.op == HY_EXPR_ADD) {
            o.a = 1.f, o.b = lit;
          } else if (t.op == HY_EXPR_SUB) {
            if (t.kind == hyk::LN_TERM_LIT_COL) o.a = -1.f, o.b = lit;
            else o.a = 1.f, o.b = -lit;
          } else if (t.op == HY_EXPR_MUL) {
            o.a = lit, o.b = -0.f;
          } else {
            return;
          }
          break;
        default:
          return;
      }
      if (i > 0) {
        if (t.comb == HY_EXPR_ADD) o.flags |= hyk::ST_ADD;
        else if (t.comb == HY_EXPR_SUB) o.flags |= t.rev ? hyk::ST_RSUB : hyk::ST_SUB;
        else if (t.comb == HY_EXPR_MUL) o.flags |= hyk::ST_MUL;
        else return;
      }
      L.terms[lt.sum_first[q] + i] = o;
    }
  }
  if (plan->dense_groups > static_cast<uint32_t>(hyk::ST_CODES)) return;
  plan->stream_plan = L;
  plan->dense_stream = true;
  // the plan-compiled kernel (default; HY_AGG_JIT=0: agg_dense_stream) when every loaded column has one encoding and
  // width over all its chunks, and so has the filter
  const char* ej = std::getenv("HY_AGG_JIT");
  if (ej && std::atoi(ej) == 0) return;
  hyjit::Shape& sh = plan->jit_shape;
  sh = hyjit::Shape{};
  sh.n_gb = static_cast<int32_t>(plan->d.n_gb);
  sh.n_load = lt.n_load;
  sh.n_sums = lt.n_sums;
  sh.words = plan->d.words;
  if (sh.n_load > hyj::MAX_COLS || sh.n_sums > hyjit::MAX_SUMS || lt.n_cnt > hyjit::MAX_CNT) return;
  for (int32_t li = 0; li < sh.n_load; ++li) {
    const auto& col = in->columns[plan->lane_cols[li]];
    int kind = -1, width = 0;
    for (uint32_t k = 0; k < col.n_chunks; ++k) {
      const auto& ch = col.chunks[k];
      if (ch.size == 0) continue;
      const int kk = ch.kind == HY_COL_DICT ? 1 : 0;
      const int ww = kk ? ch.vid_width : 4;
      if ((kind >= 0 && kind != kk) || (width && width != ww)) return;
      kind = kk;
      width = ww;
    }
    sh.dict[li] = kind == 1;
    sh.width[li] = width ? width : 4;
    sh.col_off[li] = L.col_off[li];
    sh.dict_slot[li] = L.dict_slot[li];
    if (li < sh.n_gb) {
      sh.gb_domain[li] = lt.gb_domain[li];
      sh.gb_stride[li] = lt.gb_stride[li];
    }
  }
  if (in->filter) {
    sh.filtered = 1;
    for (uint32_t k = 0; k < in->n_chunks; ++k) {
      const auto& f = in->filter[k];
      if (f.column.size == 0) continue;
      if (sh.f_width && sh.f_width != f.column.vid_width) return;
      sh.f_width = f.column.vid_width;
    }
    if (!sh.f_width) sh.f_width = 1;
    sh.filt_off = L.filt_off;
  }
  sh.stage_bytes = L.stage_bytes;
  sh.n_dslots = L.n_dslots;
  for (int32_t q = 0; q < lt.n_sums; ++q) {
    sh.sum_kind[q] = L.sum_kind[q];
    sh.sum_first[q] = L.sum_first[q];
    sh.sum_len[q] = L.sum_len[q];
    sh.sum_nfn[q] = lt.sum_nfn[q];
    for (int32_t f = 0; f < lt.sum_nfn[q] && f < hyjit::MAX_FNS; ++f) sh.sum_word[q][f] = lt.sum_word[q][f];
    sh.sum_limbs[q] = lt.sum_limbs[q];
    for (int32_t t = 0; t < L.sum_len[q]; ++t) {
      const int32_t i = L.sum_first[q] + t;
      if (i >= hyjit::MAX_TERMS) return;
      sh.terms[i] = hyjit::Term{L.terms[i].a, L.terms[i].b, L.terms[i].col, L.terms[i].flags};
    }
  }
  sh.n_cnt = lt.n_cnt;
  for (int32_t f = 0; f < lt.n_cnt; ++f) sh.cnt_word[f] = lt.cnt_word[f];
  plan->dense_jit = true;
}


// agg_dense_lanes applies on top of agg_dense_fused: no MIN / MAX; every loaded column (group-by columns, columns
// of SUM / AVG / COUNT inputs and of their expressions) 4 bytes wide, read through the single PosList group (or
// directly for a data input), its chunks dictionary-encoded or value chunks (with or without NULL flags); a group-by
// column is not also summed; every SUM / AVG / COUNT input compiles to a chain (LnTerm) of + - *; <= LN_COLS columns, <= LN_SUMS
// inputs, <= LN_TERMS terms. HY_AGG_LANES=0 disables it (tests compare the paths).
void plan_lanes(const hy_agg_input* in, const hy_agg_params* p, AggPlan* plan) {
  if (!plan->fused) return;
  if (const char* e = std::getenv("HY_AGG_LANES"))
    if (std::atoi(e) == 0) return;
  auto& lp = plan->lt;
  lp = hyk::LaneTables{};
  auto& terms = plan->lane_terms;
  terms.clear();
  const int32_t H = static_cast<int32_t>(p->n_groupby);
  const int32_t want_pg = in->n_pos_groups ? 0 : -1;
  std::vector<int32_t> load_of(in->n_columns, -1);
  plan->lane_cols.clear();
  auto load = [&](int32_t col) -> int32_t {
    if (col < 0 || col >= static_cast<int32_t>(in->n_columns)) return -1;
    if (load_of[col] >= 0) return load_of[col];
    const auto& c = in->columns[col];
    if (c.n_nodes || !four_bytes(c.value_type) || c.pos_group != want_pg || lp.n_load >= hyk::LN_COLS) return -1;
    for (uint32_t k = 0; k < c.n_chunks; ++k) {
      const auto& ch = c.chunks[k];
      if (ch.kind == HY_COL_DICT && ch.vid_width != 1 && ch.vid_width != 2 && ch.vid_width != 4) return -1;
    }
    plan->lane_cols.push_back(col);
    return load_of[col] = lp.n_load++;
  };
  if (H > hyk::FQ_MAX_GB) return;
  for (int32_t j = 0; j < H; ++j) {
    if (load(p->groupby[j]) != j) return;
    lp.gb_domain[j] = plan->d.cols[p->groupby[j]].domain;
    lp.gb_stride[j] = plan->d.cols[p->groupby[j]].stride;
  }
  // an input's chain: postfix program -> terms (see hyk::LnTerm)
  struct Ent {
    int form;  // 0 column, 1 literal, 2 literal op column / column op literal, 3 chain
    hyk::LnTerm t;
    std::vector<hyk::LnTerm> chain;
    int32_t type;
  };
  auto term_col = [&](int32_t col, int32_t type, Ent* e) -> bool {
    const int32_t li = load(col);
    if (li < H) return false;  // not loadable, or a group-by column
    *e = Ent{0, hyk::LnTerm{hyk::LN_TERM_COL, 0, li, 0, 0, 0, 0, 0}, {}, type};
    return true;
  };
  auto compile = [&](uint32_t colidx, std::vector<hyk::LnTerm>* out, bool* is_float) -> bool {
    const auto& c = in->columns[colidx];
    Ent res;
    if (!c.n_nodes) {
      if (!term_col(static_cast<int32_t>(colidx), c.value_type, &res)) return false;
    } else {
      std::vector<Ent> st;
      for (uint32_t i = 0; i < c.n_nodes; ++i) {
        const hy_expr_node& nd = c.program[i];
        if (nd.kind == HY_EXPR_COLUMN) {
          Ent e;
          if (!term_col(nd.column, nd.type, &e)) return false;
          st.push_back(e);
          continue;
        }
        if (nd.kind == HY_EXPR_VALUE) {
          if (nd.type == 0) return false;  // NULL literal
          st.push_back(Ent{1, hyk::LnTerm{hyk::LN_TERM_LIT, 0, 0, static_cast<uint32_t>(nd.value), 0, 0, 0, 0}, {},
                           nd.type});
          continue;
        }
        if (st.size() < 2) return false;
        Ent b = st.back();
        st.pop_back();
        Ent a = st.back();
        st.pop_back();
        const int32_t calc = nd.calc_type;
        if (nd.kind != HY_EXPR_ADD && nd.kind != HY_EXPR_SUB && nd.kind != HY_EXPR_MUL) return false;  // / % -> fused
        auto conv = [&](Ent& e) -> bool {  // an int32 operand of a float operation converts (columns, literals)
          if (e.type == calc) return true;
          if (e.type != HY_TYPE_INT32 || calc != HY_TYPE_FLOAT) return false;
          if (e.form == 0) {
            e.t.cvt = 1;
          } else if (e.form == 1) {
            const float f = static_cast<float>(static_cast<int32_t>(e.t.lit));
            std::memcpy(&e.t.lit, &f, 4);
          } else {
            return false;
          }
          e.type = calc;
          return true;
        };
        if (!four_bytes(calc) || nd.type != calc || !conv(a) || !conv(b)) return false;
        Ent r;
        r.type = nd.type;
        if (a.form <= 1 && b.form <= 1) {
          if (a.form == 1 && b.form == 1) return false;  // literal op literal
          if (a.form == 0 && b.form == 0) {
            r.form = 3;
            b.t.comb = nd.kind;
            r.chain = {a.t, b.t};
          } else {
            r.form = 2;
            r.t = a.form == 0 ? hyk::LnTerm{hyk::LN_TERM_COL_LIT, nd.kind, a.t.col, b.t.lit, a.t.cvt, 0, 0, 0}
                              : hyk::LnTerm{hyk::LN_TERM_LIT_COL, nd.kind, b.t.col, a.t.lit, b.t.cvt, 0, 0, 0};
          }
        } else if (a.form == 3 && b.form == 3) {
          return false;
        } else if (a.form == 3) {
          r = a;
          b.t.comb = nd.kind;
          b.t.rev = 0;
          r.chain.push_back(b.t);
        } else if (b.form == 3) {
          r = b;
          a.t.comb = nd.kind;
          a.t.rev = 1;
          r.chain.push_back(a.t);
        } else {
          r.form = 3;
          b.t.comb = nd.kind;
          r.chain = {a.t, b.t};
        }
        r.type = nd.type;
        st.push_back(r);
      }
      if (st.size() != 1) return false;
      res = st.back();
    }
    *out = res.form == 3 ? res.chain : std::vector<hyk::LnTerm>{res.t};
    *is_float = res.type == HY_TYPE_FLOAT;
    return true;
  };
  std::vector<int32_t> sum_of(in->n_columns, -1);
  for (uint32_t a = 0; a < p->n_aggregates; ++a) {
    const auto& def = p->aggregates[a];
    if (def.column < 0) continue;  // COUNT(*)
    lp.cnt_word[lp.n_cnt++] = plan->d.fns[a].word;
    if (def.function != HY_AGG_SUM && def.function != HY_AGG_AVG && def.function != HY_AGG_COUNT) return;
    int32_t& si = sum_of[def.column];
    if (si < 0) {
      std::vector<hyk::LnTerm> chain;
      bool fl = false;
      if (lp.n_sums >= hyk::LN_SUMS || !compile(static_cast<uint32_t>(def.column), &chain, &fl)) return;
      if (terms.size() + chain.size() > static_cast<size_t>(hyk::LN_TERMS)) return;
      si = lp.n_sums++;
      lp.sum_kind[si] = hyk::LN_SUM_CHECK;
      lp.sum_float[si] = fl ? 1 : 0;
      lp.sum_first[si] = static_cast<int32_t>(terms.size());
      lp.sum_len[si] = static_cast<int32_t>(chain.size());
      terms.insert(terms.end(), chain.begin(), chain.end());
    }
    if (def.function != HY_AGG_COUNT) {
      lp.sum_kind[si] = lp.sum_float[si] ? hyk::LN_SUM_FLOAT : hyk::LN_SUM_INT;
      if (lp.sum_nfn[si] >= hyk::LN_SUM_FNS) return;
      lp.sum_word[si][lp.sum_nfn[si]++] = plan->d.fns[a].word;
      lp.sum_limbs[si] = plan->d.fns[a].limbs;
    }
  }
  plan->lanes = true;
  // the contiguous-rows kernels: a data input whose loaded columns' chunks (and a dictionary filter's id arrays) start
  // 16-byte aligned, so one lane's 4 rows are one aligned vector load. agg_dense_vec (default) additionally needs
  // DICT or NULL-free VALUE chunks and < 2^32 rows; HY_AGG_VEC=1 runs agg_dense_lanes' contiguous instance instead,
  // HY_AGG_VEC=0 its strided one (A/B).
  const char* ev = std::getenv("HY_AGG_VEC");
  const int vec_mode = ev ? std::atoi(ev) : 2;
  bool vec = in->n_pos_groups == 0 && vec_mode != 0;
  auto aligned = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; };
  for (const int32_t col : plan->lane_cols)
    for (uint32_t k = 0; k < in->columns[col].n_chunks && vec; ++k)
      vec = in->columns[col].chunks[k].size == 0 || aligned(in->columns[col].chunks[k].data);
  if (in->filter)
    for (uint32_t k = 0; k < in->n_chunks && vec; ++k)
      vec = in->filter[k].column.kind != HY_COL_DICT || in->filter[k].column.size == 0 ||
            aligned(in->filter[k].column.data);
  plan->lanes_vec = vec;
  bool dv = vec && vec_mode != 1 && plan->rows < (1ull << 32) - 1;
  for (const int32_t col : plan->lane_cols)
    for (uint32_t k = 0; k < in->columns[col].n_chunks && dv; ++k) {
      const auto& ch = in->columns[col].chunks[k];
      dv = ch.size == 0 || ch.kind == HY_COL_DICT || (ch.kind == HY_COL_VALUE && ch.nulls == nullptr);
    }
  for (int32_t q = 0; q < lp.n_sums && dv; ++q) dv = lp.sum_len[q] <= hyk::VEC_TERMS;
  dv = dv && lp.n_load <= hyk::VEC_COLS;
  plan->dense_vec = dv;
  plan_stream(in, plan);
}

// Record bytes a hash table may take without a caller-given bound (at load 1/2: 2 slots per expected group).
constexpr uint64_t DEFAULT_RECORD_BUDGET = 2ull << 30;

// Groups the hash table is sized for: the caller's bound, else the product of the group-by columns' distinct-value
// bounds when every group-by column is dictionary-encoded (sum of its chunks' dictionary sizes + NULL), else as many
// groups as DEFAULT_RECORD_BUDGET holds (at least 2^20); never more than the rows.
uint64_t group_bound_of(const hy_agg_input* in, const hy_agg_params* p, uint64_t rows, uint32_t words) {
  if (p->group_bound) return std::min<uint64_t>(p->group_bound, std::max<uint64_t>(rows, 1));
  uint64_t bound = 1;
  bool dict = p->n_groupby > 0;
  for (uint32_t j = 0; j < p->n_groupby && dict; ++j) {
    const auto& c = in->columns[p->groupby[j]];
    uint64_t distinct = 1;  // NULL
    for (uint32_t k = 0; k < c.n_chunks && dict; ++k) {
      if (c.chunks[k].kind != HY_COL_DICT) dict = false;
      distinct += c.chunks[k].dictionary_size;
    }
    bound = std::min<uint64_t>(bound * std::min<uint64_t>(distinct, rows + 1), rows + 1);
  }
  if (p->n_groupby == 0) return 1;
  const uint64_t per_group = 2ull * 8 * std::max(words, 1u);
  const char* knob = std::getenv("HY_AGG_RECORD_BUDGET");  // test knob: a small table, to exercise the retry
  const uint64_t budget = knob ? std::max<uint64_t>(1, std::strtoull(knob, nullptr, 10) / per_group)
                               : std::max<uint64_t>(1ull << 20, DEFAULT_RECORD_BUDGET / per_group);
  return std::min<uint64_t>(std::max<uint64_t>(rows, 1), dict ? bound : budget);
}

inline uint32_t p_groupby(const hy_agg_params* p) { return p->n_groupby; }

// agg_dense_lanes<n_sums> on a persistent grid: as many workgroups as are resident at once (more would leave a
// partly filled last round of workgroups - each works through many tiles in turn).
inline bool agg_prefetch() {
  static const bool v = [] {
    const char* e = std::getenv("HY_AGG_PREFETCH");
    return e && std::strtol(e, nullptr, 10) != 0;
  }();
  return v;
}

template <int N, bool PF, bool VEC>
void launch_lanes_pf(uint64_t n_tiles, size_t lds, hipStream_t s, const hyk::AggDesc& d, const hyk::LanePlan& lp,
                     unsigned long long* records) {
  static int resident = 0;  // per instantiation; LDS per workgroup is small next to the VGPR limit
  if (resident == 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hyk::agg_dense_lanes<N, PF, VEC>, hyk::AGG_THREADS, lds) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = 3, cus = 256;
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(n_tiles, static_cast<uint64_t>(resident)));
  hipLaunchKernelGGL((hyk::agg_dense_lanes<N, PF, VEC>), dim3(grid), dim3(hyk::AGG_THREADS), lds, s, d, lp, records);
}

template <int N>
void launch_lanes_n(bool vec, uint64_t n_tiles, size_t lds, hipStream_t s, const hyk::AggDesc& d,
                    const hyk::LanePlan& lp, unsigned long long* records) {
  if (vec)
    launch_lanes_pf<N, false, true>(n_tiles, lds, s, d, lp, records);
  else if (agg_prefetch())
    launch_lanes_pf<N, true, false>(n_tiles, lds, s, d, lp, records);
  else
    launch_lanes_pf<N, false, false>(n_tiles, lds, s, d, lp, records);
}

// agg_dense_vec<n_sums, all float sums>, persistent like agg_dense_lanes.
template <int N, bool ALLF>
void launch_dense_vec_t(uint64_t n_tiles, size_t lds, hipStream_t s, const hyk::AggDesc& d, const hyk::LanePlan& lp,
                        unsigned long long* records) {
  static int resident = 0;
  if (resident == 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hyk::agg_dense_vec<N, ALLF>, hyk::AGG_THREADS, lds) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = 4, cus = 256;
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(n_tiles, static_cast<uint64_t>(resident)));
  hipLaunchKernelGGL((hyk::agg_dense_vec<N, ALLF>), dim3(grid), dim3(hyk::AGG_THREADS), lds, s, d, lp, records);
}

template <int N>
void launch_dense_vec(bool all_float, uint64_t n_tiles, size_t lds, hipStream_t s, const hyk::AggDesc& d,
                      const hyk::LanePlan& lp, unsigned long long* records) {
  if (all_float)
    launch_dense_vec_t<N, true>(n_tiles, lds, s, d, lp, records);
  else
    launch_dense_vec_t<N, false>(n_tiles, lds, s, d, lp, records);
}

// agg_dense_stream<n_sums>, persistent: as many workgroups as are resident at once.
template <int N>
void launch_dense_stream_t(uint64_t n_tiles, hipStream_t s, const hyk::AggDesc& d, const hyk::LanePlan& lp,
                           const hyk::StreamPlan* plan, unsigned long long* records) {
  static int resident = 0;
  if (resident == 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hyk::agg_dense_stream<N>, hyk::AGG_THREADS, 0) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = 4, cus = 256;
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  // a wave takes whole tiles: enough workgroups for every tile a wave of its own, at most the resident ones
  const uint64_t want = (n_tiles + hyk::ST_WAVES - 1) / hyk::ST_WAVES;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want, resident)));
  hipLaunchKernelGGL((hyk::agg_dense_stream<N>), dim3(grid), dim3(hyk::AGG_THREADS), 0, s, d, lp, plan, records);
}

void launch_dense_stream(int n_sums, uint64_t n_tiles, hipStream_t s, const hyk::AggDesc& d, const hyk::LanePlan& lp,
                         const hyk::StreamPlan* plan, unsigned long long* records) {
  switch (n_sums) {
#define HY_STREAM_CASE(N)                                            \
  case N:                                                            \
    launch_dense_stream_t<N>(n_tiles, s, d, lp, plan, records);      \
    return;
    HY_STREAM_CASE(0)
    HY_STREAM_CASE(1)
    HY_STREAM_CASE(2)
    HY_STREAM_CASE(3)
    HY_STREAM_CASE(4)
    HY_STREAM_CASE(5)
    HY_STREAM_CASE(6)
    HY_STREAM_CASE(7)
    HY_STREAM_CASE(8)
#undef HY_STREAM_CASE
    default:
      break;
  }
}

void launch_lanes(int n_sums, bool vec, bool dense_vec, bool all_float, uint64_t n_tiles, size_t lds, hipStream_t s,
                  const hyk::AggDesc& d, const hyk::LanePlan& lp, unsigned long long* records) {
  if (dense_vec) {
    switch (n_sums) {
#define HY_VEC_CASE(N)                                       \
  case N:                                                    \
    launch_dense_vec<N>(all_float, n_tiles, lds, s, d, lp, records);    \
    return;
      HY_VEC_CASE(0)
      HY_VEC_CASE(1)
      HY_VEC_CASE(2)
      HY_VEC_CASE(3)
      HY_VEC_CASE(4)
      HY_VEC_CASE(5)
      HY_VEC_CASE(6)
      HY_VEC_CASE(7)
      HY_VEC_CASE(8)
#undef HY_VEC_CASE
      default:
        break;
    }
  }
  switch (n_sums) {
#define HY_LANES_CASE(N)                                         \
  case N:                                                        \
    launch_lanes_n<N>(vec, n_tiles, lds, s, d, lp, records);     \
    break;
    HY_LANES_CASE(0)
    HY_LANES_CASE(1)
    HY_LANES_CASE(2)
    HY_LANES_CASE(3)
    HY_LANES_CASE(4)
    HY_LANES_CASE(5)
    HY_LANES_CASE(6)
    HY_LANES_CASE(7)
    HY_LANES_CASE(8)
#undef HY_LANES_CASE
    default:
      break;
  }
}

hy_status make_plan(const hy_agg_input* in, const hy_agg_params* p, AggPlan* plan) {
  if (!in || !p || !plan) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (in->n_columns > hyk::AGG_MAX_COLUMNS) return fail(HY_ERR_UNSUPPORTED, "too many aggregate input columns");
  if (p->n_groupby > hyk::AGG_MAX_GROUPBY) return fail(HY_ERR_UNSUPPORTED, "too many group-by columns");
  if (p->n_aggregates > hyk::AGG_MAX_AGGREGATES) return fail(HY_ERR_UNSUPPORTED, "too many aggregates");
  if (in->n_pos_groups > hyk::AGG_MAX_POS_GROUPS) return fail(HY_ERR_UNSUPPORTED, "too many PosList groups");
  if (in->n_pos_groups && in->n_chunks && !in->pos_lists) return fail(HY_ERR_INVALID_ARGUMENT, "pos_lists missing");
  if (in->n_chunks && !in->chunk_sizes) return fail(HY_ERR_INVALID_ARGUMENT, "chunk_sizes missing");
  auto& d = plan->d;
  d.n_cols = in->n_columns;
  d.n_fns = p->n_aggregates;
  d.n_gb = p->n_groupby;
  d.n_pos_groups = in->n_pos_groups;
  d.n_chunks = in->n_chunks;
  for (uint32_t j = 0; j < in->n_columns; ++j) {
    const auto& c = in->columns[j];
    if (c.value_type < HY_TYPE_INT32 || c.value_type > HY_TYPE_DOUBLE) return fail(HY_ERR_UNSUPPORTED, "column type");
    for (uint32_t k = 0; !c.n_nodes && c.chunks && k < c.n_chunks; ++k)
      if (!row_readable(c.chunks[k])) return fail(HY_ERR_UNSUPPORTED, "aggregate input chunk kind");
    if (c.n_nodes) {  // expression column: evaluated in the kernel (fused) or materialised first
      hyk::ExprProgram prog;
      const hy_status st = validate_program(in, c.program, c.n_nodes, &prog);
      if (st != HY_OK) return st;
      if (prog.out_type != c.value_type) return fail(HY_ERR_INVALID_ARGUMENT, "expression column type");
      for (uint32_t g = 0; g < p->n_groupby; ++g)
        if (p->groupby[g] == static_cast<int32_t>(j)) return fail(HY_ERR_UNSUPPORTED, "GROUP BY an expression column");
      plan->expr_cols.push_back(j);
      plan->exprs.push_back(prog);
      d.cols[j].type = c.value_type;
      d.cols[j].pos_group = -1;
      d.cols[j].ukind = HY_COL_VALUE;  // as materialised (the fused kernel reads slots instead)
      d.cols[j].uwidth = 0;
      d.cols[j].unulls = 1;
      continue;
    }
    if (c.pos_group >= static_cast<int32_t>(in->n_pos_groups)) return fail(HY_ERR_INVALID_ARGUMENT, "pos_group");
    if (c.pos_group < 0 && c.n_chunks != in->n_chunks)
      return fail(HY_ERR_INVALID_ARGUMENT, "data column must have one chunk per input chunk");
    d.cols[j].type = c.value_type;
    d.cols[j].pos_group = c.pos_group;
    d.cols[j].domain = c.domain;
    // one encoding across the column's chunks (agg_dense_span reads columns with uniform control flow)
    int32_t kind = c.n_chunks ? c.chunks[0].kind : HY_COL_VALUE;
    int32_t width = 0, nulls = 0;
    for (uint32_t k = 0; k < c.n_chunks; ++k) {
      const auto& ch = c.chunks[k];
      if (ch.kind != kind) kind = -1;
      if (ch.kind == HY_COL_DICT) {
        if (width == 0) width = ch.vid_width;
        if (ch.vid_width != width) kind = -1;
      }
      if (ch.nulls) nulls = 1;
    }
    d.cols[j].ukind = kind;
    d.cols[j].uwidth = width;
    d.cols[j].unulls = nulls;
  }
  // record layout
  const uint32_t H = p->n_groupby;
  uint32_t w = H + hyk::AGG_HDR_WORDS;
  plan->word_op.assign(w, hyk::WOP_KEY);
  plan->word_op[H + hyk::AGG_HDR_FIRST] = hyk::WOP_MIN;
  plan->word_op[H + hyk::AGG_HDR_LAST] = hyk::WOP_MAX;
  plan->word_op[H + hyk::AGG_HDR_ROWS] = hyk::WOP_ADD;
  auto& L = plan->layout;
  for (uint32_t a = 0; a < p->n_aggregates; ++a) {
    const auto& def = p->aggregates[a];
    auto& fn = d.fns[a];
    fn.function = def.function;
    fn.column = def.column;
    fn.word = w;
    fn.limbs = 0;
    L.agg_word[a] = w;
    L.agg_emin[a] = 0;
    L.agg_limbs[a] = 0;
    if (def.function < HY_AGG_MIN || def.function > HY_AGG_COUNT_DISTINCT)
      return fail(HY_ERR_INVALID_ARGUMENT, "aggregate function");
    if (def.column < 0) {
      if (def.function != HY_AGG_COUNT) return fail(HY_ERR_INVALID_ARGUMENT, "only COUNT may have no column");
      continue;  // COUNT(*): the rows word
    }
    if (def.column >= static_cast<int32_t>(in->n_columns)) return fail(HY_ERR_INVALID_ARGUMENT, "aggregate column");
    const int32_t type = in->columns[def.column].value_type;
    plan->word_op.push_back(hyk::WOP_ADD);  // count
    switch (def.function) {
      case HY_AGG_MIN:
        plan->word_op.push_back(hyk::WOP_MIN);
        break;
      case HY_AGG_MAX:
        plan->word_op.push_back(hyk::WOP_MAX);
        break;
      case HY_AGG_SUM:
      case HY_AGG_AVG:
        if (type == HY_TYPE_FLOAT || type == HY_TYPE_DOUBLE) {
          const bool f = type == HY_TYPE_FLOAT;
          fn.limbs = f ? hyk::FLOAT_LIMBS : hyk::DOUBLE_LIMBS;
          L.agg_limbs[a] = fn.limbs;
          L.agg_emin[a] = f ? hyk::FLOAT_EMIN : hyk::DOUBLE_EMIN;
          plan->word_op.push_back(hyk::WOP_OR);
          for (int l = 0; l < fn.limbs; ++l) plan->word_op.push_back(hyk::WOP_ADD);
          plan->word_op.push_back(hyk::WOP_ADD);  // integer-valued rows (agg_dense_span; zero when flushed)
        } else {
          plan->word_op.push_back(hyk::WOP_ADD);
        }
        break;
      case HY_AGG_COUNT_DISTINCT:
        plan->distinct = true;
        break;
      default:
        break;
    }
    w = static_cast<uint32_t>(plan->word_op.size());
  }
  d.words = static_cast<uint32_t>(plan->word_op.size());
  L.words = d.words;
  for (uint32_t j = 0; j < p->n_groupby; ++j) {
    if (p->groupby[j] < 0 || p->groupby[j] >= static_cast<int32_t>(in->n_columns))
      return fail(HY_ERR_INVALID_ARGUMENT, "group-by column");
    d.gb[j] = p->groupby[j];
  }
  // rows and tiles
  for (uint32_t c = 0; c < in->n_chunks; ++c) {
    plan->rows += in->chunk_sizes[c];
    plan->n_tiles += (in->chunk_sizes[c] + hyk::AGG_TILE - 1) / hyk::AGG_TILE;
  }
  d.n_tiles = plan->n_tiles;
  // dense path: every group-by column has a code domain, the mixed-radix index fits a wave's 64 lanes and the
  // records fit the LDS budget
  uint64_t groups = 1;
  bool dense = !plan->distinct;
  for (uint32_t j = 0; j < p->n_groupby && dense; ++j) {
    const auto& c = in->columns[p->groupby[j]];
    if (c.domain == 0 || (c.value_type != HY_TYPE_INT32 && c.value_type != HY_TYPE_INT64)) dense = false;
    groups *= static_cast<uint64_t>(c.domain) + 1;
    if (groups > hyk::AGG_DENSE_MAX) dense = false;
  }
  if (dense && groups * d.words > hyk::AGG_DENSE_LDS_WORDS) dense = false;
  if (dense) {
    uint32_t stride = 1;
    for (uint32_t j = 0; j < p->n_groupby; ++j) {
      auto& col = d.cols[d.gb[j]];
      col.stride = stride;
      stride *= col.domain + 1;
    }
    plan->dense_groups = static_cast<uint32_t>(groups);
  }
  L.dense = dense ? 1 : 0;
  plan_fused(in, p, plan);
  plan_lanes(in, p, plan);
  plan->materialize = !plan->fused && !plan->expr_cols.empty();
  plan->cap = next_pow2(std::max<uint64_t>(64, 2 * group_bound_of(in, p, plan->rows, d.words)));
  plan->max_groups = plan->cap / 4 * 3;  // load factor limit: past it the insert reports HY_ERR_GROUP_BOUND
  plan->dcap = plan->distinct ? next_pow2(std::max<uint64_t>(64, 2 * plan->rows * p->n_aggregates)) : 0;
  return HY_OK;
}

// Workspace carve (sizes only when base == nullptr).
struct AggWs {
  uint32_t* sizes;
  uint64_t* row_begin;
  uint64_t* tile_begin;
  uint32_t* tile_owner;
  const hy_row_id** pos_lists;
  hy_column_chunk* chunks[hyk::AGG_MAX_COLUMNS];
  int32_t* word_op;
  uint32_t* misc;  // [0] error, [2..3] n_out (u64)
  hyk::FqOp* fused_nodes;        // agg_dense_fused: its expression ops
  hyk::LnTerm* lane_terms;       // agg_dense_lanes: its chains
  uint32_t* deferred;            // agg_dense_lanes: steps left to agg_dense_fused
  hyk::LaneTables* lane_tables;
  hyk::StreamPlan* stream_plan;
  hy_scan_chunk* filter;         // fused TableScan predicate chunks
  void* mat_values[hyk::AGG_MAX_COLUMNS];    // materialised expression columns
  uint8_t* mat_nulls[hyk::AGG_MAX_COLUMNS];
  hyk::ExprProgram* mat_progs;   // their programs and outputs (one projection launch for all of them)
  hyk::ProjOut* mat_outs;
  uint32_t* state;
  unsigned long long* records;
  uint32_t* dstate;
  unsigned long long* dkeys;
};

void carve(Carver& cv, const hy_agg_input* in, const AggPlan& plan, AggWs* w) {
  w->sizes = cv.take<uint32_t>(std::max<uint32_t>(1, in->n_chunks));
  w->row_begin = cv.take<uint64_t>(in->n_chunks + 1);
  w->tile_begin = cv.take<uint64_t>(in->n_chunks + 1);
  w->tile_owner = cv.take<uint32_t>(std::max<uint64_t>(1, plan.n_tiles));
  w->pos_lists = cv.take<const hy_row_id*>(std::max<uint64_t>(1, uint64_t(in->n_pos_groups) * in->n_chunks));
  for (uint32_t j = 0; j < in->n_columns; ++j)  // expression columns: one materialised chunk per input chunk
    w->chunks[j] = cv.take<hy_column_chunk>(
        std::max<uint32_t>(1, in->columns[j].n_nodes ? in->n_chunks : in->columns[j].n_chunks));
  w->word_op = cv.take<int32_t>(plan.word_op.size());
  w->fused_nodes = cv.take<hyk::FqOp>(std::max<size_t>(1, plan.fused_nodes.size()));
  w->lane_terms = cv.take<hyk::LnTerm>(plan.lane_terms.size() + hyk::VEC_TERMS);  // padding: agg_dense_vec
  w->lane_tables = cv.take<hyk::LaneTables>(1);
  w->stream_plan = cv.take<hyk::StreamPlan>(1);
  w->filter = cv.take<hy_scan_chunk>(in->filter ? std::max<uint32_t>(1, in->n_chunks) : 1);
  w->deferred = cv.take<uint32_t>(plan.lanes ? std::max<uint64_t>(1, plan.n_tiles * hyk::FQ_STEPS_PER_TILE) : 1);
  for (uint32_t e = 0; e < plan.expr_cols.size(); ++e) {
    const uint32_t j = plan.expr_cols[e];
    w->mat_values[j] = plan.materialize ? cv.take<uint64_t>(std::max<uint64_t>(2, plan.rows)) : nullptr;
    w->mat_nulls[j] = plan.materialize ? cv.take<uint8_t>(std::max<uint64_t>(16, plan.rows)) : nullptr;
  }
  w->mat_progs = cv.take<hyk::ExprProgram>(std::max<size_t>(1, plan.expr_cols.size()));
  w->mat_outs = cv.take<hyk::ProjOut>(std::max<size_t>(1, plan.expr_cols.size()));
  w->misc = cv.take<uint32_t>(64);
  if (plan.dense_groups) {
    w->state = nullptr;
    w->records = cv.take<unsigned long long>(uint64_t(plan.dense_groups) * plan.d.words);
    w->dstate = nullptr;
    w->dkeys = nullptr;
  } else {
    w->state = cv.take<uint32_t>(plan.cap);
    w->records = cv.take<unsigned long long>(plan.cap * plan.d.words);
    w->dstate = plan.dcap ? cv.take<uint32_t>(plan.dcap) : nullptr;
    w->dkeys = plan.dcap ? cv.take<unsigned long long>(2 * plan.dcap) : nullptr;
  }
}

// The fused TableScan of hy_agg_input.filter: data input on the dense expression path (agg_dense_lanes /
// agg_dense_fused apply it); predicate chunks as hy_table_scan validates them.
hy_status check_filter(const hy_agg_input* in, const AggPlan& plan) {
  if (!in->filter) return HY_OK;
  if (in->n_pos_groups != 0 || !plan.fused || !plan.dense_groups)
    return fail(HY_ERR_UNSUPPORTED, "a fused scan needs a data input on the dense aggregate path");
  for (uint32_t c = 0; c < in->n_chunks; ++c) {
    const hy_scan_chunk& f = in->filter[c];
    if (f.column.size != in->chunk_sizes[c]) return fail(HY_ERR_INVALID_ARGUMENT, "filter chunk size != input chunk");
    if (f.op < HY_OP_EQ || f.op > HY_OP_IS_NOT_NULL || f.op == HY_OP_IS_NULL)
      return fail(HY_ERR_UNSUPPORTED, "fused scan filter op");
    if (f.op == HY_OP_NONE || f.column.size == 0) continue;
    if (!row_readable(f.column)) return fail(HY_ERR_UNSUPPORTED, "fused scan filter chunk kind");
    if (!f.column.data) return fail(HY_ERR_INVALID_ARGUMENT, "filter chunk without data");
    if (f.column.kind == HY_COL_DICT) {
      if (f.column.vid_width != 1 && f.column.vid_width != 2 && f.column.vid_width != 4)
        return fail(HY_ERR_INVALID_ARGUMENT, "filter vid width");
    } else if (!in->filter_constant || (in->filter_value_type < HY_TYPE_INT32 || in->filter_value_type > HY_TYPE_DOUBLE)) {
      return fail(HY_ERR_INVALID_ARGUMENT, "filter constant / value type");
    }
  }
  return HY_OK;
}

}  // namespace

extern "C" {

hy_status hy_aggregate_layout(const hy_agg_input* input, const hy_agg_params* params, hy_agg_layout* layout) {
  if (!layout) return fail(HY_ERR_INVALID_ARGUMENT, "null layout");
  AggPlan plan;
  const hy_status st = make_plan(input, params, &plan);
  if (st != HY_OK) return st;
  *layout = plan.layout;
  return HY_OK;
}

hy_status hy_aggregate_workspace_size(const hy_agg_input* input, const hy_agg_params* params, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null bytes");
  AggPlan plan;
  hy_status st = make_plan(input, params, &plan);
  if (st != HY_OK) return st;
  st = check_filter(input, plan);
  if (st != HY_OK) return st;
  Carver cv{nullptr, 0};
  AggWs w;
  carve(cv, input, plan, &w);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_aggregate(const hy_agg_input* input, const hy_agg_params* params, uint64_t* out_records,
                       uint64_t out_capacity, uint64_t* n_groups, void* workspace, size_t workspace_bytes,
                       hy_stream_t stream) {
  if (!n_groups) return fail(HY_ERR_INVALID_ARGUMENT, "null n_groups");
  AggPlan plan;
  hy_status st = make_plan(input, params, &plan);
  if (st != HY_OK) return st;
  st = check_filter(input, plan);
  if (st != HY_OK) return st;
  hipStream_t s = S(stream);
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  AggWs w;
  carve(cv, input, plan, &w);
  if (!cv.ok || !workspace) return fail(HY_ERR_WORKSPACE, "aggregate workspace too small");
  auto& d = plan.d;
  // descriptors
  std::vector<uint64_t> row_begin(input->n_chunks + 1, 0), tile_begin(input->n_chunks + 1, 0);
  for (uint32_t c = 0; c < input->n_chunks; ++c) {
    row_begin[c + 1] = row_begin[c] + input->chunk_sizes[c];
    tile_begin[c + 1] = tile_begin[c] + (input->chunk_sizes[c] + hyk::AGG_TILE - 1) / hyk::AGG_TILE;
  }
  if (input->n_chunks) {
    HY_STAGE(w.sizes, input->chunk_sizes, 4 * input->n_chunks, s);
    HY_STAGE(w.row_begin, row_begin.data(), 8 * row_begin.size(), s);
    HY_STAGE(w.tile_begin, tile_begin.data(), 8 * tile_begin.size(), s);
  }
  const uint64_t n_pl = uint64_t(input->n_pos_groups) * input->n_chunks;
  if (n_pl) HY_STAGE(w.pos_lists, input->pos_lists, sizeof(void*) * n_pl, s);
  for (uint32_t j = 0; j < input->n_columns; ++j) {
    const auto& c = input->columns[j];
    for (uint32_t k = 0; k < (c.n_nodes ? 0u : c.n_chunks); ++k) {
      const auto& ch = c.chunks[k];
      if (ch.size && !ch.data) return fail(HY_ERR_INVALID_ARGUMENT, "column chunk without data");
      if (ch.kind == HY_COL_DICT && ch.vid_width != 1 && ch.vid_width != 2 && ch.vid_width != 4)
        return fail(HY_ERR_INVALID_ARGUMENT, "vid width");
    }
    if (c.n_chunks && !c.n_nodes)
      HY_STAGE(w.chunks[j], c.chunks, sizeof(hy_column_chunk) * c.n_chunks, s);
    d.cols[j].chunks = w.chunks[j];
  }
  HY_STAGE(w.word_op, plan.word_op.data(), 4 * plan.word_op.size(), s);
  HY_HIP(hipMemsetAsync(w.misc, 0, 256, s));
  d.pos_lists = w.pos_lists;
  d.chunk_size = w.sizes;
  d.chunk_row_begin = w.row_begin;
  d.chunk_tile_begin = w.tile_begin;
  d.tile_chunk = w.tile_owner;
  if (plan.n_tiles) {
    hipLaunchKernelGGL(hyk::fill_tile_owner, dim3((input->n_chunks + 255) / 256), dim3(256), 0, s, w.tile_begin,
                       input->n_chunks, w.tile_owner);
    HY_HIP(hipGetLastError());
  }
  d.word_op = w.word_op;
  d.error = w.misc;
  if (input->filter && input->n_chunks) {
    HY_STAGE(w.filter, input->filter, sizeof(hy_scan_chunk) * input->n_chunks, s);
    d.filter = w.filter;
    d.filter_type = input->filter_value_type;
    d.filter_cbits = 0;
    if (input->filter_constant) {
      const bool wide = input->filter_value_type == HY_TYPE_INT64 || input->filter_value_type == HY_TYPE_DOUBLE;
      std::memcpy(&d.filter_cbits, input->filter_constant, wide ? 8 : 4);
    }
  }
  auto* n_out = reinterpret_cast<unsigned long long*>(w.misc + 2);
  auto* out = reinterpret_cast<unsigned long long*>(out_records);
  // expression columns outside the fused kernel: materialised (projection kernel over the same input), then read as
  // data columns with NULL flags
  std::vector<std::vector<hy_column_chunk>> mat_chunks(plan.expr_cols.size());
  if (!plan.expr_cols.empty() && plan.materialize && plan.rows) {
    std::vector<hyk::ProjOut> outs(plan.expr_cols.size());
    for (uint32_t e = 0; e < plan.expr_cols.size(); ++e)
      outs[e] = hyk::ProjOut{w.mat_progs + e, w.mat_values[plan.expr_cols[e]], w.mat_nulls[plan.expr_cols[e]]};
    HY_STAGE(w.mat_progs, plan.exprs.data(), sizeof(hyk::ExprProgram) * plan.expr_cols.size(), s);
    HY_STAGE(w.mat_outs, outs.data(), sizeof(hyk::ProjOut) * outs.size(), s);
    const uint32_t items = hyk::flat_items(plan.rows);
    const uint64_t tile_rows = uint64_t(hyk::AGG_THREADS) * items;
    hipLaunchKernelGGL(hyk::projection_kernel, dim3(static_cast<uint32_t>((plan.rows + tile_rows - 1) / tile_rows)),
                       dim3(hyk::AGG_THREADS), 0, s, d, w.mat_outs, static_cast<uint32_t>(outs.size()), plan.rows,
                       items);
    HY_HIP(hipGetLastError());
  }
  for (uint32_t e = 0; e < plan.expr_cols.size() && plan.materialize && plan.rows; ++e) {
    const uint32_t j = plan.expr_cols[e];
    const int bytes = (plan.exprs[e].out_type == HY_TYPE_INT64 || plan.exprs[e].out_type == HY_TYPE_DOUBLE) ? 8 : 4;
    auto& chs = mat_chunks[e];
    chs.resize(input->n_chunks);
    for (uint32_t c = 0; c < input->n_chunks; ++c) {
      chs[c] = hy_column_chunk{};
      chs[c].data = static_cast<char*>(w.mat_values[j]) + bytes * row_begin[c];
      chs[c].nulls = w.mat_nulls[j] + row_begin[c];
      chs[c].size = input->chunk_sizes[c];
      chs[c].kind = HY_COL_VALUE;
    }
    HY_STAGE(w.chunks[j], chs.data(), sizeof(hy_column_chunk) * chs.size(), s);
  }

  if (plan.fused && plan.dense_groups) {
    const uint64_t nw = uint64_t(plan.dense_groups) * d.words;
    hipLaunchKernelGGL(hyk::agg_init_records, dim3(grid_for(nw, 256)), dim3(256), 0, s, w.records,
                       uint64_t(plan.dense_groups), d.words, w.word_op);
    HY_HIP(hipGetLastError());
    if (!plan.fused_nodes.empty())
      HY_STAGE(w.fused_nodes, plan.fused_nodes.data(), sizeof(hyk::FqOp) * plan.fused_nodes.size(), s);
    hyk::FusedPlan fp = plan.fp;
    fp.progs = w.fused_nodes;
    const size_t lds = sizeof(unsigned long long) * plan.dense_groups * d.words;
    if (plan.n_tiles && plan.lanes) {
      // per-lane accumulation; the steps it cannot take (NULLs, non-finite values, ...) are listed for the fused
      // kernel, which then runs over that list only (misc[8] = its length, zeroed above)
      hyk::LaneTables lt = plan.lt;
      for (int32_t li = 0; li < lt.n_load; ++li) lt.load_chunks[li] = d.cols[plan.lane_cols[li]].chunks;
      HY_STAGE(w.lane_tables, &lt, sizeof(lt), s);
      HY_STAGE(w.lane_terms, plan.lane_terms.data(), sizeof(hyk::LnTerm) * plan.lane_terms.size(), s);
      // (agg_dense_vec reads VEC_TERMS terms per sum: the table is padded to LN_TERMS + VEC_TERMS entries)
      const hyk::LanePlan lp{lt.n_load, lt.n_sums, w.lane_tables, w.lane_terms, w.deferred, w.misc + 8};
      const int n_store = lt.n_load - static_cast<int>(params->n_groupby);
      const size_t vlds = size_t(hyk::AGG_THREADS / hyk::WAVE) * (plan.dense_vec ? hyk::vec_wave_lds(n_store, lt.n_sums)
                                                                                 : hyk::ln_wave_lds(n_store, lt.n_sums));
      // the all-float instance (no per-value choice of conversion) unless HY_VEC_ALLF=0 (A/B)
      const char* eaf = std::getenv("HY_VEC_ALLF");
      bool all_float = !(eaf && std::atoi(eaf) == 0);
      for (int32_t q = 0; q < lt.n_sums; ++q) all_float = all_float && lt.sum_kind[q] != hyk::LN_SUM_INT;
      if (plan.dense_stream) {
        hyk::StreamPlan sp = plan.stream_plan;
        sp.tile_chunk = d.tile_chunk;
        sp.chunk_tile_begin = d.chunk_tile_begin;
        sp.chunk_size = d.chunk_size;
        sp.chunk_row_begin = d.chunk_row_begin;
        sp.filter = d.filter;
        HY_STAGE(w.stream_plan, &sp, sizeof(sp), s);
        std::string jit_err;
        bool ran_jit = false;
        if (plan.dense_jit) {
          hyj::JitArgs ja{};
          for (int32_t li = 0; li < lt.n_load; ++li)
            ja.cols[li] = reinterpret_cast<const hyj::ColumnChunk*>(lt.load_chunks[li]);
          ja.filter = reinterpret_cast<const hyj::ScanChunk*>(d.filter);
          ja.tile_chunk = d.tile_chunk;
          ja.chunk_tile_begin = d.chunk_tile_begin;
          ja.chunk_size = d.chunk_size;
          ja.chunk_row_begin = d.chunk_row_begin;
          ja.records = w.records;
          ja.deferred = w.deferred;
          ja.n_deferred = w.misc + 8;
          ja.error = d.error;
          ja.n_tiles = plan.n_tiles;
          KTimer t("agg_dense_jit", s, plan.rows);
          ran_jit = hyjit::launch(plan.jit_shape, ja, s, &jit_err);
          t.done();
          if (!ran_jit) {  // (reported once per process; agg_dense_stream runs instead)
            static std::once_flag warned;
            std::call_once(warned, [&] { std::fprintf(stderr, "hyrise-amd: plan-compiled aggregate unavailable (%s); "
                                                              "using agg_dense_stream\n", jit_err.c_str()); });
          }
        }
        if (!ran_jit) {
          KTimer t("agg_dense_stream", s, plan.rows);
          launch_dense_stream(lp.n_sums, plan.n_tiles, s, d, lp, w.stream_plan, w.records);
          t.done();
        }
      } else {
        KTimer t(plan.dense_vec ? "agg_dense_vec" : "agg_dense_lanes", s, plan.rows);
        launch_lanes(lp.n_sums, plan.lanes_vec, plan.dense_vec, all_float, plan.n_tiles, vlds, s, d, lp, w.records);
        t.done();
      }
      HY_HIP(hipGetLastError());
      KTimer t("agg_dense_fused.deferred", s, 0);
      hipLaunchKernelGGL(hyk::agg_dense_fused, dim3(256), dim3(hyk::AGG_THREADS), lds, s, d, fp, plan.dense_groups,
                         w.records, static_cast<const uint32_t*>(w.deferred), static_cast<const uint32_t*>(w.misc + 8));
      t.done();
      HY_HIP(hipGetLastError());
    } else if (plan.n_tiles) {
      const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(plan.n_tiles, 256 * 16));
      KTimer t("agg_dense_fused", s, plan.rows);
      hipLaunchKernelGGL(hyk::agg_dense_fused, dim3(grid), dim3(hyk::AGG_THREADS), lds, s, d, fp, plan.dense_groups,
                         w.records, static_cast<const uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr));
      t.done();
      HY_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(hyk::agg_dense_compact, dim3((plan.dense_groups + 63) / 64), dim3(64), 0, s, d,
                       plan.dense_groups, w.records, out, out_capacity, n_out);
    HY_HIP(hipGetLastError());
  } else if (plan.dense_groups) {
    const uint64_t nw = uint64_t(plan.dense_groups) * d.words;
    hipLaunchKernelGGL(hyk::agg_init_records, dim3(grid_for(nw, 256)), dim3(256), 0, s, w.records,
                       uint64_t(plan.dense_groups), d.words, w.word_op);
    HY_HIP(hipGetLastError());
    // agg_dense_span (batched column reads, per-span register folding) unless a column mixes encodings or the
    // input has several PosList groups; HY_AGG_DENSE_ROWS=1 forces the per-64-row kernel (test knob)
    bool span = input->n_pos_groups <= 1;
    for (uint32_t j = 0; j < input->n_columns; ++j) span = span && d.cols[j].ukind >= 0;
    if (const char* e = std::getenv("HY_AGG_DENSE_ROWS")) span = span && std::atoi(e) == 0;
    if (plan.n_tiles && span) {
      const size_t lds = sizeof(unsigned long long) * plan.dense_groups * d.words;
      const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(plan.n_tiles, 256 * 16));
      KTimer t("agg_dense_span", s, plan.rows);
      hipLaunchKernelGGL(hyk::agg_dense_span, dim3(grid), dim3(hyk::AGG_THREADS), lds, s, d, plan.dense_groups,
                         w.records);
      t.done();
      HY_HIP(hipGetLastError());
    } else if (plan.n_tiles) {
      const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(plan.n_tiles, 256 * 8));
      KTimer t("agg_dense_rows", s, plan.rows);
      hipLaunchKernelGGL(hyk::agg_dense_rows, dim3(grid), dim3(hyk::AGG_THREADS), 0, s, d, plan.dense_groups,
                         w.records);
      t.done();
      HY_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(hyk::agg_dense_compact, dim3((plan.dense_groups + 63) / 64), dim3(64), 0, s, d,
                       plan.dense_groups, w.records, out, out_capacity, n_out);
    HY_HIP(hipGetLastError());
  } else {
    hyk::AggTable t{w.state, w.records, plan.cap, w.dstate, w.dkeys, plan.dcap};
    HY_HIP(hipMemsetAsync(w.state, 0, 4 * plan.cap, s));
    if (plan.dcap) HY_HIP(hipMemsetAsync(w.dstate, 0, 4 * plan.dcap, s));
    if (plan.rows) {
      KTimer kt("agg_hash_runs", s, plan.rows);
      const uint32_t items = hyk::flat_items(plan.rows);  // tiles over global rows
      const uint64_t tile_rows = uint64_t(hyk::AGG_THREADS) * items;
      hipLaunchKernelGGL(hyk::agg_hash_runs, dim3(static_cast<uint32_t>((plan.rows + tile_rows - 1) / tile_rows)),
                         dim3(hyk::AGG_THREADS), 0, s, d, t, plan.rows, items);
      kt.done();
      HY_HIP(hipGetLastError());
    }
    const uint64_t rows_of_slots = (plan.cap + 256ull * hyk::HC_ITEMS - 1) / (256ull * hyk::HC_ITEMS);
    hipLaunchKernelGGL(hyk::agg_hash_compact, dim3(static_cast<uint32_t>(std::min<uint64_t>(rows_of_slots, 4096))),
                       dim3(256), 0, s, d, t, out, out_capacity, n_out);
    HY_HIP(hipGetLastError());
  }
  uint32_t misc[4] = {0, 0, 0, 0};
  HY_HIP(hipMemcpyAsync(misc, w.misc, 16, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  uint64_t n = 0;
  std::memcpy(&n, misc + 2, 8);
  *n_groups = n;
  if (misc[0] & 2u) return fail(HY_ERR_INVALID_ARGUMENT, "dense group-by code outside its domain");
  const bool hashed = !plan.dense_groups;  // (the hash table branch above)
  if ((misc[0] & 4u) || (hashed && n > plan.max_groups)) {  // more groups than the table was sized for: suggest a
                                                            // bound 4x larger
    *n_groups = std::min<uint64_t>(std::max<uint64_t>(plan.rows, 1), std::max<uint64_t>(64, plan.cap / 2) * 4);
    return fail(HY_ERR_GROUP_BOUND, "more groups than group_bound; retry with *n_groups");
  }
  if (misc[0] & 1u) return fail(HY_ERR_KERNEL, "aggregate hash table probe did not terminate");
  if (n > out_capacity) return fail(HY_ERR_CAPACITY, "more groups than out_capacity");
  return HY_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Projection (expression evaluation over an aggregate-style input)
// ---------------------------------------------------------------------------------------------------------------
namespace {

struct ProjWs {
  uint64_t* row_begin;
  const hy_row_id** pos_lists;
  hy_column_chunk* chunks[hyk::AGG_MAX_COLUMNS];
  hyk::ExprProgram* progs;  // HY_PROJ_MAX_OUTPUTS
  hyk::ProjOut* outs;
};

void carve_proj(Carver& cv, const hy_agg_input* in, ProjWs* w) {
  w->row_begin = cv.take<uint64_t>(in->n_chunks + 1);
  w->pos_lists = cv.take<const hy_row_id*>(std::max<uint64_t>(1, uint64_t(in->n_pos_groups) * in->n_chunks));
  for (uint32_t j = 0; j < in->n_columns; ++j)
    w->chunks[j] = cv.take<hy_column_chunk>(std::max<uint32_t>(1, in->columns[j].n_chunks));
  w->progs = cv.take<hyk::ExprProgram>(HY_PROJ_MAX_OUTPUTS);
  w->outs = cv.take<hyk::ProjOut>(HY_PROJ_MAX_OUTPUTS);
}

// A postfix program checked against the input (stack depth, column indexes, types) into its kernel form.
hy_status compile_program(const hy_agg_input* input, const hy_expr_node* program, uint32_t n_nodes,
                          hyk::ExprProgram* prog) {
  if (!program || n_nodes == 0 || n_nodes > HY_EXPR_MAX_NODES) return fail(HY_ERR_INVALID_ARGUMENT, "program size");
  *prog = hyk::ExprProgram{};
  int depth = 0;
  for (uint32_t i = 0; i < n_nodes; ++i) {
    const hy_expr_node& nd = program[i];
    prog->nodes[i] = nd;
    const bool typed = nd.type >= HY_TYPE_INT32 && nd.type <= HY_TYPE_DOUBLE;
    switch (nd.kind) {
      case HY_EXPR_COLUMN:
        if (nd.column < 0 || nd.column >= static_cast<int32_t>(input->n_columns))
          return fail(HY_ERR_INVALID_ARGUMENT, "expression column");
        if (nd.type != input->columns[nd.column].value_type) return fail(HY_ERR_INVALID_ARGUMENT, "column node type");
        ++depth;
        break;
      case HY_EXPR_VALUE:
        if (!typed && nd.type != 0) return fail(HY_ERR_INVALID_ARGUMENT, "literal type");
        ++depth;
        break;
      case HY_EXPR_ADD:
      case HY_EXPR_SUB:
      case HY_EXPR_MUL:
      case HY_EXPR_DIV:
      case HY_EXPR_MOD:
        if (depth < 2) return fail(HY_ERR_INVALID_ARGUMENT, "expression stack underflow");
        if (!typed || nd.calc_type < HY_TYPE_INT32 || nd.calc_type > HY_TYPE_DOUBLE)
          return fail(HY_ERR_INVALID_ARGUMENT, "arithmetic node types");
        --depth;
        break;
      default:
        return fail(HY_ERR_INVALID_ARGUMENT, "expression node kind");
    }
    if (depth > HY_EXPR_MAX_DEPTH) return fail(HY_ERR_UNSUPPORTED, "expression deeper than HY_EXPR_MAX_DEPTH");
  }
  if (depth != 1) return fail(HY_ERR_INVALID_ARGUMENT, "program does not leave one value");
  prog->n_nodes = n_nodes;
  prog->out_type = program[n_nodes - 1].type;
  if (prog->out_type == 0) return fail(HY_ERR_UNSUPPORTED, "an all-NULL expression has no column type");
  return HY_OK;
}

hy_status check_proj_input(const hy_agg_input* in) {
  if (!in) return fail(HY_ERR_INVALID_ARGUMENT, "null input");
  if (in->n_columns > hyk::AGG_MAX_COLUMNS) return fail(HY_ERR_UNSUPPORTED, "too many projection input columns");
  if (in->n_pos_groups > hyk::AGG_MAX_POS_GROUPS) return fail(HY_ERR_UNSUPPORTED, "too many PosList groups");
  if (in->n_chunks && !in->chunk_sizes) return fail(HY_ERR_INVALID_ARGUMENT, "chunk_sizes missing");
  if (in->n_pos_groups && in->n_chunks && !in->pos_lists) return fail(HY_ERR_INVALID_ARGUMENT, "pos_lists missing");
  for (uint32_t j = 0; j < in->n_columns; ++j) {
    const auto& c = in->columns[j];
    if (c.value_type < HY_TYPE_INT32 || c.value_type > HY_TYPE_DOUBLE) return fail(HY_ERR_UNSUPPORTED, "column type");
    if (c.pos_group >= static_cast<int32_t>(in->n_pos_groups)) return fail(HY_ERR_INVALID_ARGUMENT, "pos_group");
    if (c.pos_group < 0 && c.n_chunks != in->n_chunks)
      return fail(HY_ERR_INVALID_ARGUMENT, "data column must have one chunk per input chunk");
    for (uint32_t k = 0; c.chunks && k < c.n_chunks; ++k)
      if (!row_readable(c.chunks[k])) return fail(HY_ERR_UNSUPPORTED, "projection input chunk kind");
  }
  return HY_OK;
}

}  // namespace

hy_status hy_projection_workspace_size(const hy_agg_input* input, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null bytes");
  hy_status st = check_proj_input(input);
  if (st != HY_OK) return st;
  Carver cv{nullptr, 0};
  ProjWs w;
  carve_proj(cv, input, &w);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_projection_multi(const hy_agg_input* input, const hy_expr_node* const* programs, const uint32_t* n_nodes,
                              uint32_t n_programs, void* const* out_values, uint8_t* const* out_nulls, void* workspace,
                              size_t workspace_bytes, hy_stream_t stream) {
  hy_status st = check_proj_input(input);
  if (st != HY_OK) return st;
  if (n_programs == 0 || n_programs > HY_PROJ_MAX_OUTPUTS || !programs || !n_nodes || !out_values)
    return fail(HY_ERR_INVALID_ARGUMENT, "programs");
  hyk::ExprProgram progs[HY_PROJ_MAX_OUTPUTS];
  for (uint32_t i = 0; i < n_programs; ++i) {
    st = compile_program(input, programs[i], n_nodes[i], &progs[i]);
    if (st != HY_OK) return st;
  }
  std::vector<uint64_t> row_begin(input->n_chunks + 1, 0);
  for (uint32_t c = 0; c < input->n_chunks; ++c) row_begin[c + 1] = row_begin[c] + input->chunk_sizes[c];
  const uint64_t rows = row_begin[input->n_chunks];
  if (rows == 0) return HY_OK;
  for (uint32_t i = 0; i < n_programs; ++i)
    if (!out_values[i]) return fail(HY_ERR_INVALID_ARGUMENT, "out_values");
  const uint32_t items = hyk::flat_items(rows);  // tiles over global rows
  const uint64_t tiles = (rows + uint64_t(hyk::AGG_THREADS) * items - 1) / (uint64_t(hyk::AGG_THREADS) * items);
  hipStream_t s = S(stream);
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  ProjWs w;
  carve_proj(cv, input, &w);
  if (!cv.ok || !workspace) return fail(HY_ERR_WORKSPACE, "projection workspace too small");
  HY_STAGE(w.row_begin, row_begin.data(), 8 * row_begin.size(), s);
  const uint64_t n_pl = uint64_t(input->n_pos_groups) * input->n_chunks;
  if (n_pl) HY_STAGE(w.pos_lists, input->pos_lists, sizeof(void*) * n_pl, s);
  hyk::ProjOut outs[HY_PROJ_MAX_OUTPUTS];
  for (uint32_t i = 0; i < n_programs; ++i) outs[i] = hyk::ProjOut{w.progs + i, out_values[i], out_nulls ? out_nulls[i] : nullptr};
  HY_STAGE(w.progs, progs, sizeof(hyk::ExprProgram) * n_programs, s);
  HY_STAGE(w.outs, outs, sizeof(hyk::ProjOut) * n_programs, s);
  hyk::AggDesc d{};
  d.n_cols = input->n_columns;
  d.n_pos_groups = input->n_pos_groups;
  d.n_chunks = input->n_chunks;
  d.n_tiles = tiles;
  for (uint32_t j = 0; j < input->n_columns; ++j) {
    const auto& c = input->columns[j];
    for (uint32_t k = 0; k < c.n_chunks; ++k)
      if (c.chunks[k].size && !c.chunks[k].data) return fail(HY_ERR_INVALID_ARGUMENT, "column chunk without data");
    if (c.n_chunks)
      HY_STAGE(w.chunks[j], c.chunks, sizeof(hy_column_chunk) * c.n_chunks, s);
    d.cols[j].chunks = w.chunks[j];
    d.cols[j].type = c.value_type;
    d.cols[j].pos_group = c.pos_group;
  }
  d.pos_lists = w.pos_lists;
  d.chunk_row_begin = w.row_begin;
  KTimer t("projection", s, rows);
  hipLaunchKernelGGL(hyk::projection_kernel, dim3(static_cast<uint32_t>(tiles)), dim3(hyk::AGG_THREADS), 0, s, d, w.outs,
                     n_programs, rows, items);
  t.done();
  HY_HIP(hipGetLastError());
  return HY_OK;  // asynchronous: the descriptors went through the pinned staging ring
}

hy_status hy_projection(const hy_agg_input* input, const hy_expr_node* program, uint32_t n_nodes, void* out_values,
                        uint8_t* out_nulls, void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  // (a null out_values is rejected after the empty-input early return, as hy_projection_multi checks it)
  return hy_projection_multi(input, &program, &n_nodes, 1, &out_values, &out_nulls, workspace, workspace_bytes, stream);
}

hy_status hy_agg_float_sum(const uint64_t* limbs, uint32_t n_limbs, int32_t emin, uint64_t special, double* out) {
  if (!out || (n_limbs && !limbs)) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if ((special & 4u) || ((special & 1u) && (special & 2u))) {
    *out = NAN;
    return HY_OK;
  }
  if (special & 1u) {
    *out = INFINITY;
    return HY_OK;
  }
  if (special & 2u) {
    *out = -INFINITY;
    return HY_OK;
  }
  // carry-normalise the signed limbs into base-2^32 digits of a two's complement integer
  std::vector<uint32_t> dig(n_limbs + 3, 0);
  __int128 carry = 0;
  for (uint32_t i = 0; i < n_limbs + 3; ++i) {
    const __int128 t = carry + (i < n_limbs ? static_cast<__int128>(static_cast<int64_t>(limbs[i])) : 0);
    dig[i] = static_cast<uint32_t>(static_cast<unsigned __int128>(t) & 0xFFFFFFFFu);
    carry = t >> 32;  // arithmetic
  }
  const bool neg = carry < 0;
  if (neg) {  // magnitude = two's complement negation
    uint64_t c = 1;
    for (auto& x : dig) {
      const uint64_t v = static_cast<uint64_t>(static_cast<uint32_t>(~x)) + c;
      x = static_cast<uint32_t>(v);
      c = v >> 32;
    }
  }
  int top = static_cast<int>(dig.size()) - 1;
  while (top >= 0 && dig[top] == 0) --top;
  if (top < 0) {
    *out = 0.0;
    return HY_OK;
  }
  // 64-bit window below the leading one, plus sticky bits
  const int lead = 31 - __builtin_clz(dig[top]);
  const int64_t msb = static_cast<int64_t>(top) * 32 + lead;  // bit index of the leading one
  auto bit_at = [&](int64_t b) -> uint64_t {
    if (b < 0) return 0;
    return (dig[b >> 5] >> (b & 31)) & 1u;
  };
  uint64_t m = 0;
  for (int64_t b = msb; b > msb - 64; --b) m = (m << 1) | bit_at(b);
  bool sticky = false;
  for (int64_t b = msb - 64; b >= 0 && !sticky; --b) sticky = bit_at(b) != 0;
  // round the 64-bit window to 53 bits, nearest-even
  const uint64_t low = m & 0x7FFu;
  uint64_t mant = m >> 11;
  if (low > 0x400u || (low == 0x400u && (sticky || (mant & 1u)))) ++mant;
  const double v = std::ldexp(static_cast<double>(mant), static_cast<int>(msb - 52 + emin));
  *out = neg ? -v : v;
  return HY_OK;
}

hy_status hy_agg_float_sums(const uint64_t* records, uint64_t n_records, uint32_t words, uint32_t sum_word,
                            uint32_t n_limbs, int32_t emin, double* out) {
  if (n_records && (!records || !out)) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (sum_word + 2 + n_limbs > words) return fail(HY_ERR_INVALID_ARGUMENT, "sum words outside the record");
  for (uint64_t g = 0; g < n_records; ++g) {
    const uint64_t* r = records + g * words;
    const hy_status st = hy_agg_float_sum(r + sum_word + 2, n_limbs, emin, r[sum_word + 1], out + g);
    if (st != HY_OK) return st;
  }
  return HY_OK;
}

// Merge of partial aggregates (the multi-GPU Aggregate: each rank aggregates its chunk range, the ranks' records are
// all-gathered and merged here). Exact: counts and integer sums add; float sums add limb by limb in 128-bit and are
// carry-normalised back into the layout's limbs (the exact sum of the parts, so hy_agg_float_sum of the merged record
// equals that of a single-GPU aggregate over all rows); MIN / MAX take the extreme order-preserving bits of the parts
// with values; the first / last row words take the parts' row bases (global row numbering) and combine by min / max.
hy_status hy_aggregate_merge(const hy_agg_params* params, const hy_agg_layout* layout, const uint64_t* const* parts,
                             const uint64_t* part_groups, const uint64_t* part_row_base, uint32_t n_parts,
                             uint64_t* out, uint64_t out_capacity, uint64_t* n_out) {
  if (!params || !layout || !n_out || (n_parts && (!parts || !part_groups))) return fail(HY_ERR_INVALID_ARGUMENT, "null");
  const uint32_t W = layout->words, G = params->n_groupby;
  for (uint32_t a = 0; a < params->n_aggregates; ++a)
    if (params->aggregates[a].function == HY_AGG_COUNT_DISTINCT)
      return fail(HY_ERR_UNSUPPORTED, "COUNT(DISTINCT) partials cannot be merged from counts");
  std::vector<std::vector<uint64_t>> merged;
  std::vector<std::vector<__int128>> wide;  // per merged group: float-sum limbs summed in 128 bits
  std::unordered_map<std::string, size_t> index;
  for (uint32_t p = 0; p < n_parts; ++p) {
    const uint64_t base = part_row_base ? part_row_base[p] : 0;
    for (uint64_t g = 0; g < part_groups[p]; ++g) {
      const uint64_t* r = parts[p] + g * W;
      const std::string key(reinterpret_cast<const char*>(r), 8 * (G + 1));  // key words + NULL mask
      auto it = index.find(key);
      if (it == index.end()) {
        it = index.emplace(key, merged.size()).first;
        std::vector<uint64_t> m(r, r + W);
        m[G + 1] += base;
        m[G + 2] += base;
        merged.push_back(std::move(m));
        std::vector<__int128> wl;
        for (uint32_t a = 0; a < params->n_aggregates; ++a)
          for (uint32_t i = 0; i < layout->agg_limbs[a]; ++i)
            wl.push_back(static_cast<__int128>(static_cast<int64_t>(r[layout->agg_word[a] + 2 + i])));
        wide.push_back(std::move(wl));
        continue;
      }
      auto& m = merged[it->second];
      auto& wl = wide[it->second];
      m[G + 1] = std::min(m[G + 1], r[G + 1] + base);
      m[G + 2] = std::max(m[G + 2], r[G + 2] + base);
      m[G + 3] += r[G + 3];
      size_t li = 0;
      for (uint32_t a = 0; a < params->n_aggregates; ++a) {
        const int32_t f = params->aggregates[a].function;
        const uint32_t w = layout->agg_word[a];
        if (params->aggregates[a].column < 0) continue;  // COUNT(*): the rows word
        if (f == HY_AGG_COUNT) {
          m[w] += r[w];
        } else if (f == HY_AGG_MIN || f == HY_AGG_MAX) {
          if (r[w] != 0) {
            if (m[w] == 0)
              m[w + 1] = r[w + 1];
            else
              m[w + 1] = f == HY_AGG_MIN ? std::min(m[w + 1], r[w + 1]) : std::max(m[w + 1], r[w + 1]);
          }
          m[w] += r[w];
        } else if (layout->agg_limbs[a] == 0) {  // integer SUM / AVG
          m[w] += r[w];
          m[w + 1] += r[w + 1];
        } else {  // float SUM / AVG
          m[w] += r[w];
          m[w + 1] |= r[w + 1];
          for (uint32_t i = 0; i < layout->agg_limbs[a]; ++i)
            wl[li + i] += static_cast<__int128>(static_cast<int64_t>(r[w + 2 + i]));
        }
        li += layout->agg_limbs[a];
      }
    }
  }
  *n_out = merged.size();
  if (merged.size() > out_capacity) return fail(HY_ERR_CAPACITY, "merged groups exceed out_capacity");
  for (size_t g = 0; g < merged.size(); ++g) {
    auto& m = merged[g];
    size_t li = 0;
    for (uint32_t a = 0; a < params->n_aggregates; ++a) {
      const uint32_t n = layout->agg_limbs[a], w = layout->agg_word[a];
      __int128 carry = 0;
      for (uint32_t i = 0; i < n; ++i) {  // base-2^32 digits, the remaining carry in the top limb
        const __int128 t = carry + wide[g][li + i];
        if (i + 1 < n) {
          m[w + 2 + i] = static_cast<uint64_t>(t & 0xFFFFFFFF);
          carry = t >> 32;
        } else {
          m[w + 2 + i] = static_cast<uint64_t>(static_cast<int64_t>(t));
        }
      }
      li += n;
    }
    if (out) std::memcpy(out + g * W, m.data(), 8ull * W);
  }
  return HY_OK;
}

uint64_t hy_agg_decode_ordered(uint64_t o, int32_t value_type) {
  switch (value_type) {
    case HY_TYPE_INT32:
      return static_cast<uint32_t>(o) ^ 0x80000000u;
    case HY_TYPE_INT64:
      return o ^ (1ull << 63);
    case HY_TYPE_FLOAT: {
      const uint32_t b = static_cast<uint32_t>(o);
      return (b & 0x80000000u) ? (b & 0x7FFFFFFFu) : static_cast<uint32_t>(~b);
    }
    default:
      return (o >> 63) ? (o & ~(1ull << 63)) : ~o;
  }
}

}  // extern "C"
