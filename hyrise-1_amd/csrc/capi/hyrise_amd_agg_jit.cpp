// Plan-compiled dense aggregation (agg_jit.hpp). agg_dense_stream (kernels/aggregate_stream.hip) runs TPC-H 1 as an
// interpreter: the loaded columns' widths and encodings, the stage offsets, the chains' terms and the record words
// are read from the plan at run time, and the kernel spends ~1040 VALU and ~700 SALU instructions per 256-row step
// (PMC, profiles/r04_pmc_agg_dense_stream_v2_sq.txt) - most of them on that interpretation, on the SGPRs it pins
// (spilled to VGPR lanes: ~570 v_readlane in its code) and on uniform branches, not on the 80 double FMAs per step
// that accumulate. The kernel generated here is the same algorithm (same stage, decode tables, entry table, one-hot
// FMA accumulation, exactness per flush period, deferral of NULL / out-of-window steps to agg_dense_fused) with every
// plan constant a literal: straight-line code per column and per term, values in registers, no plan reads.
//
// Reference: Projection::_on_execute (projection.cpp:39-87) materialising the SELECT list, then Aggregate
// (aggregate.cpp:133-249, 291-498) summing it; the fused predicate is SingleColumnTableScanImpl's dictionary rewrite
// (single_column_table_scan_impl.cpp:145-205). Results are bit-identical to agg_dense_stream's (same exact sums).
#include "agg_jit.hpp"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <unistd.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <memory>
#include <mutex>
#include <sstream>
#include <unordered_map>
#include <vector>

#include "hyrise_amd.h"

namespace hyjit {

#include "agg_jit_prelude.inc"  // kJitPrelude: the text of kernels/agg_jit_prelude.hpp (Makefile)

static_assert(sizeof(hyj::ColumnChunk) == sizeof(hy_column_chunk), "ColumnChunk mirrors hy_column_chunk");
static_assert(offsetof(hyj::ColumnChunk, dictionary) == offsetof(hy_column_chunk, dictionary), "layout");
static_assert(offsetof(hyj::ColumnChunk, dictionary_size) == offsetof(hy_column_chunk, dictionary_size), "layout");
static_assert(offsetof(hyj::ColumnChunk, vid_width) == offsetof(hy_column_chunk, vid_width), "layout");
static_assert(sizeof(hyj::ScanChunk) == sizeof(hy_scan_chunk), "ScanChunk mirrors hy_scan_chunk");
static_assert(offsetof(hyj::ScanChunk, op) == offsetof(hy_scan_chunk, op), "layout");
static_assert(offsetof(hyj::ScanChunk, search_vid) == offsetof(hy_scan_chunk, search_vid), "layout");
static_assert(hyj::OP_EQ == HY_OP_EQ && hyj::OP_NE == HY_OP_NE && hyj::OP_LT == HY_OP_LT && hyj::OP_LE == HY_OP_LE &&
                  hyj::OP_GT == HY_OP_GT && hyj::OP_GE == HY_OP_GE && hyj::OP_ALL == HY_OP_ALL &&
                  hyj::OP_NONE == HY_OP_NONE && hyj::OP_IS_NOT_NULL == HY_OP_IS_NOT_NULL,
              "scan operators");

namespace {

std::string flt(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  char s[48];
  std::snprintf(s, sizeof(s), "__uint_as_float(0x%08xu)", b);
  return s;
}

// the wave's tile context: chunk, bounds, every loaded column's data (and dictionary size), the filter's range
void emit_load_ctx(std::ostringstream& o, const Shape& p, const char* tile_expr) {
  o << "    {\n      const uint32_t t_ = " << tile_expr << ";\n"
    << "      valid = t_ < n_tiles;\n"
    << "      if (valid) {\n"
    << "        tile = t_;\n        c = tile_chunk[t_];\n        size = chunk_size[c];\n"
    << "        base0 = static_cast<uint32_t>(t_ - chunk_tile_begin[c]) * TILE;\n"
    << "        n_steps = min(static_cast<uint32_t>(STEPS), (size - base0 + WAVE * R - 1) / (WAVE * R));\n";
  for (int li = 0; li < p.n_load; ++li) {
    o << "        d" << li << " = cols" << li << "[c].data;\n";
    if (p.dict[li]) o << "        ds" << li << " = cols" << li << "[c].dictionary_size;\n";
  }
  if (p.filtered)
    o << "        fdata = filt[c].column.data;\n"
      << "        fr = id_range(filt[c].op, filt[c].search_vid, filt[c].column.dictionary_size);\n";
  o << "      }\n    }\n";
}

void emit_issue(std::ostringstream& o, const Shape& p) {
  o << "    if (valid) {\n      const uint32_t ib = base0 + h * (WAVE * R);\n"
    << "      if (ib + WAVE * R <= size) {  // inside the chunk: uniform bases + shared lane offsets\n"
    << "        const uint32_t il = lane_id();\n";
  for (int li = 0; li < p.n_load; ++li)
    o << "        load_column_inside<" << p.width[li] << ">(d" << li << ", ib, il, stage + " << p.col_off[li] << "u);\n";
  if (p.filtered) o << "        load_column_inside<" << p.f_width << ">(fdata, ib, il, stage + " << p.filt_off << "u);\n";
  o << "      } else {  // the chunk's last step: pieces clamped to the chunk\n";
  for (int li = 0; li < p.n_load; ++li)
    o << "        load_column<" << p.width[li] << ">(d" << li << ", ib, size, stage + " << p.col_off[li] << "u);\n";
  if (p.filtered) o << "        load_column<" << p.f_width << ">(fdata, ib, size, stage + " << p.filt_off << "u);\n";
  o << "      }\n    }\n";
}

}  // namespace

std::string source(const Shape& p) {
  // waves per SIMD the kernel is compiled for: 3 (TPC-H 1 SF100, one box, alternating runs, profiles/r06_q1_jit_ab.txt:
  // 3 waves with per-group selects 3.84 ms; 2 waves 4.64, or 4.13 with the round-5 0/1 FMA form; 3 waves with the FMA
  // form 4.87 - 168 VGPRs, a few spilled, beat 181 at 2 waves). HY_AGG_JIT_WAVES: A/B
  static const int wpe = [] {
    const char* e = std::getenv("HY_AGG_JIT_WAVES");
    const int v = e ? std::atoi(e) : 3;
    return v >= 1 && v <= 8 ? v : 3;
  }();
  std::ostringstream o;
  const int H = p.n_gb, NS = p.n_sums, NA = NS > 0 ? NS : 1;
  const uint32_t stage = p.stage_bytes ? p.stage_bytes : 16u;
  const uint32_t ndt = p.n_dslots ? p.n_dslots : 1u;
  o << "#include \"agg_jit_prelude.hpp\"\nusing namespace hyj;\n"
    << "extern \"C\" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(" << wpe
    << "))) void agg_jit(JitArgs a) {\n"
    << "  constexpr uint32_t NONE = GROUPS;\n  constexpr int NA = " << NA << ";\n"
    << "  __shared__ __align__(16) unsigned char s_stage[WAVES][" << stage << "];\n"
    << "  __shared__ __align__(16) uint32_t s_dtab[WAVES][" << ndt << "][WAVE];\n"
    << "  __shared__ __align__(16) uint32_t s_entry[WAVES][CODES];\n"
    << "  __shared__ uint2 s_plist[WAVES][PLIST];\n"
    << "  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);\n"
    << "  unsigned char* const stage = &s_stage[w][0];\n"
    << "  uint32_t* const dtab = &s_dtab[w][0][0];\n"
    << "  uint32_t* const entry = &s_entry[w][0];\n"
    << "  uint2* const plist = &s_plist[w][0];\n"
    << "  const uint64_t n_tiles = a.n_tiles;\n"
    << "  const uint32_t* const tile_chunk = a.tile_chunk;\n"
    << "  const uint64_t* const chunk_tile_begin = a.chunk_tile_begin;\n"
    << "  const uint32_t* const chunk_size = a.chunk_size;\n"
    << "  const uint64_t* const chunk_row_begin = a.chunk_row_begin;\n"
    << "  unsigned long long* const records = a.records;\n"
    << "  uint32_t* const error = a.error;\n"
    << "  uint32_t* const deferred = a.deferred;\n"
    << "  uint32_t* const n_deferred = a.n_deferred;\n";
  for (int li = 0; li < p.n_load; ++li) o << "  const ColumnChunk* const cols" << li << " = a.cols[" << li << "];\n";
  if (p.filtered) o << "  const ScanChunk* const filt = a.filter;\n";
  o << "  double acc[GROUPS][NA];\n  uint32_t cnt[GROUPS], lo[GROUPS], hi[GROUPS];\n  int32_t tab[GROUPS];\n"
    << "  float emax[NA];\n  uint32_t emin[NA];\n"
    << "#pragma unroll\n  for (int j = 0; j < GROUPS; ++j) {\n    tab[j] = -1;\n    cnt[j] = 0;\n"
    << "    lo[j] = 0xFFFFFFFFu;\n    hi[j] = 0;\n#pragma unroll\n    for (int s = 0; s < NA; ++s) acc[j][s] = 0.0;\n  }\n"
    << "#pragma unroll\n  for (int s = 0; s < NA; ++s) {\n    emax[s] = 0.f;\n    emin[s] = 0xFFFFFFFFu;\n  }\n"
    << "  entry[lane_id()] = NONE;\n  uint32_t n_period = 0, n_plist = 0;\n"
    << "  const uint32_t GW = gridDim.x * WAVES;\n"
    << "  bool valid = false;\n  uint32_t tile = 0, c = 0, size = 0, base0 = 0, n_steps = 0;\n";
  for (int li = 0; li < p.n_load; ++li) {
    o << "  const void* d" << li << " = nullptr;\n";
    if (p.dict[li]) o << "  uint32_t ds" << li << " = 0;\n";
  }
  if (p.filtered) o << "  const void* fdata = nullptr;\n  IdRange fr{0u, 0u, 0u, 0u};\n";
  o << "  uint32_t h = 0;\n";
  emit_load_ctx(o, p, "blockIdx.x * WAVES + static_cast<uint32_t>(w)");
  emit_issue(o, p);
  o << "  bool period_full = false;\n"
    << "  for (;;) {\n"
    << "    const bool done = !valid;\n"
    << "    const uint32_t tile_s = tile, step = h, c_s = c;\n"
    << "    const uint32_t base = base0 + h * (WAVE * R);\n"
    << "    const uint32_t lane = lane_id();\n"
    << "    const uint32_t first = base + lane * R;\n"
    << "    uint32_t act = 0, vnull = 0, g[R] = {0, 0, 0, 0};\n    uint32_t rowv = 0;\n";
  for (int li = H; li < p.n_load; ++li) o << "    uint32_t v" << li << "[R] = {0, 0, 0, 0};\n";
  o << "    if (!done) {\n"
    << "      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
    << "      if (h == 0) {  // the tile's decode tables\n";
  for (int li = 0; li < p.n_load; ++li) {
    if (!p.dict[li]) continue;
    o << "        if (ds" << li << " != 0) {\n"
      << "          uint32_t v = reinterpret_cast<const uint32_t*>(cols" << li << "[c].dictionary)[min(lane_id(), ds" << li
      << " - 1u)];\n";
    if (li < H)
      o << "          const bool ent = lane_id() < ds" << li << ";\n"
        << "          if (__ballot(ent && v >= " << p.gb_domain[li] << "u) != 0ull && lane_id() == 0) atomicOr(error, 2u);\n"
        << "          v = ent ? min(v, " << p.gb_domain[li] << "u) : " << p.gb_domain[li] << "u;\n";
    o << "          dtab[" << p.dict_slot[li] << " * WAVE + lane_id()] = v;\n        }\n";
  }
  o << "      }\n"
    << "      rowv = static_cast<uint32_t>(chunk_row_begin[c]) + first;\n"
    << "      act = base + WAVE * R <= size ? 0xFu : 0u;\n"
    << "      if (!act) {\n#pragma unroll\n        for (int k = 0; k < R; ++k) act |= static_cast<uint32_t>(first + k < size) << k;\n      }\n";
  if (p.filtered)
    o << "      {\n        uint32_t ids[R];\n        read4<" << p.f_width << ">(stage + " << p.filt_off << "u, lane, ids);\n"
      << "#pragma unroll\n        for (int k = 0; k < R; ++k) act &= ~(static_cast<uint32_t>(!id_in_range(fr, ids[k])) << k);\n      }\n";
  o << "      bool bad_code = false;\n";
  for (int li = 0; li < p.n_load; ++li) {
    const bool gb = li < H;
    o << "      {\n        uint32_t v[R];\n        read4<" << p.width[li] << ">(stage + " << p.col_off[li] << "u, lane, v);\n";
    if (p.dict[li]) {
      o << "        const uint32_t* tb = dtab + " << p.dict_slot[li] << " * WAVE;\n"
        << "#pragma unroll\n        for (int k = 0; k < R; ++k) {\n";
      if (!gb) o << "          vnull |= static_cast<uint32_t>(v[k] >= ds" << li << ") << k;\n";
      o << "          v[k] = tb[min(v[k], static_cast<uint32_t>(DICT_MAX))];\n        }\n";
    }
    if (gb) {
      if (!p.dict[li])
        o << "#pragma unroll\n        for (int k = 0; k < R; ++k) {\n"
          << "          bad_code = bad_code || (v[k] >= " << p.gb_domain[li] << "u && ((act >> k) & 1u));\n"
          << "          v[k] = min(v[k], " << p.gb_domain[li] << "u);\n        }\n";
      o << "#pragma unroll\n        for (int k = 0; k < R; ++k) g[k] += v[k] * " << p.gb_stride[li] << "u;\n";
    } else {
      o << "#pragma unroll\n        for (int k = 0; k < R; ++k) v" << li << "[k] = v[k];\n";
    }
    o << "      }\n";
  }
  o << "      if (__ballot(bad_code) != 0ull && lane_id() == 0) atomicOr(error, 2u);\n"
    << "      asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");  // the stage is read: the next loads may land\n"
    << "      if (h + 1 < n_steps) {\n        ++h;\n      } else {\n";
  emit_load_ctx(o, p, "tile + GW");
  o << "        h = 0;\n      }\n";
  emit_issue(o, p);
  o << "    }\n"
    << "    const bool active = !done && __ballot(act != 0) != 0ull;\n"
    << "    const uint32_t step_id = tile_s * STEPS + step;\n"
    // (B) group codes -> table entries
    << "    uint32_t e[R];\n    bool unmapped = false;\n"
    << "#pragma unroll\n    for (int k = 0; k < R; ++k) {\n      const bool ak = (act >> k) & 1u;\n"
    << "      const uint32_t ek = entry[min(g[k], static_cast<uint32_t>(CODES - 1))];\n"
    << "      e[k] = ak ? ek : NONE;\n"
    << "      unmapped = unmapped || (ak && e[k] == NONE);\n    }\n"
    << "    const bool remap = active && __ballot(unmapped) != 0ull;\n"
    << "    uint64_t present = 0, need = 0;\n    bool refill = false;\n"
    << "    if (remap) {\n      uint64_t mine = 0;\n"
    << "#pragma unroll\n      for (int k = 0; k < R; ++k) mine |= ((act >> k) & 1u) ? (1ull << (g[k] & 63u)) : 0ull;\n"
    << "      present = uniform64(wave_or64(mine));\n      uint64_t have = 0;\n      int free_slots = 0;\n"
    << "#pragma unroll\n      for (int j = 0; j < GROUPS; ++j) {\n        if (tab[j] >= 0) have |= 1ull << tab[j];\n"
    << "        else ++free_slots;\n      }\n      need = present & ~have;\n"
    << "      refill = __popcll(need) > free_slots;\n    }\n";
  // the flush (one site): exactness of the period, then the entries' rows and sums into their records
  o << "    if (done || period_full || refill) {\n"
    << "      const int lane = __lane_id();\n      int32_t fb[NA];\n      bool exact = true;\n";
  for (int s = 0; s < NA; ++s) {
    o << "      fb[" << s << "] = 1;\n";
    if (s < NS && p.sum_kind[s] == 1)
      o << "      {\n        bool nan = false;\n"
        << "#pragma unroll\n        for (int j = 0; j < GROUPS; ++j) nan = nan || acc[j][" << s << "] != acc[j][" << s << "];\n"
        << "        if (__ballot(nan) != 0ull) exact = false;\n"
        << "        const uint32_t hb = wave_max_u(__float_as_uint(emax[" << s << "]));\n"
        << "        if (hb != 0) {\n          const int e_hi = static_cast<int>(hb >> 23);\n"
        << "          const int e_lo = max(static_cast<int>((wave_min_u(emin[" << s << "]) + 1u) >> 24), 1);\n"
        << "          fb[" << s << "] = __builtin_amdgcn_readfirstlane(e_lo);\n"
        << "          if (e_hi >= 0xFF || e_hi - e_lo > WINDOW || e_lo > BASE_MAX) exact = false;\n        }\n      }\n";
  }
  o << "      if (!exact) {  // discard the period: its steps go to agg_dense_fused\n"
    << "        for (uint32_t i = 0; i < n_plist; ++i) {\n          const uint2 pe = plist[i];\n"
    << "          if (static_cast<uint32_t>(lane) < STEPS && ((pe.y >> lane) & 1u)) {\n"
    << "            const uint32_t q = atomicAdd(n_deferred, 1u);\n"
    << "            deferred[q] = pe.x * STEPS + static_cast<uint32_t>(lane);\n          }\n        }\n      }\n"
    << "#pragma unroll\n      for (int j = 0; j < GROUPS; ++j) {\n"
    << "        if (tab[j] < 0) continue;\n"
    << "        unsigned long long* rec = records + static_cast<uint64_t>(tab[j]) * " << p.words << "u;\n"
    << "        const unsigned long long rows = exact ? wave_sum64(cnt[j]) : 0ull;\n"
    << "        const uint32_t frow = exact ? lo[j] : 0u;\n"
    << "        const uint32_t last1 = exact ? wave_max_u(hi[j]) : 0u;\n"
    << "        cnt[j] = 0;\n        lo[j] = 0xFFFFFFFFu;\n        hi[j] = 0;\n"
    << "        if (rows && lane == 0) {\n"
    << "          atomicAdd(rec + " << H << " + HDR_ROWS, rows);\n"
    << "          atomicMin(rec + " << H << " + HDR_FIRST, static_cast<unsigned long long>(frow));\n"
    << "          atomicMax(rec + " << H << " + HDR_LAST, static_cast<unsigned long long>(last1 - 1u));\n";
  for (int f = 0; f < p.n_cnt; ++f) o << "          atomicAdd(rec + " << p.cnt_word[f] << ", rows);\n";
  o << "        }\n";
  for (int s = 0; s < NS; ++s) {
    o << "        {\n          const double av = acc[j][" << s << "];\n          acc[j][" << s << "] = 0.0;\n";
    if (p.sum_kind[s] != 0) {
      o << "          if (exact && __ballot(av != 0.0) != 0ull) {\n";
      if (p.sum_kind[s] == 1)
        o << "            const double units = ldexp(av, 150 - fb[" << s << "]);\n";
      else
        o << "            const double units = av;\n";
      o << "            const int64_t tot = static_cast<int64_t>(wave_sum64(static_cast<uint64_t>(static_cast<int64_t>(units))));\n"
        << "            if (lane == 0) {\n";
      for (int q = 0; q < p.sum_nfn[s]; ++q) {
        if (p.sum_kind[s] == 1)
          o << "              add_scaled(rec + " << p.sum_word[s][q] + 2 << ", " << p.sum_limbs[s] << ", tot, fb[" << s
            << "] - 1);\n";
        else
          o << "              atomicAdd(rec + " << p.sum_word[s][q] + 1 << ", static_cast<unsigned long long>(tot));\n";
      }
      o << "            }\n          }\n";
    }
    o << "        }\n";
  }
  o << "      }\n"
    << "#pragma unroll\n      for (int s = 0; s < NA; ++s) {\n        emax[s] = 0.f;\n        emin[s] = 0xFFFFFFFFu;\n      }\n"
    << "      n_period = 0;\n      n_plist = 0;\n    }\n"
    << "    period_full = false;\n    if (done) break;\n    if (!active) continue;\n"
    << "    if (remap) {\n      if (refill) {\n"
    << "#pragma unroll\n        for (int j = 0; j < GROUPS; ++j) {\n"
    << "          if (tab[j] >= 0 && lane_id() == 0) entry[tab[j]] = NONE;\n          tab[j] = -1;\n        }\n"
    << "        need = present;\n      }\n"
    << "      if (__popcll(need) > GROUPS) {\n        defer_step(a, step_id);\n        continue;\n      }\n"
    << "#pragma unroll\n      for (int j = 0; j < GROUPS; ++j) {\n        if (tab[j] < 0 && need) {\n"
    << "          tab[j] = __builtin_ctzll(need);\n          need &= need - 1;\n"
    << "          if (lane_id() == 0) entry[tab[j]] = static_cast<uint32_t>(j);\n        }\n      }\n"
    << "#pragma unroll\n      for (int k = 0; k < R; ++k) {\n        e[k] = NONE;\n"
    << "#pragma unroll\n        for (int j = 0; j < GROUPS; ++j)\n"
    << "          e[k] = ((act >> k) & 1u) && g[k] == static_cast<uint32_t>(tab[j]) ? static_cast<uint32_t>(j) : e[k];\n"
    << "      }\n    }\n"
    << "    if (__ballot((vnull & act) != 0) != 0ull) {  // NULLs in the other loaded columns\n"
    << "      defer_step(a, step_id);\n      continue;\n    }\n"
    << "    uint32_t onehot = 0;\n"
    << "#pragma unroll\n    for (int k = 0; k < R; ++k) onehot |= 1u << (e[k] * 4u + static_cast<uint32_t>(k));\n";
  // HY_AGG_JIT_SELECT=0 (A/B): the round-5 form, one FMA per group with a 0/1 double per row and group
  static const bool select = [] {
    const char* e = std::getenv("HY_AGG_JIT_SELECT");
    return !(e && std::strtol(e, nullptr, 10) == 0);
  }();
  if (!select)
    o << "    double m[R][GROUPS];\n"
      << "#pragma unroll\n    for (int k = 0; k < R; ++k)\n#pragma unroll\n      for (int j = 0; j < GROUPS; ++j) "
         "m[k][j] = (onehot >> (4 * j + k)) & 1u ? 1.0 : 0.0;\n";
  // (C) the sums: chains straight-line, then (D) their accumulation
  for (int s = 0; s < NS; ++s) {
    const int kind = p.sum_kind[s];
    if (kind == 0) continue;
    o << "    {  // sum " << s << "\n      float rf[R] = {0.f, 0.f, 0.f, 0.f};\n      uint32_t ri[R] = {0u, 0u, 0u, 0u};\n";
    for (int t = 0; t < p.sum_len[s]; ++t) {
      const Term& tm = p.terms[p.sum_first[s] + t];
      if (kind == 2) {  // a plain int32 column
        o << "#pragma unroll\n      for (int k = 0; k < R; ++k) ri[k] = v" << tm.col << "[k];\n";
        break;
      }
      o << "      {\n        float tv[R];\n#pragma unroll\n        for (int k = 0; k < R; ++k) {\n";
      if (tm.flags & 16)
        o << "          const float x = 0.f;\n";
      else if (tm.flags & 8)
        o << "          const float x = static_cast<float>(static_cast<int32_t>(v" << tm.col << "[k]));\n";
      else
        o << "          const float x = __uint_as_float(v" << tm.col << "[k]);\n";
      o << "          tv[k] = __builtin_fmaf(x, " << flt(tm.a) << ", " << flt(tm.b) << ");\n        }\n"
        << "#pragma unroll\n        for (int k = 0; k < R; ++k) ";
      switch (t == 0 ? 0 : (tm.flags & 7)) {
        case 0: o << "rf[k] = tv[k];\n"; break;
        case 1: o << "rf[k] = rf[k] + tv[k];\n"; break;
        case 2: o << "rf[k] = rf[k] - tv[k];\n"; break;
        case 3: o << "rf[k] = tv[k] - rf[k];\n"; break;
        default: o << "rf[k] = rf[k] * tv[k];\n"; break;
      }
      o << "      }\n";
    }
    if (kind == 1)
      o << "      emax[" << s << "] = fmaxf(emax[" << s << "], fmaxf(fmaxf(fabsf(rf[0]), fabsf(rf[1])), fmaxf(fabsf(rf[2]), fabsf(rf[3]))));\n"
        << "#pragma unroll\n      for (int k = 0; k < R; ++k) emin[" << s << "] = min(emin[" << s
        << "], (__float_as_uint(rf[k]) << 1) - 1u);\n";
    o << "#pragma unroll\n      for (int k = 0; k < R; ++k) {\n"
      << "        const double xv = " << (kind == 2 ? "static_cast<double>(static_cast<int32_t>(ri[k]))" : "static_cast<double>(rf[k])")
      << ";\n#pragma unroll\n        for (int j = 0; j < GROUPS; ++j) acc[j][" << s << "] = ";
    if (select)  // the row's value added to its group's accumulator only (no 0/1 doubles in registers)
      o << "(onehot >> (4 * j + k)) & 1u ? acc[j][" << s << "] + xv : acc[j][" << s << "];\n      }\n    }\n";
    else
      o << "__builtin_fma(m[k][j], xv, acc[j][" << s << "]);\n      }\n    }\n";
  }
  o << "#pragma unroll\n    for (int j = 0; j < GROUPS; ++j) {\n"
    << "      const uint32_t mb = (onehot >> (4 * j)) & 0xFu;\n"
    << "      cnt[j] += static_cast<uint32_t>(__popc(mb));\n"
    << "      hi[j] = mb ? rowv + static_cast<uint32_t>(31 - __builtin_clz(mb)) + 1u : hi[j];\n"
    << "      if (lo[j] == 0xFFFFFFFFu && __ballot(mb != 0) != 0ull)\n"
    << "        lo[j] = __builtin_amdgcn_readfirstlane(wave_min_u(mb ? rowv + static_cast<uint32_t>(__builtin_ctz(mb)) : 0xFFFFFFFFu));\n"
    << "    }\n"
    << "    if (n_plist == 0 || plist[n_plist - 1].x != tile_s) {\n"
    << "      if (lane_id() == 0) plist[n_plist] = make_uint2(tile_s, 1u << step);\n      ++n_plist;\n"
    << "    } else if (lane_id() == 0) {\n      plist[n_plist - 1].y |= 1u << step;\n    }\n"
    << "    period_full = ++n_period >= FLUSH_STEPS || n_plist >= PLIST;\n"
    << "    (void)c_s;\n"
    << "  }\n}\n";
  return o.str();
}

namespace {

// hiprtc of one generated source into a code object for `arch`; empty on failure (log in *err)
std::vector<char> rtc(const std::string& src, const std::string& arch, std::string* err) {
  hiprtcProgram prog;
  const char* headers[] = {kJitPrelude};
  const char* names[] = {"agg_jit_prelude.hpp"};
  if (hiprtcCreateProgram(&prog, src.c_str(), "agg_jit.hip", 1, headers, names) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return {};
  }
  const std::string a = "--offload-arch=" + arch;
  const char* opts[] = {a.c_str(), "-O3", "-ffp-contract=off", "-std=c++17"};
  if (hiprtcCompileProgram(prog, 4, opts) != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    *err = "hiprtc: " + log.substr(0, 4000);
    hiprtcDestroyProgram(&prog);
    return {};
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return code;
}

// Code objects persist on disk, keyed by a hash of the target and the generated source: a plan shape pays hiprtc's
// ~1.7 s once per machine and library build instead of once per process. The directory is jit_cache/ next to this
// library (HY_JIT_CACHE_DIR overrides it, HY_JIT_CACHE=0 turns the cache off); entries are written to a temporary file
// and renamed, so concurrent processes never read a partial one, and an entry that fails to load is recompiled.
uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

std::string cache_dir() {
  if (const char* e = std::getenv("HY_JIT_CACHE")) {
    if (std::strtol(e, nullptr, 10) == 0) return {};
  }
  if (const char* d = std::getenv("HY_JIT_CACHE_DIR")) return d;
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&fnv1a), &info) == 0 || !info.dli_fname) return {};
  std::string lib = info.dli_fname;
  const size_t slash = lib.rfind('/');
  return (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/jit_cache";
}

std::string cache_path(const std::string& src, const std::string& arch) {
  const std::string dir = cache_dir();
  if (dir.empty()) return {};
  char name[64];
  std::snprintf(name, sizeof(name), "/agg_jit_%016llx.co",
                static_cast<unsigned long long>(fnv1a(src, fnv1a(arch + "\n" + std::string(kJitPrelude)))));
  return dir + name;
}

std::vector<char> cache_load(const std::string& path) {
  if (path.empty()) return {};
  std::ifstream f(path, std::ios::binary);
  if (!f) return {};
  return std::vector<char>(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

void cache_store(const std::string& path, const std::vector<char>& code) {
  if (path.empty() || code.empty()) return;
  const std::string dir = path.substr(0, path.rfind('/'));
  (void)std::system(("mkdir -p '" + dir + "' 2>/dev/null").c_str());
  const std::string tmp = path + ".tmp" + std::to_string(static_cast<long>(getpid()));
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(code.data(), static_cast<std::streamsize>(code.size()));
    if (!f) return;
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

struct Compiled {
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
  int resident = 0;  // workgroups resident at once (occupancy x CUs)
  std::string error;
};

std::mutex g_m;
std::unordered_map<std::string, std::shared_ptr<Compiled>>& cache() {
  static auto* c = new std::unordered_map<std::string, std::shared_ptr<Compiled>>;  // (leaked: outlives HIP teardown)
  return *c;
}

std::shared_ptr<Compiled> compile(const std::string& src) {
  auto out = std::make_shared<Compiled>();
  int dev = 0;
  hipDeviceProp_t prop{};
  std::string arch = "gfx950";
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.gcnArchName[0])
    arch = prop.gcnArchName;
  const std::string path = cache_path(src, arch);
  std::vector<char> code = cache_load(path);
  bool cached = !code.empty();
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (code.empty()) {
      code = rtc(src, arch, &out->error);
      if (code.empty()) return out;
      cached = false;
    }
    if (hipModuleLoadData(&out->module, code.data()) == hipSuccess &&
        hipModuleGetFunction(&out->fn, out->module, "agg_jit") == hipSuccess)
      break;
    (void)hipGetLastError();
    out->fn = nullptr;
    out->error = "hipModuleLoadData / hipModuleGetFunction failed";
    if (!cached) return out;
    code.clear();  // a stale or damaged cache entry: compile it again
  }
  if (!out->fn) return out;
  out->error.clear();
  if (!cached) cache_store(path, code);
  int per_cu = 0, cus = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, out->fn, 256, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    per_cu = 3, cus = 256;
  out->resident = std::max(1, per_cu) * std::max(1, cus);
  return out;
}

}  // namespace

bool launch(const Shape& shape, const hyj::JitArgs& args, hipStream_t s, std::string* err) {
  const std::string src = source(shape);
  std::shared_ptr<Compiled> k;
  {
    std::lock_guard<std::mutex> lock(g_m);  // (one compile per source; concurrent callers of the same plan wait)
    auto& c = cache();
    auto it = c.find(src);
    if (it == c.end()) it = c.emplace(src, compile(src)).first;
    k = it->second;
  }
  if (!k->fn) {
    if (err) *err = k->error;
    return false;
  }
  const uint64_t want = (args.n_tiles + hyj::WAVES - 1) / hyj::WAVES;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want, uint64_t(k->resident))));
  hyj::JitArgs a = args;
  size_t bytes = sizeof(a);
  void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes, HIP_LAUNCH_PARAM_END};
  if (hipModuleLaunchKernel(k->fn, grid, 1, 1, 256, 1, 1, 0, s, nullptr, config) != hipSuccess) {
    if (err) *err = "hipModuleLaunchKernel failed";
    return false;
  }
  return true;
}

bool compile_only(const Shape& shape, const std::string& arch, std::string* err) {
  return !rtc(source(shape), arch, err).empty();
}

}  // namespace hyjit

// Internal self-test (not part of include/hyrise_amd.h; tests/test_agg_jit.py): generates the kernel for a TPC-H-1
// shaped plan - two dictionary group-by columns, three dictionary and one float value column, a u16 dictionary
// filter, five sums with + - * chains - and compiles it with hiprtc for gfx950, without a GPU. Returns 0 on success;
// the compiler log (or the source with `want_source`) goes to buf.
extern "C" int hy_internal_agg_jit_selftest(int want_source, char* buf, size_t n) {
  hyjit::Shape p;
  p.n_gb = 2;
  p.n_load = 6;
  p.n_sums = 5;
  p.words = 30;
  const int dict[] = {1, 1, 1, 0, 1, 1}, width[] = {1, 1, 1, 4, 1, 1};
  for (int li = 0; li < 6; ++li) {
    p.dict[li] = dict[li];
    p.width[li] = width[li];
    p.col_off[li] = li < 3 ? 256u * li : li == 3 ? 768u : 1792u + 256u * (li - 4);
    p.dict_slot[li] = li < 3 ? li : li == 3 ? 0xFFFFFFFFu : li - 1;
  }
  p.gb_domain[0] = 3, p.gb_stride[0] = 3, p.gb_domain[1] = 2, p.gb_stride[1] = 1;
  p.filtered = 1, p.f_width = 2, p.filt_off = 2304, p.stage_bytes = 2816, p.n_dslots = 5;
  // qty; price; price * (1 - disc); price * (1 - disc) * (1 + tax); disc
  const hyjit::Term T[] = {{1.f, -0.f, 2, 0}, {1.f, -0.f, 3, 0}, {1.f, -0.f, 3, 0}, {-1.f, 1.f, 4, 4},
                           {1.f, -0.f, 3, 0}, {-1.f, 1.f, 4, 4}, {1.f, 1.f, 5, 4}, {1.f, -0.f, 4, 0}};
  const int first[] = {0, 1, 2, 4, 7}, len[] = {1, 1, 2, 3, 1};
  for (int i = 0; i < 8; ++i) p.terms[i] = T[i];
  for (int q = 0; q < 5; ++q) {
    p.sum_kind[q] = 1;
    p.sum_first[q] = first[q];
    p.sum_len[q] = len[q];
    p.sum_nfn[q] = 1;
    p.sum_word[q][0] = 6u + 12u * static_cast<uint32_t>(q);
    p.sum_limbs[q] = 9;
  }
  p.n_cnt = 1;
  p.cnt_word[0] = 6;
  std::string out;
  int rc = 0;
  if (want_source) {
    out = hyjit::source(p);
  } else if (!hyjit::compile_only(p, "gfx950", &out)) {
    rc = 1;
  }
  if (buf && n) {
    std::strncpy(buf, out.c_str(), n - 1);
    buf[n - 1] = '\0';
  }
  return rc;
}
