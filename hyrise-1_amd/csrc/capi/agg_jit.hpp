// Plan-compiled dense aggregation (hyrise_amd_agg_jit.cpp): agg_dense_stream's algorithm with the plan's shape - the
// loaded columns' encodings and widths, the stage layout, the group-code strides, the sums' FMA-form chains and the
// record words - compiled into the kernel by hiprtc, so that the kernel interprets nothing at run time.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../kernels/agg_jit_prelude.hpp"

namespace hyjit {

constexpr int MAX_SUMS = 8;
constexpr int MAX_TERMS = 36;
constexpr int MAX_FNS = 2;
constexpr int MAX_CNT = 16;

struct Term {  // hyk::StreamTerm: term = fma(x, a, b), then combined into the running value
  float a, b;
  int32_t col;
  int32_t flags;  // 0 set, 1 add, 2 sub, 3 reverse sub, 4 mul; | 8 int32 -> float; | 16 literal (x = 0)
};

struct Shape {
  int32_t n_gb = 0, n_load = 0, n_sums = 0;
  uint32_t words = 0;
  int32_t dict[hyj::MAX_COLS] = {};   // every chunk of column li is DICT (1) / VALUE (0)
  int32_t width[hyj::MAX_COLS] = {};  // its element width in every chunk (1, 2, 4)
  uint32_t col_off[hyj::MAX_COLS] = {}, dict_slot[hyj::MAX_COLS] = {};
  uint32_t gb_domain[hyj::MAX_COLS] = {}, gb_stride[hyj::MAX_COLS] = {};
  int32_t filtered = 0, f_width = 0;
  uint32_t filt_off = 0, stage_bytes = 0, n_dslots = 0;
  int32_t sum_kind[MAX_SUMS] = {};  // 0 none (count only), 1 float chain, 2 int32 column
  int32_t sum_first[MAX_SUMS] = {}, sum_len[MAX_SUMS] = {};
  Term terms[MAX_TERMS] = {};
  int32_t sum_nfn[MAX_SUMS] = {};
  uint32_t sum_word[MAX_SUMS][MAX_FNS] = {};
  int32_t sum_limbs[MAX_SUMS] = {};
  int32_t n_cnt = 0;
  uint32_t cnt_word[MAX_CNT] = {};
};

// The kernel's source for a shape (exposed for tests).
std::string source(const Shape& shape);
// Compiles (once per distinct source, process-wide cache) and launches over n_tiles tiles on stream s. False, with
// the reason in *err, when the kernel cannot be compiled or launched (the caller then runs agg_dense_stream).
bool launch(const Shape& shape, const hyj::JitArgs& args, hipStream_t s, std::string* err);
// hiprtc only (no device needed): false with the compiler log in *err
bool compile_only(const Shape& shape, const std::string& arch, std::string* err);

}  // namespace hyjit
