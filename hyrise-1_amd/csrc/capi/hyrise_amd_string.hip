// TableScans over std::string columns held on the device (include/hyrise_amd.h, "String scans"): unencoded
// ValueColumn<std::string> chunks as packed string arrays (offsets + bytes), next to dictionary chunks.
//
// Reference: SingleColumnTableScanImpl::handle_column on a ValueColumn<std::string> (single_column_table_scan_impl.cpp:
// 38-85: the comparator of type_comparison.hpp:100-123 between the row's std::string and type_cast<std::string>(value),
// i.e. std::string::compare, bytes as unsigned char), LikeTableScanImpl on a value column (like_table_scan_impl.cpp:
// 22-31, 86-97) with the LikeMatcher (like_matcher.cpp:9-118), and IsNullTableScanImpl for string value columns.
// Dictionary chunks keep the host's dictionary rewrite (op + search_vid, or the LIKE id set) exactly as hy_table_scan.
//
// LIKE on the device: the pattern compiles (on the host, per call) to a bit-parallel NFA over up to 1023 positions
// (one 64-bit word per 64 of them; patterns of up to 63 positions take a one-word fast path) - per position a byte
// set (a literal byte, '_' = any byte, a [...] class of the regex path) or a '%' star; per input byte c:
// S = ((S & lit[c]) << 1) | (S & star & star_ok[c]), then the star closure S |= (S & star) << 1. The
// reference's simple patterns ('abc%', '%abc', '%abc%', '%a%b%...%') are plain string searches: their '%' and '_'
// match any byte. Other patterns take the reference's regex path (pattern -> ECMAScript '^...$', every regex special
// escaped except '[' ']'): '_' and '%' become '.', which does not match '\n' or '\r', and [...] is a class.
//
// One flag launch evaluates every row (one thread per row, 256-row tiles never straddle chunks) and writes a flag and
// the row's output item; one order-preserving compaction (hipcub DeviceSelect::Flagged) yields the matches in row
// order. Not a headline path: string rows are read once, the flag/item pass adds 9-13 B per row.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <string>
#include <vector>

#include "hyrise_amd.h"
#include "capi_common.hpp"
#include "../kernels/common.hpp"

using namespace hyc;

namespace {

constexpr int STR_THREADS = 256;
constexpr int LIKE_MAX_WORDS = 16;                           // 64-bit state words of the NFA
constexpr int LIKE_MAX_POSITIONS = 64 * LIKE_MAX_WORDS - 1;  // 1023 positions (+ the accept bit)

// The compiled LIKE pattern (device copy in the workspace): a bitset NFA of `words` 64-bit words, position j in bit
// j % 64 of word j / 64.
struct LikeNfa {
  uint64_t lit[256][LIKE_MAX_WORDS];      // bit j: position j accepts byte c
  uint64_t star_ok[256][LIKE_MAX_WORDS];  // bit j: star position j may consume byte c
  uint64_t star[LIKE_MAX_WORDS];          // star positions
  uint64_t accept[LIKE_MAX_WORDS];        // bit m
  uint64_t start[LIKE_MAX_WORDS];         // closure of position 0
  uint32_t words;
};

struct StrPred {
  const char* value;  // device copy of the constant
  uint32_t value_len;
  const LikeNfa* nfa;  // null: no LIKE pattern
};

__host__ __device__ inline uint64_t star_closure(uint64_t s, uint64_t star) {
  for (;;) {
    const uint64_t n = s | ((s & star) << 1);
    if (n == s) return s;
    s = n;
  }
}

// The closure over a state of several words: a star position's successor is active too (carries cross words).
__host__ __device__ inline void star_closure_words(uint64_t (&s)[LIKE_MAX_WORDS], const uint64_t* star, uint32_t words) {
  for (bool changed = true; changed;) {
    changed = false;
    uint64_t carry = 0;
#pragma unroll
    for (int w = 0; w < LIKE_MAX_WORDS; ++w) {
      if (w >= static_cast<int>(words)) break;
      const uint64_t t = s[w] & star[w];
      const uint64_t n = s[w] | (t << 1) | carry;
      carry = t >> 63;
      changed |= n != s[w];
      s[w] = n;
    }
  }
}

__device__ inline bool like_match(const LikeNfa& a, const unsigned char* p, uint32_t n) {
  if (a.words == 1) {  // patterns of up to 63 positions: one word
    uint64_t s = a.start[0];
    for (uint32_t i = 0; i < n && s; ++i) {
      const unsigned c = p[i];
      s = star_closure(((s & a.lit[c][0]) << 1) | (s & a.star[0] & a.star_ok[c][0]), a.star[0]);
    }
    return (s & a.accept[0]) != 0;
  }
  uint64_t s[LIKE_MAX_WORDS];
#pragma unroll
  for (int w = 0; w < LIKE_MAX_WORDS; ++w) s[w] = w < static_cast<int>(a.words) ? a.start[w] : 0;
  for (uint32_t i = 0; i < n; ++i) {
    const unsigned c = p[i];
    uint64_t carry = 0, any = 0;
#pragma unroll
    for (int w = 0; w < LIKE_MAX_WORDS; ++w) {
      if (w >= static_cast<int>(a.words)) break;
      const uint64_t adv = s[w] & a.lit[c][w];
      s[w] = (adv << 1) | carry | (s[w] & a.star[w] & a.star_ok[c][w]);
      carry = adv >> 63;
      any |= s[w];
    }
    if (!any) return false;
    star_closure_words(s, a.star, a.words);
  }
  uint64_t hit = 0;
#pragma unroll
  for (int w = 0; w < LIKE_MAX_WORDS; ++w)
    if (w < static_cast<int>(a.words)) hit |= s[w] & a.accept[w];
  return hit != 0;
}

// The predicate on one string value (NULL or not): compare with the constant, LIKE, IS [NOT] NULL.
__device__ inline bool string_value_match(int op, bool is_null, const hyk::DevString& v, const StrPred& p) {
  if (op == HY_OP_IS_NULL) return is_null;
  if (is_null) return false;
  if (op == HY_OP_ALL || op == HY_OP_IS_NOT_NULL) return true;
  if (op == HY_OP_LIKE || op == HY_OP_NOT_LIKE) return like_match(*p.nfa, v.p, v.n) == (op == HY_OP_LIKE);
  return hyk::cmp_result(op, hyk::string_compare(v, hyk::DevString{reinterpret_cast<const unsigned char*>(p.value),
                                                                   p.value_len}));
}

// The run of row `off` of a RunLength chunk (run_length_column.cpp:24-36: the first run whose end position is >= off;
// end positions in column.dictionary, dictionary_size runs).
__device__ inline uint32_t rle_run_of(const hy_column_chunk& col, uint32_t off) {
  const uint32_t* ends = static_cast<const uint32_t*>(col.dictionary);
  uint32_t lo = 0, hi = col.dictionary_size - 1u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ends[mid] < off)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// Run r of a RunLength string chunk: its packed value and NULL flag.
__device__ inline bool rle_run_match(const hy_scan_chunk& ch, uint32_t r, const StrPred& p) {
  const hy_column_chunk& col = ch.column;
  return string_value_match(ch.op, col.nulls != nullptr && col.nulls[r], hyk::packed_string(col.data, col.dictionary_size, r),
                            p);
}

// Row `off` of a scan chunk: the reference's predicate for a dictionary chunk (value id vs search_vid / id set, as
// hy_table_scan), for a string value chunk (compare with the constant, LIKE, IS [NOT] NULL) or for a RunLength chunk
// (the predicate of the row's run).
__device__ inline bool string_row_match(const hy_scan_chunk& ch, uint32_t off, const StrPred& p) {
  const int op = ch.op;
  if (op == HY_OP_NONE) return false;
  const hy_column_chunk& col = ch.column;
  if (col.kind == HY_COL_DICT) {
    const uint32_t vid = col.vid_width == 1   ? static_cast<const uint8_t*>(col.data)[off]
                         : col.vid_width == 2 ? static_cast<const uint16_t*>(col.data)[off]
                                              : static_cast<const uint32_t*>(col.data)[off];
    const bool is_null = vid == col.dictionary_size;
    if (op == HY_OP_IS_NULL) return is_null;
    if (is_null) return false;
    if (op == HY_OP_ALL || op == HY_OP_IS_NOT_NULL) return true;
    if (op == HY_OP_VID_SET) return (ch.vid_set[vid >> 5] >> (vid & 31)) & 1u;
    return hyk::cmp_op<uint32_t>(op, vid, ch.search_vid);
  }
  if (col.kind == HY_COL_RLE) return rle_run_match(ch, rle_run_of(col, off), p);
  return string_value_match(op, col.nulls != nullptr && col.nulls[off], hyk::packed_string(col.data, col.size, off), p);
}

struct TableDesc {
  const hy_scan_chunk* chunks;
  const uint32_t* chunk_ids;
  const uint32_t* tile_chunk;
  const uint64_t* chunk_tile_begin;
  const uint64_t* chunk_row_begin;
  uint64_t n_tiles;
  const uint64_t* run_base;  // RunLength chunks: index of the chunk's first run in run_flags
  const uint8_t* run_flags;  // the predicate per run (string_rle_runs)
};

// RunLength chunks of a table scan: the predicate once per run (the reference's RunLength iterable yields a run's value
// for each of its positions; the value and the predicate are the same for all of them). One thread per run, 256-run
// tiles inside one chunk.
__global__ __launch_bounds__(STR_THREADS) void string_rle_runs(const hy_scan_chunk* __restrict__ chunks,
                                                              const uint32_t* __restrict__ tile_chunk,
                                                              const uint64_t* __restrict__ chunk_tile_begin,
                                                              const uint64_t* __restrict__ run_base, uint64_t n_tiles,
                                                              StrPred p, uint8_t* __restrict__ run_flags) {
  const uint64_t tile = blockIdx.x;
  if (tile >= n_tiles) return;
  const uint32_t c = tile_chunk[tile];
  const hy_scan_chunk& ch = chunks[c];
  const uint32_t r = static_cast<uint32_t>(tile - chunk_tile_begin[c]) * STR_THREADS + threadIdx.x;
  if (r < ch.column.dictionary_size) run_flags[run_base[c] + r] = ch.op != HY_OP_NONE && rle_run_match(ch, r, p);
}

__global__ __launch_bounds__(STR_THREADS) void string_table_flags(TableDesc d, StrPred p, hy_row_id* __restrict__ items,
                                                                 uint8_t* __restrict__ flags,
                                                                 uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_count;
  const uint64_t tile = blockIdx.x;
  if (tile >= d.n_tiles) return;
  const uint32_t c = d.tile_chunk[tile];
  const hy_scan_chunk& ch = d.chunks[c];
  const uint32_t off = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * STR_THREADS + threadIdx.x;
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  if (off < ch.column.size) {
    const bool m = ch.column.kind == HY_COL_RLE
                       ? ch.op != HY_OP_NONE && d.run_flags[d.run_base[c] + rle_run_of(ch.column, off)] != 0
                       : string_row_match(ch, off, p);
    const uint64_t g = d.chunk_row_begin[c] + off;
    flags[g] = m;
    items[g] = hy_row_id{d.chunk_ids[c], off};
    if (m) atomicAdd(&s_count, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_count) atomicAdd(&counts[c], s_count);
}

__global__ __launch_bounds__(STR_THREADS) void string_reference_flags(const hy_row_id* __restrict__ pos_list, uint64_t n,
                                                                     const hy_scan_chunk* __restrict__ referenced,
                                                                     uint32_t n_referenced, StrPred p,
                                                                     uint32_t* __restrict__ items,
                                                                     uint8_t* __restrict__ flags) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const hy_row_id rid = pos_list[i];
    bool m = false;
    if (rid.chunk_offset != 0xFFFFFFFFu && rid.chunk_id < n_referenced)
      m = string_row_match(referenced[rid.chunk_id], rid.chunk_offset, p);
    flags[i] = m;
    items[i] = static_cast<uint32_t>(i);
  }
}

// ---- host: the LIKE pattern's NFA ----
// The reference's regex text of a LIKE pattern (like_matcher.cpp:104-125, sql_like_to_regex without the anchors):
// backslash doubled first, then the regex specials escaped, '%' -> ".*", '_' -> "." - inside [...] too.
std::string like_to_regex(const char* pattern, uint32_t len) {
  std::string r;
  for (uint32_t i = 0; i < len; ++i) {
    const char ch = pattern[i];
    switch (ch) {
      case '\\':
        r += "\\\\";
        break;
      case '.': case '^': case '$': case '+': case '?': case '(': case ')': case '{': case '}': case '|': case '*':
        r += '\\';
        r += ch;
        break;
      case '%':
        r += ".*";
        break;
      case '_':
        r += '.';
        break;
      default:
        r += ch;
    }
  }
  return r;
}

hy_status compile_like(const char* pattern, uint32_t len, int32_t regex, LikeNfa* a) {
  std::memset(a, 0, sizeof(*a));
  int m = 0;
  auto bit = [](uint64_t* words, int j) { words[j >> 6] |= 1ull << (j & 63); };
  auto position = [&](bool star) -> int {
    if (m >= LIKE_MAX_POSITIONS) return -1;
    if (star) bit(a->star, m);
    return m++;
  };
  const char* too_long = "LIKE pattern longer than 1023 positions";
  const auto newline = [](unsigned c) { return c == '\n' || c == '\r'; };
  if (!regex) {  // the reference's string-search patterns: '%' any bytes, '_' any byte, everything else literal
    for (uint32_t i = 0; i < len; ++i) {
      const unsigned char ch = static_cast<unsigned char>(pattern[i]);
      const int j = position(ch == '%');
      if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
      for (unsigned c = 0; c < 256; ++c) {
        if (ch == '%') bit(a->star_ok[c], j);
        else if (ch == '_' || c == ch) bit(a->lit[c], j);
      }
    }
  } else {
    // the reference's std::regex (ECMAScript) over the regex text: '.' any byte but '\n' / '\r', ".*" a star of it,
    // "\x" the literal x, [...] a class (members: "\x" escapes and plain bytes, "x-y" ranges; "[]" matches nothing),
    // every other byte literal (a ']' outside a class too, as libstdc++ reads it)
    const std::string re = like_to_regex(pattern, len);
    const uint32_t n = static_cast<uint32_t>(re.size());
    for (uint32_t i = 0; i < n; ++i) {
      const unsigned char ch = static_cast<unsigned char>(re[i]);
      if (ch == '.' && i + 1 < n && re[i + 1] == '*') {
        const int j = position(true);
        if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
        for (unsigned c = 0; c < 256; ++c)
          if (!newline(c)) bit(a->star_ok[c], j);
        ++i;
      } else if (ch == '.') {
        const int j = position(false);
        if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
        for (unsigned c = 0; c < 256; ++c)
          if (!newline(c)) bit(a->lit[c], j);
      } else if (ch == '\\' && i + 1 < n) {
        const int j = position(false);
        if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
        bit(a->lit[static_cast<unsigned char>(re[++i])], j);
      } else if (ch == '[') {
        const int j = position(false);
        if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
        uint32_t k = i + 1;
        // one class atom at k: an escaped or plain byte; returns the byte and advances k
        auto atom = [&](uint32_t& at) -> unsigned char {
          if (re[at] == '\\' && at + 1 < n) {
            at += 2;
            return static_cast<unsigned char>(re[at - 1]);
          }
          return static_cast<unsigned char>(re[at++]);
        };
        bool closed = false;
        while (k < n) {
          if (re[k] == ']') {  // (the first ']' closes: "[]" is the empty class)
            closed = true;
            break;
          }
          const unsigned char x = atom(k);
          if (k + 1 < n && re[k] == '-' && re[k + 1] != ']') {
            uint32_t k2 = k + 1;
            const unsigned char y = atom(k2);
            if (y < x) return fail(HY_ERR_INVALID_ARGUMENT, "LIKE character class range out of order (the reference's regex fails)");
            for (unsigned c = x; c <= y; ++c) bit(a->lit[c], j);
            k = k2;
          } else {
            bit(a->lit[x], j);
          }
        }
        if (!closed) return fail(HY_ERR_INVALID_ARGUMENT, "unterminated [ in a LIKE pattern (the reference's regex fails)");
        i = k;
      } else {
        const int j = position(false);
        if (j < 0) return fail(HY_ERR_UNSUPPORTED, too_long);
        bit(a->lit[ch], j);
      }
    }
  }
  bit(a->accept, m);
  a->words = static_cast<uint32_t>(m / 64 + 1);
  a->start[0] = 1;
  star_closure_words(a->start, a->star, a->words);
  return HY_OK;
}

struct Staged {
  char* value;
  LikeNfa* nfa;
};

void carve_pred(Carver& cv, const hy_string_predicate* pred, Staged* st) {
  st->value = cv.take<char>(pred && pred->value_len ? pred->value_len + 16 : 16);
  st->nfa = cv.take<LikeNfa>(1);
}

hy_status stage_pred(const hy_string_predicate* pred, const Staged& st, hipStream_t s, StrPred* p, bool need_like) {
  p->value = st.value;
  p->value_len = 0;
  p->nfa = nullptr;
  if (pred && pred->value_len) {
    if (!pred->value) return fail(HY_ERR_INVALID_ARGUMENT, "string constant");
    HY_STAGE(st.value, pred->value, pred->value_len, s);
    p->value_len = pred->value_len;
  }
  if (need_like) {
    if (!pred || (pred->pattern_len && !pred->pattern)) return fail(HY_ERR_INVALID_ARGUMENT, "LIKE pattern");
    LikeNfa a;
    const hy_status r = compile_like(pred->pattern, pred->pattern_len, pred->pattern_regex, &a);
    if (r != HY_OK) return r;
    HY_STAGE(st.nfa, &a, sizeof(a), s);
    p->nfa = st.nfa;
  }
  return HY_OK;
}

hy_status check_ops(const hy_scan_chunk* chunks, uint32_t n, bool* need_like) {
  *need_like = false;
  for (uint32_t c = 0; c < n; ++c) {
    const auto& ch = chunks[c];
    if (ch.column.kind == HY_COL_DICT) {
      if (ch.op < HY_OP_EQ || ch.op > HY_OP_VID_SET || (ch.op == HY_OP_VID_SET && !ch.vid_set))
        return fail(HY_ERR_INVALID_ARGUMENT, "dictionary chunk op");
    } else if (ch.column.kind == HY_COL_STRING || ch.column.kind == HY_COL_RLE) {
      if (ch.op == HY_OP_VID_SET || ch.op < HY_OP_EQ || ch.op > HY_OP_NOT_LIKE)
        return fail(HY_ERR_INVALID_ARGUMENT, "string chunk op");
      if (ch.column.kind == HY_COL_RLE && ch.column.size && (ch.column.dictionary_size == 0 || !ch.column.dictionary))
        return fail(HY_ERR_INVALID_ARGUMENT, "RunLength chunk without runs");
      if (ch.op == HY_OP_LIKE || ch.op == HY_OP_NOT_LIKE) *need_like = true;
    } else if (ch.column.size) {
      return fail(HY_ERR_INVALID_ARGUMENT, "string scans take STRING, RLE or DICT chunks");
    }
  }
  return HY_OK;
}

template <typename Item>
size_t select_temp(uint64_t rows) {
  size_t t = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, t, static_cast<const Item*>(nullptr), static_cast<const uint8_t*>(nullptr),
                                      static_cast<Item*>(nullptr), static_cast<uint64_t*>(nullptr),
                                      static_cast<int>(rows));
  return t + 16;
}

struct TableWs {
  hy_scan_chunk* chunks;
  uint32_t* ids;
  uint32_t* tile_chunk;
  uint64_t *tile_begin, *row_begin;
  uint32_t* run_tile_chunk;
  uint64_t *run_tile_begin, *run_base;
  uint8_t* run_flags;
  hy_row_id* items;
  uint8_t* flags;
  char* temp;
  size_t temp_bytes;
  Staged st;
};

void carve_table(Carver& cv, uint64_t rows, uint64_t tiles, uint64_t runs, uint64_t run_tiles, uint32_t n,
                 const hy_string_predicate* pred, TableWs* w) {
  w->chunks = cv.take<hy_scan_chunk>(std::max<uint32_t>(1, n));
  w->ids = cv.take<uint32_t>(std::max<uint32_t>(1, n));
  w->tile_chunk = cv.take<uint32_t>(tiles + 1);
  w->tile_begin = cv.take<uint64_t>(n + 1);
  w->row_begin = cv.take<uint64_t>(n + 1);
  w->run_tile_chunk = cv.take<uint32_t>(run_tiles + 1);
  w->run_tile_begin = cv.take<uint64_t>(n + 1);
  w->run_base = cv.take<uint64_t>(n + 1);
  w->run_flags = cv.take<uint8_t>(runs + 16);
  w->items = cv.take<hy_row_id>(rows + 1);
  w->flags = cv.take<uint8_t>(rows + 16);
  w->temp_bytes = select_temp<hy_row_id>(rows);
  w->temp = cv.take<char>(w->temp_bytes);
  carve_pred(cv, pred, &w->st);
}

void table_geometry(const hy_scan_chunk* chunks, uint32_t n, uint64_t* rows, uint64_t* tiles, uint64_t* runs,
                    uint64_t* run_tiles) {
  *rows = *tiles = *runs = *run_tiles = 0;
  for (uint32_t c = 0; c < n; ++c) {
    *rows += chunks[c].column.size;
    *tiles += (chunks[c].column.size + STR_THREADS - 1) / STR_THREADS;
    if (chunks[c].column.kind == HY_COL_RLE && chunks[c].column.size) {
      *runs += chunks[c].column.dictionary_size;
      *run_tiles += (chunks[c].column.dictionary_size + STR_THREADS - 1) / STR_THREADS;
    }
  }
}

}  // namespace

extern "C" {

hy_status hy_string_table_scan_workspace_size(const hy_scan_chunk* chunks, uint32_t n_chunks,
                                              const hy_string_predicate* pred, size_t* bytes) {
  if (!bytes || (n_chunks && !chunks)) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  uint64_t rows, tiles, runs, run_tiles;
  table_geometry(chunks, n_chunks, &rows, &tiles, &runs, &run_tiles);
  Carver cv{nullptr, 0};
  TableWs w;
  carve_table(cv, rows, tiles, runs, run_tiles, n_chunks, pred, &w);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_string_table_scan(const hy_scan_chunk* chunks, uint32_t n_chunks, const hy_string_predicate* pred,
                               const uint32_t* chunk_ids, hy_row_id* out_rows, uint32_t* counts, uint64_t* n_out,
                               void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  if ((n_chunks && (!chunks || !chunk_ids || !counts)) || !n_out) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  bool need_like = false;
  hy_status st = check_ops(chunks, n_chunks, &need_like);
  if (st != HY_OK) return st;
  uint64_t rows, tiles, runs, run_tiles;
  table_geometry(chunks, n_chunks, &rows, &tiles, &runs, &run_tiles);
  if (rows >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 rows");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(n_out, 0, 8, s));
  if (n_chunks) HY_HIP(hipMemsetAsync(counts, 0, 4ull * n_chunks, s));
  if (rows == 0) return HY_OK;
  if (!out_rows) return fail(HY_ERR_INVALID_ARGUMENT, "out_rows");
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  TableWs w;
  carve_table(cv, rows, tiles, runs, run_tiles, n_chunks, pred, &w);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "string scan workspace too small");
  StrPred p{};
  st = stage_pred(pred, w.st, s, &p, need_like);
  if (st != HY_OK) return st;
  std::vector<uint32_t> tc(tiles);
  std::vector<uint64_t> tb(n_chunks + 1), rb(n_chunks + 1);
  uint64_t t = 0, r = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    tb[c] = t;
    rb[c] = r;
    const uint64_t k = (chunks[c].column.size + STR_THREADS - 1) / STR_THREADS;
    for (uint64_t i = 0; i < k; ++i) tc[t + i] = c;
    t += k;
    r += chunks[c].column.size;
  }
  tb[n_chunks] = t;
  rb[n_chunks] = r;
  // RunLength chunks: their runs' tiles and each chunk's first run in run_flags
  std::vector<uint32_t> rtc(run_tiles);
  std::vector<uint64_t> rtb(n_chunks + 1), rbase(n_chunks + 1);
  uint64_t rt = 0, rr = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    rtb[c] = rt;
    rbase[c] = rr;
    if (chunks[c].column.kind != HY_COL_RLE || chunks[c].column.size == 0) continue;
    const uint64_t k = (chunks[c].column.dictionary_size + STR_THREADS - 1) / STR_THREADS;
    for (uint64_t i = 0; i < k; ++i) rtc[rt + i] = c;
    rt += k;
    rr += chunks[c].column.dictionary_size;
  }
  rtb[n_chunks] = rt;
  rbase[n_chunks] = rr;
  HY_STAGE(w.chunks, chunks, sizeof(hy_scan_chunk) * n_chunks, s);
  HY_STAGE(w.ids, chunk_ids, 4ull * n_chunks, s);
  HY_STAGE(w.tile_chunk, tc.data(), 4 * tiles, s);
  HY_STAGE(w.tile_begin, tb.data(), 8ull * (n_chunks + 1), s);
  HY_STAGE(w.row_begin, rb.data(), 8ull * (n_chunks + 1), s);
  if (run_tiles) {
    HY_STAGE(w.run_tile_chunk, rtc.data(), 4 * run_tiles, s);
    HY_STAGE(w.run_tile_begin, rtb.data(), 8ull * (n_chunks + 1), s);
    HY_STAGE(w.run_base, rbase.data(), 8ull * (n_chunks + 1), s);
    KTimer kt_("string_rle_runs", s, runs);
    hipLaunchKernelGGL(string_rle_runs, dim3(static_cast<uint32_t>(run_tiles)), dim3(STR_THREADS), 0, s, w.chunks,
                       w.run_tile_chunk, w.run_tile_begin, w.run_base, run_tiles, p, w.run_flags);
    kt_.done();
    HY_HIP(hipGetLastError());
  }
  const TableDesc d{w.chunks, w.ids, w.tile_chunk, w.tile_begin, w.row_begin, tiles, w.run_base, w.run_flags};
  {
    KTimer kt_("string_table_flags", s, rows);
    hipLaunchKernelGGL(string_table_flags, dim3(static_cast<uint32_t>(tiles)), dim3(STR_THREADS), 0, s, d, p, w.items,
                       w.flags, counts);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  HY_HIP(hipcub::DeviceSelect::Flagged(w.temp, w.temp_bytes, static_cast<const hy_row_id*>(w.items), w.flags, out_rows,
                                       n_out, static_cast<int>(rows), s));
  return HY_OK;
}

hy_status hy_string_reference_scan_workspace_size(uint64_t pos_list_size, uint32_t n_referenced,
                                                  const hy_string_predicate* pred, size_t* bytes) {
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "null bytes");
  Carver cv{nullptr, 0};
  cv.take<hy_scan_chunk>(std::max<uint32_t>(1, n_referenced));
  cv.take<uint32_t>(pos_list_size + 1);
  cv.take<uint8_t>(pos_list_size + 16);
  cv.take<char>(select_temp<uint32_t>(pos_list_size));
  Staged stg;
  carve_pred(cv, pred, &stg);
  *bytes = cv.used + 256;
  return HY_OK;
}

hy_status hy_string_reference_scan(const hy_row_id* pos_list, uint64_t pos_list_size,
                                   const hy_scan_chunk* referenced_chunks, uint32_t n_referenced_chunks,
                                   const hy_string_predicate* pred, uint32_t* out_positions, uint64_t* count,
                                   void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  if (!count || (n_referenced_chunks && !referenced_chunks)) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  bool need_like = false;
  hy_status st = check_ops(referenced_chunks, n_referenced_chunks, &need_like);
  if (st != HY_OK) return st;
  if (pos_list_size >= 0x7FFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^31-1 positions");
  hipStream_t s = S(stream);
  HY_HIP(hipMemsetAsync(count, 0, 8, s));
  if (pos_list_size == 0) return HY_OK;
  if (!pos_list || !out_positions) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  Carver cv{static_cast<char*>(workspace), workspace_bytes};
  auto* dch = cv.take<hy_scan_chunk>(std::max<uint32_t>(1, n_referenced_chunks));
  auto* items = cv.take<uint32_t>(pos_list_size + 1);
  auto* flags = cv.take<uint8_t>(pos_list_size + 16);
  size_t tb = select_temp<uint32_t>(pos_list_size);
  char* temp = cv.take<char>(tb);
  Staged stg;
  carve_pred(cv, pred, &stg);
  if (!cv.ok) return fail(HY_ERR_WORKSPACE, "string reference scan workspace too small");
  StrPred p{};
  st = stage_pred(pred, stg, s, &p, need_like);
  if (st != HY_OK) return st;
  HY_STAGE(dch, referenced_chunks, sizeof(hy_scan_chunk) * n_referenced_chunks, s);
  {
    KTimer kt_("string_reference_flags", s, pos_list_size);
    hipLaunchKernelGGL(string_reference_flags, dim3(grid_for(pos_list_size, STR_THREADS)), dim3(STR_THREADS), 0, s,
                       pos_list, pos_list_size, dch, n_referenced_chunks, p, items, flags);
    kt_.done();
  }
  HY_HIP(hipGetLastError());
  HY_HIP(hipcub::DeviceSelect::Flagged(temp, tb, static_cast<const uint32_t*>(items), flags, out_positions, count,
                                       static_cast<int>(pos_list_size), s));
  return HY_OK;
}

}  // extern "C"
