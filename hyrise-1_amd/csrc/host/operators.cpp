#include "operators.hpp"
#include "scheduler.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

#include "hyrise_amd_trace.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <exception>
#include <map>
#include <mutex>
#include <numeric>
#include <regex>
#include <thread>
#include <unordered_map>

#include <unistd.h>  // environ

namespace hyrise {

namespace {
// Host wall time of operator phases (where an operator step's time goes): HY_OP_TRACE=1 prints them on stderr;
// op_trace_enable(true) records them for op_trace_take() (bench_ops.py keeps every step's split).
std::atomic<bool> g_trace_record{false};
std::mutex g_trace_m;
std::vector<OpTraceRecord> g_trace;

struct PhaseTrace {
  const char* op;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  bool print = std::getenv("HY_OP_TRACE") != nullptr;
  bool record = g_trace_record.load(std::memory_order_relaxed);
  bool on = print || record;
  void mark(const char* phase) { note(phase, since()); }
  double since() {
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
    return ms;
  }
  void note(const std::string& phase, double ms) const {
    if (print) std::fprintf(stderr, "[op] %s %s %.3f ms\n", op, phase.c_str(), ms);
    if (record) {
      std::lock_guard<std::mutex> lock(g_trace_m);
      g_trace.push_back({op, phase, ms});
    }
  }
};
}  // namespace

void op_trace_enable(bool on) { g_trace_record.store(on); }

std::vector<OpTraceRecord> op_trace_take() {
  std::lock_guard<std::mutex> lock(g_trace_m);
  std::vector<OpTraceRecord> out;
  out.swap(g_trace);
  return out;
}

namespace {
// A roctx range per operator execution (rocprofv3 --marker-trace shows each operator around its kernels).
struct OperatorRange {
  explicit OperatorRange(const std::string& name) { roctxRangePushA(name.c_str()); }
  ~OperatorRange() { roctxRangePop(); }
};

// The device time of the operator's stream work: an event on this thread's operator stream before _on_execute and
// one after it. finish() (after the stream's synchronisation) returns the nanoseconds between them, 0 when the
// operator issued nothing on the stream (the events then complete back to back).
struct DeviceSpan {
  struct Events {
    hy_event_t start = nullptr, stop = nullptr;
    ~Events() {
      hy_event_destroy(start);
      hy_event_destroy(stop);
    }
  };
  Events* ev = nullptr;
  DeviceSpan() {
    int n = 0;
    if (hy_get_device_count(&n) != HY_OK || n <= 0) return;  // (no device: the operator fails on its own)
    // the thread's operator stream first: thread-local objects are destroyed in the reverse order of their first use,
    // so the events go before the stream they are recorded on (hy_stream_destroy)
    hy_stream_t s = operator_stream();
    thread_local Events events;
    if (!events.start && (hy_event_create(&events.start) != HY_OK || hy_event_create(&events.stop) != HY_OK)) return;
    if (hy_event_record(events.start, s) == HY_OK) ev = &events;
  }
  uint64_t finish() {
    uint64_t ns = 0;
    if (ev && hy_event_record(ev->stop, operator_stream()) == HY_OK &&
        hy_event_elapsed_ns(ev->start, ev->stop, &ns) == HY_OK)
      return ns;
    return 0;
  }
};
}  // namespace

// reference abstract_operator.cpp:25-54
void AbstractOperator::execute() {
  Assert(!_input_left || _input_left->get_output(), "Left input has not been executed");
  Assert(!_input_right || _input_right->get_output(), "Right input has not been executed");
  Assert(!_output, "Operator has already been executed");
  const auto t0 = std::chrono::steady_clock::now();
  // abstract_operator.cpp:32-41: an aborted transaction skips the operator; its output stays unset
  const auto context = transaction_context();
  if (context && context->aborted()) return;
  OperatorRange range(name());
  DeviceSpan span;
  _output = _on_execute(context);
  // The output is complete when execute() returns (the reference's contract): consumers may run on other threads,
  // whose non-blocking operator streams are not ordered after this thread's kernels.
  operator_stream_synchronize_if_used();
  _performance_data.device_ns = span.finish();
  _on_cleanup();
  _performance_data.walltime_ns = static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
}

// abstract_operator.cpp:100-106
void AbstractOperator::set_transaction_context_recursively(const std::weak_ptr<TransactionContext>& context) {
  set_transaction_context(context);
  if (_input_left) mutable_input_left()->set_transaction_context_recursively(context);
  if (_input_right) mutable_input_right()->set_transaction_context_recursively(context);
}

// abstract_operator.cpp:77-81
std::shared_ptr<AbstractOperator> AbstractOperator::deep_copy() const {
  std::unordered_map<const AbstractOperator*, std::shared_ptr<AbstractOperator>> copied_ops;
  return _deep_copy_impl(copied_ops);
}

// abstract_operator.cpp:157-173
std::shared_ptr<AbstractOperator> AbstractOperator::_deep_copy_impl(
    std::unordered_map<const AbstractOperator*, std::shared_ptr<AbstractOperator>>& copied_ops) const {
  const auto it = copied_ops.find(this);
  if (it != copied_ops.end()) return it->second;
  const auto left = _input_left ? _input_left->_deep_copy_impl(copied_ops) : std::shared_ptr<AbstractOperator>{};
  const auto right = _input_right ? _input_right->_deep_copy_impl(copied_ops) : std::shared_ptr<AbstractOperator>{};
  auto copy = _on_deep_copy(left, right);
  if (_transaction_context) copy->set_transaction_context(*_transaction_context);
  copied_ops.emplace(this, copy);
  return copy;
}

// abstract_operator.cpp:147-151
void AbstractOperator::set_parameters(const ParameterMap& parameters) {
  _on_set_parameters(parameters);
  if (_input_left) mutable_input_left()->set_parameters(parameters);
  if (_input_right) mutable_input_right()->set_parameters(parameters);
}

// ================================================================================================================
// TableScan
// ================================================================================================================
namespace {

int32_t value_op(PredicateCondition c) {
  switch (c) {
    case PredicateCondition::Equals:
      return HY_OP_EQ;
    case PredicateCondition::NotEquals:
      return HY_OP_NE;
    case PredicateCondition::LessThan:
      return HY_OP_LT;
    case PredicateCondition::LessThanEquals:
      return HY_OP_LE;
    case PredicateCondition::GreaterThan:
      return HY_OP_GT;
    case PredicateCondition::GreaterThanEquals:
      return HY_OP_GE;
    default:
      Fail("Unsupported operator.");  // reference with_comparator, type_comparison.hpp:100-123
  }
}

// Dictionary rewrite: reference single_column_table_scan_impl.cpp:87-205 and .hpp:52-76.
void dictionary_predicate(const BaseDictionaryColumn& col, PredicateCondition cond, const AllTypeVariant& value,
                          int32_t* op, uint32_t* search_vid) {
  ValueID svid;
  switch (cond) {
    case PredicateCondition::Equals:
    case PredicateCondition::NotEquals:
    case PredicateCondition::LessThan:
    case PredicateCondition::GreaterThanEquals:
      svid = col.lower_bound(value);
      break;
    case PredicateCondition::LessThanEquals:
    case PredicateCondition::GreaterThan:
      svid = col.upper_bound(value);
      break;
    default:
      Fail("Unsupported comparison type encountered");
  }
  // _right_value_matches_all
  bool all = false, none = false;
  switch (cond) {
    case PredicateCondition::Equals:
      all = svid != col.upper_bound(value) && col.unique_values_count() == 1u;
      none = svid == col.upper_bound(value);
      break;
    case PredicateCondition::NotEquals:
      all = svid == col.upper_bound(value);
      none = svid == col.upper_bound(value) && col.unique_values_count() == 1u;
      break;
    case PredicateCondition::LessThan:
    case PredicateCondition::LessThanEquals:
      all = svid == INVALID_VALUE_ID;
      none = svid == 0u;
      break;
    case PredicateCondition::GreaterThanEquals:
    case PredicateCondition::GreaterThan:
      all = svid == 0u;
      none = svid == INVALID_VALUE_ID;
      break;
    default:
      break;
  }
  *search_vid = svid;
  if (all) {
    *op = HY_OP_ALL;
    return;
  }
  if (none) {
    *op = HY_OP_NONE;
    return;
  }
  switch (cond) {  // _with_operator_for_dict_column_scan
    case PredicateCondition::Equals:
      *op = HY_OP_EQ;
      break;
    case PredicateCondition::NotEquals:
      *op = HY_OP_NE;
      break;
    case PredicateCondition::LessThan:
    case PredicateCondition::LessThanEquals:
      *op = HY_OP_LT;
      break;
    default:
      *op = HY_OP_GE;
      break;
  }
}

// SQL LIKE semantics of the reference's LikeMatcher (src/lib/expression/evaluation/like_matcher.cpp:9-118): the
// pattern is split into literal runs and the wildcards '%' / '_'; 'abc%', '%abc', '%abc%' and '%a%b%...%' are matched
// with plain string searches, anything else through the ECMAScript regex '^...$' the reference builds (its escaping
// leaves '[' and ']' as regex syntax, so those patterns behave as the reference's do).
class LikePattern {
 public:
  explicit LikePattern(const std::string& pattern) : _source(pattern) {
    std::vector<std::string> tokens;  // "%" / "_" wildcards, other tokens are literal runs
    std::vector<bool> is_wild;
    for (size_t i = 0; i < pattern.size();) {
      if (pattern[i] == '%' || pattern[i] == '_') {
        tokens.emplace_back(1, pattern[i]);
        is_wild.push_back(true);
        ++i;
        continue;
      }
      const size_t next = pattern.find_first_of("_%", i);
      tokens.push_back(pattern.substr(i, next == std::string::npos ? std::string::npos : next - i));
      is_wild.push_back(false);
      i = next == std::string::npos ? pattern.size() : next;
    }
    auto any = [&](size_t k) { return is_wild[k] && tokens[k] == "%"; };
    auto lit = [&](size_t k) { return !is_wild[k]; };
    const size_t n = tokens.size();
    if (n == 2 && lit(0) && any(1)) {
      _kind = Kind::StartsWith;
      _parts = {tokens[0]};
    } else if (n == 2 && any(0) && lit(1)) {
      _kind = Kind::EndsWith;
      _parts = {tokens[1]};
    } else if (n == 3 && any(0) && lit(1) && any(2)) {
      _kind = Kind::Contains;
      _parts = {tokens[1]};
    } else {
      bool multi = true, expect_any = true;
      for (size_t k = 0; k < n && multi; ++k) {
        if (expect_any ? !any(k) : !lit(k)) multi = false;
        if (multi && !expect_any) _parts.push_back(tokens[k]);
        expect_any = !expect_any;
      }
      if (multi) {
        _kind = Kind::MultipleContains;
      } else {
        _kind = Kind::Regex;
        _parts.clear();
        std::string re = "^";
        for (const char ch : pattern) {
          if (ch == '%') {
            re += ".*";
          } else if (ch == '_') {
            re += '.';
          } else {
            if (std::strchr("\\.^$+?(){}|*", ch) != nullptr) re += '\\';
            re += ch;
          }
        }
        _regex = std::regex(re + "$");
      }
    }
  }

  // The pattern the device matcher takes (hy_string_predicate): the simple kinds as the '%'-only pattern they match
  // (a MultipleContains pattern matches anywhere, so it becomes '%a%b%'; '' matches every string, like '%'), the regex
  // kind as written.
  std::string device_pattern(int32_t* regex) const {
    *regex = _kind == Kind::Regex ? 1 : 0;
    switch (_kind) {
      case Kind::StartsWith:
        return _parts[0] + "%";
      case Kind::EndsWith:
        return "%" + _parts[0];
      case Kind::Contains:
        return "%" + _parts[0] + "%";
      case Kind::MultipleContains: {
        std::string p = "%";
        for (const auto& x : _parts) p += x + "%";
        return p;
      }
      default:
        return _source;
    }
  }

  bool operator()(const std::string& v) const {
    switch (_kind) {
      case Kind::StartsWith:
        return v.compare(0, _parts[0].size(), _parts[0]) == 0 && v.size() >= _parts[0].size();
      case Kind::EndsWith:
        return v.size() >= _parts[0].size() && v.compare(v.size() - _parts[0].size(), _parts[0].size(), _parts[0]) == 0;
      case Kind::Contains:
        return v.find(_parts[0]) != std::string::npos;
      case Kind::MultipleContains: {
        size_t at = 0;
        for (const auto& p : _parts) {
          const size_t f = v.find(p, at);
          if (f == std::string::npos) return false;
          at = f + p.size();
        }
        return true;
      }
      default:
        return std::regex_match(v, _regex);
    }
  }

 private:
  enum class Kind { StartsWith, EndsWith, Contains, MultipleContains, Regex };
  Kind _kind = Kind::Regex;
  std::vector<std::string> _parts;
  std::regex _regex;
  std::string _source;
};

// The id sets of one scan's LIKE / NOT LIKE dictionary chunks, uploaded together: the pattern is compiled once, every
// chunk's bitmap is appended to one host array, and one copy (one stream sync) moves them all (instead of an
// allocation, a copy and a sync per chunk).
struct LikeBatch {
  std::unique_ptr<LikePattern> matcher;
  std::vector<uint32_t> words;
  std::vector<std::pair<hy_scan_chunk*, size_t>> fix;  // descriptor, word offset of its id set
  // Uploads the id sets and points the descriptors at them (the descriptors must not have moved since).
  void finish(std::vector<std::shared_ptr<DeviceBuffer>>* keep) {
    if (fix.empty()) return;
    auto buf = std::make_shared<DeviceBuffer>(words.size() * 4);
    hy_stream_t s = operator_stream();
    hy_check(hy_memcpy_htod(buf->get(), words.data(), words.size() * 4, s), "htod");
    hy_check(hy_stream_synchronize(s), "sync");  // `words` is pageable host memory
    for (auto& [sc, off] : fix) sc->vid_set = buf->as<uint32_t>() + off;
    keep->push_back(std::move(buf));
    fix.clear();
  }
};

// LIKE / NOT LIKE over a dictionary chunk (like_table_scan_impl.cpp:48-83, 102-120): the pattern is evaluated once per
// dictionary entry on the host; all / none early-outs, otherwise the device scans against the set of matching ids
// (appended to the scan's LikeBatch; the caller registers the descriptor's final address with it).
size_t like_predicate(const BaseDictionaryColumn& column, PredicateCondition cond, const AllTypeVariant& value,
                      hy_scan_chunk* sc, LikeBatch* batch) {
  const auto* dict = dynamic_cast<const DictionaryColumn<std::string>*>(&column);
  Assert(dict != nullptr, "LIKE operator only applicable on string columns.");
  Assert(!variant_is_null(value), "Right value must not be NULL.");
  if (!batch->matcher) batch->matcher = std::make_unique<LikePattern>(type_cast<std::string>(value));
  const LikePattern& matcher = *batch->matcher;
  const bool invert = cond == PredicateCondition::NotLike;
  const auto& d = dict->dictionary();
  const size_t off = (batch->words.size() + 3) & ~size_t(3);  // 16-byte aligned id sets
  batch->words.resize(off + (d.size() + 31) / 32 + 1, 0u);
  uint32_t* bits = batch->words.data() + off;
  size_t count = 0;
  for (size_t v = 0; v < d.size(); ++v) {
    if (matcher(d[v]) != invert) {
      bits[v >> 5] |= 1u << (v & 31);
      ++count;
    }
  }
  if (count == d.size() || count == 0) {
    sc->op = count ? HY_OP_ALL : HY_OP_NONE;
    batch->words.resize(off);
    return SIZE_MAX;
  }
  sc->op = HY_OP_VID_SET;
  return off;
}

// Builds the scan descriptor of one data column chunk. constant_out receives type_cast<T>(value) for value columns.
// LIKE id sets go to `batch` (*like_off: their word offset, SIZE_MAX if none): the caller registers the stored
// descriptor with batch->fix and calls batch->finish (which keeps the device buffer alive in `keep`).
hy_scan_chunk scan_descriptor(const BaseColumn& column, DataType type, PredicateCondition cond,
                              const AllTypeVariant& value, LikeBatch* batch, size_t* like_off) {
  hy_scan_chunk sc{};
  *like_off = SIZE_MAX;
  const auto* dict = dynamic_cast<const BaseDictionaryColumn*>(&column);
  if (cond == PredicateCondition::Like || cond == PredicateCondition::NotLike) {
    Assert(type == DataType::String, "LIKE operator only applicable on string columns.");
    if (dict)
      *like_off = like_predicate(*dict, cond, value, &sc, batch);
    else  // LikeTableScanImpl on a value column (like_table_scan_impl.cpp:86-97): the device matches every row
      sc.op = cond == PredicateCondition::Like ? HY_OP_LIKE : HY_OP_NOT_LIKE;
  } else if (cond == PredicateCondition::IsNull || cond == PredicateCondition::IsNotNull) {
    // IsNullTableScanImpl (is_null_table_scan_impl.cpp:35-117): no dictionary rewrite, the null test is per row
    sc.op = cond == PredicateCondition::IsNull ? HY_OP_IS_NULL : HY_OP_IS_NOT_NULL;
  } else if (dict) {
    dictionary_predicate(*dict, cond, value, &sc.op, &sc.search_vid);
  } else {
    sc.op = value_op(cond);
  }
  sc.column = device_scan_chunk(column);  // RunLength / FrameOfReference: scanned in compressed form
  return sc;
}

// The constant / LIKE pattern of a scan over a string column (hy_string_table_scan / hy_string_reference_scan); the
// strings are owned here and must outlive the call.
struct StringScanPredicate {
  std::string value, pattern;
  hy_string_predicate pred{};
  StringScanPredicate(PredicateCondition cond, const AllTypeVariant& v) {
    if (cond == PredicateCondition::Like || cond == PredicateCondition::NotLike) {
      Assert(!variant_is_null(v), "Right value must not be NULL.");
      pattern = LikePattern(type_cast<std::string>(v)).device_pattern(&pred.pattern_regex);
    } else if (cond != PredicateCondition::IsNull && cond != PredicateCondition::IsNotNull && !variant_is_null(v)) {
      value = type_cast<std::string>(v);  // type_comparison.hpp:100-123 compares with type_cast<std::string>(value)
    }
    pred.value = value.data();
    pred.value_len = static_cast<uint32_t>(value.size());
    pred.pattern = pattern.data();
    pred.pattern_len = static_cast<uint32_t>(pattern.size());
  }
};

struct ScanConstant {
  alignas(8) unsigned char bytes[8] = {0};
};

ScanConstant typed_constant(DataType type, const AllTypeVariant& value) {
  ScanConstant c;
  switch (type) {
    case DataType::Int: {
      const int32_t v = type_cast<int32_t>(value);
      std::memcpy(c.bytes, &v, 4);
      break;
    }
    case DataType::Long: {
      const int64_t v = type_cast<int64_t>(value);
      std::memcpy(c.bytes, &v, 8);
      break;
    }
    case DataType::Float: {
      const float v = type_cast<float>(value);
      std::memcpy(c.bytes, &v, 4);
      break;
    }
    case DataType::Double: {
      const double v = type_cast<double>(value);
      std::memcpy(c.bytes, &v, 8);
      break;
    }
    default:
      break;
  }
  return c;
}

// Iteration order of the reference's std::unordered_map<ChunkID, ChunkOffsetsList> built by
// split_pos_list_by_chunk_id (chunk_offset_mapping.cpp:5-21): replay the insertion of the distinct chunk ids in
// order of first appearance into the same libstdc++ container type.
std::vector<ChunkID> unordered_map_order(const std::vector<ChunkID>& first_appearance_order) {
  std::unordered_map<ChunkID, int> m;
  for (const auto c : first_appearance_order) m[c];
  std::vector<ChunkID> out;
  for (const auto& kv : m) out.push_back(kv.first);
  return out;
}

std::shared_ptr<Table> column_comparison_scan(const std::shared_ptr<const Table>& in_table, ColumnID left_column_id,
                                              PredicateCondition cond, ColumnID right_column_id,
                                              const std::vector<bool>& excluded);

}  // namespace

namespace {

// all_parameter_variant.cpp:11-23 (to_string): placeholder, column, or the value as boost::lexical_cast prints it
std::string parameter_to_string(const AllParameterVariant& x) {
  if (is_parameter_id(x)) return "Placeholder #" + std::to_string(std::get<ParameterID>(x).t);
  if (is_column_id(x)) return "Col #" + std::to_string(std::get<ColumnParameter>(x).column_id);
  const AllTypeVariant& v = std::get<AllTypeVariant>(x);
  return variant_is_null(v) ? std::string("NULL") : detail::to_lexical_string(v, 6);
}

std::string join_mode_to_string(JoinMode m) {  // constant_mappings.cpp:54-57
  switch (m) {
    case JoinMode::Cross:
      return "Cross";
    case JoinMode::Inner:
      return "Inner";
    case JoinMode::Left:
      return "Left";
    case JoinMode::Outer:
      return "Outer";
    case JoinMode::Right:
      return "Right";
    case JoinMode::Semi:
      return "Semi";
    default:
      return "Anti";
  }
}

}  // namespace

// table_scan.cpp:51-61
const std::string TableScan::description(DescriptionMode description_mode) const {
  std::string column_name = "Col #" + std::to_string(_left_column_id);
  if (_input_left && input_table_left()) column_name = input_table_left()->column_name(_left_column_id);
  const char* separator = description_mode == DescriptionMode::MultiLine ? "\n" : " ";
  return name() + separator + "(" + column_name + " " + predicate_condition_to_string(_predicate_condition) + " " +
         parameter_to_string(_right_parameter) + ")";
}

// abstract_join_operator.cpp:30-43
const std::string AbstractJoinOperator::description(DescriptionMode description_mode) const {
  std::string left = "Col #" + std::to_string(_column_ids.first);
  std::string right = "Col #" + std::to_string(_column_ids.second);
  if (_input_left && input_table_left()) left = input_table_left()->column_name(_column_ids.first);
  if (_input_right && input_table_right()) right = input_table_right()->column_name(_column_ids.second);
  const char* separator = description_mode == DescriptionMode::MultiLine ? "\n" : " ";
  return name() + separator + "(" + join_mode_to_string(_mode) + " Join where " + left + " " +
         predicate_condition_to_string(_predicate_condition) + " " + right + ")";
}

// table_scan.cpp:63-70: a ParameterID placeholder is replaced by its value when the map holds one
void TableScan::_on_set_parameters(const ParameterMap& parameters) {
  if (!is_parameter_id(_right_parameter)) return;
  const auto it = parameters.find(std::get<ParameterID>(_right_parameter));
  if (it == parameters.end()) return;
  _right_parameter = it->second;
}

// table_scan.cpp:72-76 (excluded chunk ids are not part of the configuration, as in the reference)
std::shared_ptr<AbstractOperator> TableScan::_on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                           const std::shared_ptr<AbstractOperator>&) const {
  return std::make_shared<TableScan>(copied_input_left, _left_column_id, _predicate_condition, _right_parameter);
}

namespace {

// A TableScan over a data table (not strings), as a deferred producer of its output (Table::Producer): it runs on the
// first access of the output - or inside the JoinHash that consumes the output, which evaluates the predicate in its
// first radix pass and hands the matches back (fulfil_from_offsets; JoinHash::_on_execute, "fused TableScan").
struct DataScan final : Table::Producer {
  std::shared_ptr<const Table> in_table;
  ColumnID column_id = 0;
  DataType col_type = DataType::Int;
  std::vector<hy_scan_chunk> descs;  // one per scanned chunk, out_begin = its first row in `rows`
  std::vector<ChunkID> chunk_ids;
  std::vector<uint32_t> sizes;
  ScanConstant constant;
  uint64_t total = 0;
  bool all_chunks = false;  // the scanned chunks are every chunk of in_table, in order

  // the output chunks: one per scanned chunk with a match (table_scan.cpp:99), its PosList a view of `rows`
  std::vector<std::shared_ptr<Chunk>> chunks_from(const std::shared_ptr<DeviceBuffer>& rows,
                                                  const std::vector<std::pair<uint64_t, uint32_t>>& views) const {
    OutputArena arena;
    std::vector<std::shared_ptr<Chunk>> out;
    for (size_t k = 0; k < descs.size(); ++k) {
      if (views[k].second == 0) continue;
      auto pl = pos_list_from_device(arena, rows, views[k].first, views[k].second);
      pl->set_single_chunk_id(chunk_ids[k]);
      ChunkColumns cols;
      cols.reserve(in_table->column_count());
      for (ColumnID col = 0; col < in_table->column_count(); ++col)
        cols.push_back(arena_reference_column(arena, in_table, col, pl));
      out.push_back(arena_chunk(arena, std::move(cols)));
    }
    return out;
  }

  // the scan on its own: one launch writes every chunk's RowIDs at its row range of `rows`
  std::vector<std::shared_ptr<Chunk>> produce() override {
    hy_stream_t s = operator_stream();
    PhaseTrace tr{"TableScan (deferred)"};
    size_t ws_bytes = 0;
    hy_check(hy_table_scan_workspace_size(sizes.data(), static_cast<uint32_t>(sizes.size()), &ws_bytes),
             "hy_table_scan_workspace_size");
    DeviceBuffer ws(ws_bytes, s);
    auto rows = std::make_shared<DeviceBuffer>(std::max<uint64_t>(total, 1) * sizeof(RowID));
    DeviceBuffer counts(descs.size() * 4, s);
    std::vector<uint32_t> h_counts(descs.size());
    hy_check(hy_table_scan_row_ids(descs.data(), static_cast<uint32_t>(descs.size()), hy_type_of(col_type),
                                   constant.bytes, chunk_ids.data(), rows->as<hy_row_id>(), counts.as<uint32_t>(),
                                   ws.get(), ws_bytes, s),
             "hy_table_scan_row_ids");
    hy_check(hy_memcpy_dtoh(h_counts.data(), counts.get(), 4 * descs.size(), s), "hy_memcpy_dtoh");
    hy_check(hy_stream_synchronize(s), "sync");
    tr.mark("scan + counts");
    std::vector<std::pair<uint64_t, uint32_t>> views;
    for (size_t k = 0; k < descs.size(); ++k) views.emplace_back(descs[k].out_begin, h_counts[k]);
    auto out = chunks_from(rows, views);
    tr.mark("output chunks");
    return out;
  }

  // matches of the scan per chunk, counted without output (the fused consumer's swap rule needs the output's row
  // count; with the counts the output chunks are built while the consumer's join runs): kept in `counts`
  std::vector<uint32_t> counts;
  uint64_t count_matches() {
    hy_stream_t s = operator_stream();
    DeviceBuffer ws(std::max<size_t>(sizeof(hy_scan_chunk) * descs.size(), 16), s), d_counts(descs.size() * 4, s);
    hy_check(hy_table_scan_count(descs.data(), static_cast<uint32_t>(descs.size()), d_counts.as<uint32_t>(), ws.get(),
                                 ws.bytes(), s),
             "hy_table_scan_count");
    counts.assign(descs.size(), 0);
    hy_check(hy_memcpy_dtoh(counts.data(), d_counts.get(), 4 * descs.size(), s), "hy_memcpy_dtoh");
    hy_check(hy_stream_synchronize(s), "sync");
    uint64_t n = 0;
    for (const uint32_t c : counts) n += c;
    return n;
  }
  // the output chunks over `rows` laid out by `counts` (chunk k's RowIDs at the sum of the counts before it)
  std::vector<std::shared_ptr<Chunk>> chunks_for(const std::shared_ptr<DeviceBuffer>& rows) const {
    std::vector<std::pair<uint64_t, uint32_t>> views;
    uint64_t at = 0;
    for (const uint32_t c : counts) {
      views.emplace_back(at, c);
      at += c;
    }
    return chunks_from(rows, views);
  }

  // the predicate as the fused join's filter can take it: every chunk a dictionary chunk of one id width (the
  // hy_table_scan_count preconditions), no IS NULL, every chunk of the table scanned
  bool fusable() const {
    if (!all_chunks || descs.empty()) return false;
    // the descriptors were built when the scan executed: the table may have grown since (Table::append_chunks)
    if (descs.size() != in_table->chunk_count()) return false;
    for (size_t k = 0; k < descs.size(); ++k)
      if (in_table->get_chunk(chunk_ids[k])->size() != sizes[k]) return false;
    int width = 0;
    for (const auto& d : descs) {
      if (d.column.kind != HY_COL_DICT || d.op == HY_OP_IS_NULL || d.op == HY_OP_IS_NOT_NULL || d.op == HY_OP_VID_SET)
        return false;
      if ((reinterpret_cast<uintptr_t>(d.column.data) & 15u) != 0) return false;
      if (d.column.size) {
        if (width && width != d.column.vid_width) return false;
        width = d.column.vid_width;
      }
    }
    return true;
  }
};

// HY_OP_FUSE_SCAN=0: TableScans run when they execute (no deferral, no fusion into JoinHash)
bool scan_fusion_enabled() {
  const char* e = std::getenv("HY_OP_FUSE_SCAN");
  return !(e && std::atoi(e) == 0);
}

}  // namespace

std::shared_ptr<const Table> TableScan::_on_execute() {
  const auto in_table = input_table_left();
  // the reference's scan impls boost::get the value / column id: an unset placeholder cannot execute
  if (is_parameter_id(_right_parameter))
    Fail("TableScan: parameter " + std::to_string(std::get<ParameterID>(_right_parameter).t) +
         " has no value (set_parameters first)");
  static const AllTypeVariant no_value{};
  const AllTypeVariant& right_value = is_variant(_right_parameter) ? std::get<AllTypeVariant>(_right_parameter)
                                                                      : no_value;
  const ColumnID right_column_id =
      is_column_id(_right_parameter) ? std::get<ColumnParameter>(_right_parameter).column_id : INVALID_COLUMN_ID;
  switch (_predicate_condition) {
    case PredicateCondition::In:
      Fail("hyrise-amd: predicate " + predicate_condition_to_string(_predicate_condition) +
           " is not supported by the device TableScan");
    case PredicateCondition::Between:
      Fail("Unsupported comparison type encountered");  // reference: BETWEEN is split before it reaches the scan
    default:
      break;
  }
  if (right_column_id != INVALID_COLUMN_ID) {
    // ColumnComparisonTableScanImpl (table_scan.cpp:191-199, column_comparison_table_scan_impl.cpp:23-84)
    Assert(_predicate_condition != PredicateCondition::IsNull && _predicate_condition != PredicateCondition::IsNotNull,
           "Unsupported comparison type encountered");
    std::vector<bool> excluded(in_table->chunk_count(), false);
    for (const auto c : _excluded_chunk_ids)
      if (c < excluded.size()) excluded[c] = true;
    _performance_data.rows_in = in_table->row_count();
    return column_comparison_scan(in_table, _left_column_id, _predicate_condition, right_column_id, excluded);
  }
  if (_predicate_condition == PredicateCondition::Like || _predicate_condition == PredicateCondition::NotLike)
    Assert(in_table->column_data_type(_left_column_id) == DataType::String,
           "LIKE operator only applicable on string columns.");  // table_scan.cpp:170-171
  auto output = std::make_shared<Table>(in_table->column_definitions(), TableType::References);
  std::vector<std::shared_ptr<DeviceBuffer>> keep;  // LIKE id sets of the descriptors
  const bool like = _predicate_condition == PredicateCondition::Like ||
                    _predicate_condition == PredicateCondition::NotLike;
  const bool null_test =
      _predicate_condition == PredicateCondition::IsNull || _predicate_condition == PredicateCondition::IsNotNull;
  // reference single_column_table_scan_impl.cpp:23-36: comparing with NULL matches nothing (IS [NOT] NULL ignores the
  // right value, table_scan.cpp:186-189)
  if (!null_test && variant_is_null(right_value)) return output;
  require_device();
  hy_stream_t s = operator_stream();
  const auto col_type = in_table->column_data_type(_left_column_id);
  std::vector<bool> excluded(in_table->chunk_count(), false);
  for (const auto c : _excluded_chunk_ids)
    if (c < excluded.size()) excluded[c] = true;
  _performance_data.rows_in = in_table->row_count();

  if (in_table->type() == TableType::Data) {
    PhaseTrace tr{"TableScan"};
    std::vector<hy_scan_chunk> descs;
    std::vector<ChunkID> chunk_ids;
    std::vector<uint32_t> sizes;
    std::vector<size_t> like_offs;
    LikeBatch like_sets;
    uint64_t total = 0;
    for (ChunkID c = 0; c < in_table->chunk_count(); ++c)
      if (!excluded[c]) chunk_ids.push_back(c);
    descs.resize(chunk_ids.size());
    like_offs.assign(chunk_ids.size(), SIZE_MAX);
    sizes.resize(chunk_ids.size());
    // the descriptors (dictionary rewrite per chunk, ~0.25 us each: 1.5 ms for SF100's 6,000 chunks on one thread)
    // by jobs of the host's scheduler; LIKE patterns share one batch of id sets and stay on this thread
    auto describe = [&](size_t k0, size_t k1, LikeBatch* batch) {
      for (size_t k = k0; k < k1; ++k) {
        const auto column = in_table->get_chunk(chunk_ids[k])->get_column(_left_column_id);
        descs[k] = scan_descriptor(*column, col_type, _predicate_condition, right_value, batch, &like_offs[k]);
        sizes[k] = static_cast<uint32_t>(column->size());
      }
    };
    constexpr size_t CHUNKS_PER_JOB = 512;
    if (like || chunk_ids.size() < 2 * CHUNKS_PER_JOB) {
      describe(0, chunk_ids.size(), &like_sets);
    } else {
      JobGroup jobs;
      const size_t n_jobs = std::min<size_t>(jobs.concurrency(host_cpu_share()),
                                             (chunk_ids.size() + CHUNKS_PER_JOB - 1) / CHUNKS_PER_JOB);
      const size_t per = (chunk_ids.size() + n_jobs - 1) / n_jobs;
      for (size_t j = 0; j < n_jobs; ++j)
        jobs.schedule([&, j] {
          LikeBatch unused;
          describe(j * per, std::min(chunk_ids.size(), (j + 1) * per), &unused);
        });
      jobs.wait();
    }
    for (size_t k = 0; k < descs.size(); ++k) {
      descs[k].out_begin = total;
      total += sizes[k];
    }
    if (descs.empty()) return output;
    for (size_t k = 0; k < descs.size(); ++k)
      if (like_offs[k] != SIZE_MAX) like_sets.fix.emplace_back(&descs[k], like_offs[k]);
    like_sets.finish(&keep);
    tr.mark("descriptors");
    if (col_type != DataType::String && !like && scan_fusion_enabled()) {
      // deferred: the scan runs when its output is first read, or inside the JoinHash that consumes it
      auto scan = std::make_shared<DataScan>();
      scan->in_table = in_table;
      scan->column_id = _left_column_id;
      scan->col_type = col_type;
      scan->descs = std::move(descs);
      scan->chunk_ids = std::move(chunk_ids);
      scan->sizes = std::move(sizes);
      scan->constant = null_test ? ScanConstant{} : typed_constant(col_type, right_value);
      scan->total = total;
      scan->all_chunks = scan->descs.size() == in_table->chunk_count();
      output->set_pending(std::move(scan));
      tr.mark("deferred");
      return output;
    }
    auto rows = std::make_shared<DeviceBuffer>(std::max<uint64_t>(total, 1) * sizeof(RowID));
    DeviceBuffer counts(descs.size() * 4, s);
    std::vector<uint32_t> h_counts(descs.size());
    std::vector<std::pair<uint64_t, uint32_t>> views;  // (offset, count) per chunk
    if (col_type == DataType::String) {
      // string column (unencoded and / or dictionary chunks): the matches arrive compacted, chunk-major
      const StringScanPredicate sp(_predicate_condition, right_value);
      size_t ws_bytes = 0;
      hy_check(hy_string_table_scan_workspace_size(descs.data(), static_cast<uint32_t>(descs.size()), &sp.pred,
                                                   &ws_bytes),
               "hy_string_table_scan_workspace_size");
      DeviceBuffer ws(ws_bytes, s), n_out(8, s);
      hy_check(hy_string_table_scan(descs.data(), static_cast<uint32_t>(descs.size()), &sp.pred, chunk_ids.data(),
                                    rows->as<hy_row_id>(), counts.as<uint32_t>(), n_out.as<uint64_t>(), ws.get(),
                                    ws_bytes, s),
               "hy_string_table_scan");
      hy_check(hy_memcpy_dtoh(h_counts.data(), counts.get(), 4 * descs.size(), s), "hy_memcpy_dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
      uint64_t at = 0;
      for (size_t k = 0; k < descs.size(); ++k) {
        views.emplace_back(at, h_counts[k]);
        at += h_counts[k];
      }
    } else {
      const auto constant = null_test || like ? ScanConstant{} : typed_constant(col_type, right_value);
      size_t ws_bytes = 0;
      hy_check(hy_table_scan_workspace_size(sizes.data(), static_cast<uint32_t>(sizes.size()), &ws_bytes),
               "hy_table_scan_workspace_size");
      DeviceBuffer ws(ws_bytes, s);
      // one launch writes every chunk's output RowIDs {chunk id, offset} at its input row range of `rows` (the
      // PosLists the output chunks share), so no per-chunk expansion launch follows
      hy_check(hy_table_scan_row_ids(descs.data(), static_cast<uint32_t>(descs.size()), hy_type_of(col_type),
                                     constant.bytes, chunk_ids.data(), rows->as<hy_row_id>(), counts.as<uint32_t>(),
                                     ws.get(), ws_bytes, s),
               "hy_table_scan_row_ids");
      tr.mark("scan launched");
      hy_check(hy_memcpy_dtoh(h_counts.data(), counts.get(), 4 * descs.size(), s), "hy_memcpy_dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
      for (size_t k = 0; k < descs.size(); ++k) views.emplace_back(descs[k].out_begin, h_counts[k]);
    }
    tr.mark("counts synchronised");
    {  // algorithmic bytes: the predicate column's stored bytes (ids / values), 8 B per output RowID
      uint64_t rd = 0, wr = 0;
      for (size_t k = 0; k < descs.size(); ++k) {
        const auto& c = descs[k].column;
        rd += uint64_t(sizes[k]) * (c.kind == HY_COL_DICT ? c.vid_width : col_type == DataType::String ? 4 : data_type_size(col_type));
        wr += uint64_t(views[k].second) * sizeof(RowID);
      }
      _performance_data.bytes_read = rd;
      _performance_data.bytes_written = wr;
    }
    // output PosLists are lazy views of `rows` (no copy to the host, no wait: later work is ordered on the stream);
    // chunks, columns and PosLists from an output arena (device.hpp)
    OutputArena arena;
    std::vector<std::shared_ptr<Chunk>> out_chunks;
    for (size_t k = 0; k < descs.size(); ++k) {
      if (views[k].second == 0) continue;  // reference table_scan.cpp:99: no empty output chunks
      auto pl = pos_list_from_device(arena, rows, views[k].first, views[k].second);
      pl->set_single_chunk_id(chunk_ids[k]);
      ChunkColumns cols;
      cols.reserve(in_table->column_count());
      for (ColumnID col = 0; col < in_table->column_count(); ++col)
        cols.push_back(arena_reference_column(arena, in_table, col, pl));
      out_chunks.push_back(arena_chunk(arena, std::move(cols)));
    }
    output->append_chunks(std::move(out_chunks));
    tr.mark("output chunks");
    return output;
  }

  // ---- reference-table input (base_single_column_table_scan_impl.cpp:36-60, table_scan.cpp:104-145) ----
  // the referenced chunks' descriptors (dictionary rewrite, LIKE id sets uploaded) once per referenced table and column,
  // not once per input chunk
  std::map<std::pair<const Table*, ColumnID>, std::vector<hy_scan_chunk>> rdescs;
  for (ChunkID c = 0; c < in_table->chunk_count(); ++c) {
    if (excluded[c]) continue;
    const auto chunk = in_table->get_chunk(c);
    const auto ref = std::dynamic_pointer_cast<const ReferenceColumn>(chunk->get_column(_left_column_id));
    Assert(ref != nullptr, "All columns should be of type ReferenceColumn.");
    const auto& pos_list = *ref->pos_list();
    if (pos_list.empty()) continue;
    const auto& rtable = ref->referenced_table();
    const ColumnID rcol = ref->referenced_column_id();
    auto& rdesc = rdescs[{rtable.get(), rcol}];
    if (rdesc.empty()) {
      rdesc.resize(rtable->chunk_count());
      LikeBatch like_sets;
      for (ChunkID r = 0; r < rtable->chunk_count(); ++r) {
        size_t off;
        rdesc[r] = scan_descriptor(*rtable->get_chunk(r)->get_column(rcol), col_type, _predicate_condition,
                                   right_value, &like_sets, &off);
        if (off != SIZE_MAX) like_sets.fix.emplace_back(&rdesc[r], off);  // (rdesc is sized: no reallocation)
      }
      like_sets.finish(&keep);
    }
    const auto constant = null_test || like ? ScanConstant{} : typed_constant(col_type, right_value);
    const auto dpl = device_pos_list(pos_list);
    const uint64_t m = pos_list.size();

    // distinct referenced chunks in order of first appearance -> the reference's unordered_map iteration order; a
    // PosList whose producer knows its only chunk (a TableScan's output) is one group without a device pass
    std::vector<ChunkID> seen;
    if (pos_list.single_chunk_id() != INVALID_CHUNK_ID) {
      seen.push_back(pos_list.single_chunk_id());
    } else {
      DeviceBuffer first(std::max<size_t>(rtable->chunk_count(), 1) * 8, s);
      hy_check(hy_pos_list_chunk_first_seen(dpl->ptr(), m, rtable->chunk_count(), first.as<uint64_t>(), s),
               "hy_pos_list_chunk_first_seen");
      std::vector<uint64_t> h_first(rtable->chunk_count());
      hy_check(hy_memcpy_dtoh(h_first.data(), first.get(), 8 * h_first.size(), s), "dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
      for (ChunkID r = 0; r < h_first.size(); ++r)
        if (h_first[r] != ~0ull) seen.push_back(r);
      std::sort(seen.begin(), seen.end(), [&](ChunkID a, ChunkID b) { return h_first[a] < h_first[b]; });
    }
    const auto groups = unordered_map_order(seen);

    const bool strings = col_type == DataType::String;
    const StringScanPredicate sp(_predicate_condition, right_value);
    size_t ws_bytes = 0;  // also the workspace of hy_pos_list_null_positions
    hy_check(hy_reference_scan_workspace_size(m, &ws_bytes), "hy_reference_scan_workspace_size");
    if (strings) {
      size_t sb = 0;
      hy_check(hy_string_reference_scan_workspace_size(m, static_cast<uint32_t>(rdesc.size()), &sp.pred, &sb),
               "hy_string_reference_scan_workspace_size");
      ws_bytes = std::max(ws_bytes, sb);
    }
    DeviceBuffer ws(ws_bytes, s);
    DeviceBuffer positions(std::max<uint64_t>(m, 1) * 4, s);
    DeviceBuffer count(8, s);
    // one scan over all referenced chunks: matching positions ascending
    auto scan_into = [&](uint32_t* out) {
      if (strings)
        hy_check(hy_string_reference_scan(dpl->ptr(), m, rdesc.data(), static_cast<uint32_t>(rdesc.size()), &sp.pred,
                                          out, count.as<uint64_t>(), ws.get(), ws_bytes, s),
                 "hy_string_reference_scan");
      else
        hy_check(hy_reference_scan(dpl->ptr(), m, rdesc.data(), static_cast<uint32_t>(rdesc.size()),
                                   hy_type_of(col_type), constant.bytes, out, count.as<uint64_t>(), ws.get(), ws_bytes,
                                   s),
                 "hy_reference_scan");
    };
    uint64_t total = 0;
    if (groups.size() <= 1) {
      scan_into(positions.as<uint32_t>());
      hy_check(hy_memcpy_dtoh(&total, count.get(), 8, s), "dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
    } else {
      // all referenced chunks in one scan (ascending positions), then the matches reordered into the unordered_map's
      // group order (positions ascending inside each group) by one stable sort on the device
      DeviceBuffer asc(std::max<uint64_t>(m, 1) * 4, s);
      scan_into(asc.as<uint32_t>());
      hy_check(hy_memcpy_dtoh(&total, count.get(), 8, s), "dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
      std::vector<uint32_t> rank(rtable->chunk_count(), 0);
      for (size_t g = 0; g < groups.size(); ++g) rank[groups[g]] = static_cast<uint32_t>(g);
      DeviceBuffer d_rank(rank.size() * 4, s);
      hy_check(hy_memcpy_htod(d_rank.get(), rank.data(), rank.size() * 4, s), "htod");
      size_t ob = 0;
      hy_check(hy_reference_scan_order_workspace_size(total, static_cast<uint32_t>(groups.size()), &ob),
               "hy_reference_scan_order_workspace_size");
      DeviceBuffer ows(ob, s);
      hy_check(hy_reference_scan_order(dpl->ptr(), asc.as<uint32_t>(), total, d_rank.as<uint32_t>(),
                                       static_cast<uint32_t>(rank.size()), static_cast<uint32_t>(groups.size()),
                                       positions.as<uint32_t>(), ows.get(), ob, s),
               "hy_reference_scan_order");
      hy_check(hy_stream_synchronize(s), "sync");  // d_rank / asc / ows are released at scope end
    }
    if (_predicate_condition == PredicateCondition::IsNull) {
      // IsNullTableScanImpl::handle_column(const ReferenceColumn&) (is_null_table_scan_impl.cpp:20-33): the NULL
      // RowIDs of the referencing column match too, appended after the referenced columns' matches
      uint64_t nulls = 0;
      hy_check(hy_pos_list_null_positions(dpl->ptr(), m, positions.as<uint32_t>() + total, count.as<uint64_t>(),
                                          ws.get(), ws_bytes, s),
               "hy_pos_list_null_positions");
      hy_check(hy_memcpy_dtoh(&nulls, count.get(), 8, s), "dtoh");
      hy_check(hy_stream_synchronize(s), "sync");
      total += nulls;
    }
    if (total == 0) continue;
    // filtered PosLists, shared per distinct input PosList (table_scan.cpp:115-145)
    std::map<const PosList*, std::shared_ptr<PosList>> filtered;
    ChunkColumns cols;
    for (ColumnID col = 0; col < in_table->column_count(); ++col) {
      const auto rc = std::dynamic_pointer_cast<const ReferenceColumn>(chunk->get_column(col));
      Assert(rc != nullptr, "All columns should be of type ReferenceColumn.");
      auto& f = filtered[rc->pos_list().get()];
      if (!f) {
        const auto src = device_pos_list(*rc->pos_list());
        auto rows = std::make_shared<DeviceBuffer>(total * sizeof(RowID));
        hy_check(hy_gather_row_ids(src->ptr(), positions.as<uint32_t>(), total, rows->as<hy_row_id>(), s),
                 "hy_gather_row_ids");
        hy_check(hy_stream_synchronize(s), "sync");
        f = pos_list_from_device(rows, 0, total);
        f->set_single_chunk_id(rc->pos_list()->single_chunk_id());  // a filtered PosList stays within its chunk
      }
      cols.push_back(std::make_shared<ReferenceColumn>(rc->referenced_table(), rc->referenced_column_id(), f));
    }
    output->append_chunk(cols);
  }
  return output;
}

// ================================================================================================================
// Validate
// ================================================================================================================
namespace {

// Device descriptors of a table's MVCC columns; each chunk's HBM copy is made once and cached on its MvccColumns.
struct DeviceMvcc {
  std::vector<hy_mvcc_chunk> chunks;
  std::vector<std::shared_ptr<DeviceBuffer>> keep;
};

DeviceMvcc upload_mvcc(const Table& table, hy_stream_t s) {
  DeviceMvcc out;
  for (ChunkID c = 0; c < table.chunk_count(); ++c) {
    const auto chunk = table.get_chunk(c);
    const auto m = chunk->mvcc_columns();
    Assert(m != nullptr, "Trying to use Validate on a table that has no MVCC columns");
    // validate.cpp:101 iterates the chunk's rows: the MVCC vectors must cover them (they may be longer, as the
    // reference's are while a chunk is being filled)
    const uint64_t n = chunk->size();
    Assert(m->tids.size() >= n && m->begin_cids.size() >= n && m->end_cids.size() >= n,
           "MVCC columns shorter than the chunk");
    std::shared_ptr<DeviceBuffer> buf;
    {
      std::lock_guard<std::mutex> lock(m->device_mutex);
      buf = std::static_pointer_cast<DeviceBuffer>(m->device);
      if (buf && m->device_rows != n) buf.reset();  // the chunk grew since the copy was made
      if (!buf) {  // first use: one upload of the chunk's three vectors, kept with the MvccColumns
        buf = std::make_shared<DeviceBuffer>(std::max<uint64_t>(3 * n, 4) * 4);
        if (n) {
          hy_check(hy_memcpy_htod(buf->get(), m->tids.data(), 4 * n, s), "htod");
          hy_check(hy_memcpy_htod(buf->as<uint32_t>() + n, m->begin_cids.data(), 4 * n, s), "htod");
          hy_check(hy_memcpy_htod(buf->as<uint32_t>() + 2 * n, m->end_cids.data(), 4 * n, s), "htod");
          // published only once the copies have landed: another thread's Validate may use the cached buffer on its
          // own stream right after the lock is released
          hy_check(hy_stream_synchronize(s), "sync");
        }
        m->device = buf;
        m->device_rows = n;
      }
    }
    const uint32_t* base = buf->as<uint32_t>();
    out.chunks.push_back(hy_mvcc_chunk{base, base + n, base + 2 * n, static_cast<uint32_t>(n), 0});
    out.keep.push_back(std::move(buf));
  }
  hy_check(hy_stream_synchronize(s), "sync");
  return out;
}

}  // namespace

std::shared_ptr<const Table> Validate::_on_execute() {
  Fail("Validate can't be called without a transaction context.");
}

std::shared_ptr<const Table> Validate::_on_execute(std::shared_ptr<TransactionContext> transaction_context) {
  if (!transaction_context) return _on_execute();
  const uint32_t _transaction_id = transaction_context->transaction_id();
  const uint32_t _snapshot_commit_id = transaction_context->snapshot_commit_id();
  const auto in_table = input_table_left();
  auto output = std::make_shared<Table>(in_table->column_definitions(), TableType::References);
  if (in_table->chunk_count() == 0) return output;
  require_device();
  hy_stream_t s = operator_stream();
  _performance_data.rows_in = in_table->row_count();
  if (in_table->type() == TableType::Data) {
    const auto mvcc = upload_mvcc(*in_table, s);
    std::vector<uint32_t> ids(in_table->chunk_count());
    std::iota(ids.begin(), ids.end(), 0u);
    const uint64_t rows = in_table->row_count();
    size_t ws_bytes = 0;
    hy_check(hy_validate_workspace_size(rows, in_table->chunk_count(), &ws_bytes), "hy_validate_workspace_size");
    DeviceBuffer ws(ws_bytes, s), counts(in_table->chunk_count() * 4, s), n_out(8, s);
    auto out_rows = std::make_shared<DeviceBuffer>(std::max<uint64_t>(rows, 1) * sizeof(RowID));
    hy_check(hy_validate(mvcc.chunks.data(), in_table->chunk_count(), ids.data(), _transaction_id, _snapshot_commit_id,
                         out_rows->as<hy_row_id>(), counts.as<uint32_t>(), n_out.as<uint64_t>(), ws.get(), ws_bytes, s),
             "hy_validate");
    std::vector<uint32_t> h_counts(in_table->chunk_count());
    hy_check(hy_memcpy_dtoh(h_counts.data(), counts.get(), 4 * h_counts.size(), s), "dtoh");
    hy_check(hy_stream_synchronize(s), "sync");
    uint64_t begin = 0;
    for (ChunkID c = 0; c < in_table->chunk_count(); ++c) {
      if (h_counts[c] == 0) continue;  // validate.cpp:89-91: no empty output chunks
      auto pl = pos_list_from_device(out_rows, begin, h_counts[c]);
      pl->set_single_chunk_id(c);
      ChunkColumns cols;
      for (ColumnID col = 0; col < in_table->column_count(); ++col)
        cols.push_back(std::make_shared<ReferenceColumn>(in_table, col, pl));
      output->append_chunk(cols);
      begin += h_counts[c];
    }
    return output;
  }
  // reference input (validate.cpp:47-70): column 0's PosList, checked against the referenced table's MVCC columns,
  // becomes the PosList of every output column of the chunk
  std::map<const Table*, DeviceMvcc> uploaded;
  for (ChunkID c = 0; c < in_table->chunk_count(); ++c) {
    const auto chunk = in_table->get_chunk(c);
    const auto ref0 = std::dynamic_pointer_cast<const ReferenceColumn>(chunk->get_column(0));
    Assert(ref0 != nullptr, "All columns should be of type ReferenceColumn.");
    const auto& referenced = ref0->referenced_table();
    auto it = uploaded.find(referenced.get());
    if (it == uploaded.end()) it = uploaded.emplace(referenced.get(), upload_mvcc(*referenced, s)).first;
    const auto& pos_list = *ref0->pos_list();
    const uint64_t n = pos_list.size();
    if (n == 0) continue;
    const auto dpl = device_pos_list(pos_list);
    size_t ws_bytes = 0;
    hy_check(hy_validate_workspace_size(n, referenced->chunk_count(), &ws_bytes), "hy_validate_workspace_size");
    DeviceBuffer ws(ws_bytes, s), n_out(8, s);
    auto out_rows = std::make_shared<DeviceBuffer>(n * sizeof(RowID));
    hy_check(hy_validate_pos_list(dpl->ptr(), n, it->second.chunks.data(), referenced->chunk_count(), _transaction_id,
                                  _snapshot_commit_id, out_rows->as<hy_row_id>(), n_out.as<uint64_t>(), ws.get(),
                                  ws_bytes, s),
             "hy_validate_pos_list");
    uint64_t visible = 0;
    hy_check(hy_memcpy_dtoh(&visible, n_out.get(), 8, s), "dtoh");
    hy_check(hy_stream_synchronize(s), "sync");
    if (visible == 0) continue;
    auto pl = pos_list_from_device(out_rows, 0, visible);
    pl->set_single_chunk_id(ref0->pos_list()->single_chunk_id());
    ChunkColumns cols;
    for (ColumnID col = 0; col < in_table->column_count(); ++col) {
      const auto rc = std::static_pointer_cast<const ReferenceColumn>(chunk->get_column(col));
      cols.push_back(std::make_shared<ReferenceColumn>(referenced, rc->referenced_column_id(), pl));
    }
    output->append_chunk(cols);
  }
  return output;
}

// ================================================================================================================
// JoinHash
// ================================================================================================================
DataType join_hashed_type(DataType l, DataType r) {
  auto is_float = [](DataType t) { return t == DataType::Float || t == DataType::Double; };
  if (l == DataType::String || r == DataType::String) return DataType::String;
  if (is_float(l) && is_float(r)) return data_type_size(l) < data_type_size(r) ? r : l;
  if (!is_float(l) && !is_float(r)) return data_type_size(l) < data_type_size(r) ? r : l;
  return is_float(l) ? l : r;
}

namespace {

using PosListsVec = std::vector<std::shared_ptr<const PosList>>;

struct JoinSideInput {
  std::vector<hy_join_chunk> chunks;
  std::vector<hy_column_chunk> referenced;
  int32_t fuse = 0;
  // per-column PosList groups for reference tables (setup_pos_lists_by_column, join_hash.cpp:533-562)
  std::vector<int> column_group;         // column -> group id
  std::vector<PosListsVec> groups;       // group id -> per-chunk PosLists
  int join_group = -1;
  uint32_t n_referenced_tables = 0;  // distinct (table, column) pairs the join column's chunks reference
};

// String join keys (JoinHashTraits HashType std::string, hash_traits.hpp:36-41; the other side lexically cast):
// every distinct string of both sides gets an int32 id ("" = 0, the value NULL rows carry), the device joins the ids,
// and key_hash[id] = murmur2(string, 17) (murmur_hash.hpp:16-20) makes the radix partitioning the reference's. The
// id columns are built on the host per column chunk (the device holds no string bytes): dictionary chunks map their
// dictionary once and each row through its value id, other chunks row by row.
struct StringKeys {
  std::unordered_map<std::string, int32_t> ids{{"", 0}};
  std::vector<uint32_t> hashes{hy_murmur2_bytes("", 0, 17)};
  std::vector<std::shared_ptr<DeviceBuffer>> keep;  // id / NULL-flag chunks (alive until the join has run)
  std::shared_ptr<DeviceBuffer> d_hashes;

  int32_t id_of(const std::string& v) {
    auto it = ids.find(v);
    if (it != ids.end()) return it->second;
    const auto id = static_cast<int32_t>(hashes.size());
    ids.emplace(v, id);
    hashes.push_back(hy_murmur2_bytes(v.data(), static_cast<uint32_t>(v.size()), 17));
    return id;
  }

  hy_column_chunk map(const BaseColumn& column) {
    const size_t n = column.size();
    std::vector<int32_t> vals(std::max<size_t>(n, 1) + 4, 0);
    std::vector<uint8_t> nulls(std::max<size_t>(n, 1) + 16, 0);
    bool any_null = false;
    if (const auto* dict = dynamic_cast<const BaseDictionaryColumn*>(&column)) {
      std::vector<int32_t> entry(dict->unique_values_count());
      for (size_t v = 0; v < entry.size(); ++v)  // the dictionary's values through the column's operator[]
        entry[v] = -1;
      const auto& av = dict->attribute_vector();
      for (size_t i = 0; i < n; ++i) {
        const uint32_t vid = av.get(i);
        if (vid >= entry.size()) {
          nulls[i] = 1;
          any_null = true;
          continue;
        }
        if (entry[vid] < 0) entry[vid] = id_of(type_cast<std::string>(column[static_cast<ChunkOffset>(i)]));
        vals[i] = entry[vid];
      }
    } else {
      for (size_t i = 0; i < n; ++i) {
        const auto v = column[static_cast<ChunkOffset>(i)];
        if (variant_is_null(v)) {
          nulls[i] = 1;
          any_null = true;
        } else {
          vals[i] = id_of(type_cast<std::string>(v));
        }
      }
    }
    hy_stream_t s = operator_stream();
    auto d_vals = std::make_shared<DeviceBuffer>(vals.size() * 4);
    hy_check(hy_memcpy_htod(d_vals->get(), vals.data(), vals.size() * 4, s), "htod");
    keep.push_back(d_vals);
    hy_column_chunk c{};
    c.data = d_vals->get();
    c.size = static_cast<uint32_t>(n);
    c.kind = HY_COL_VALUE;
    if (any_null) {
      auto d_nulls = std::make_shared<DeviceBuffer>(nulls.size());
      hy_check(hy_memcpy_htod(d_nulls->get(), nulls.data(), nulls.size(), s), "htod");
      keep.push_back(d_nulls);
      c.nulls = static_cast<const uint8_t*>(d_nulls->get());
    }
    hy_check(hy_stream_synchronize(s), "sync");  // the host vectors are pageable
    return c;
  }

  const uint32_t* upload_hashes() {
    hy_stream_t s = operator_stream();
    d_hashes = std::make_shared<DeviceBuffer>(hashes.size() * 4);
    hy_check(hy_memcpy_htod(d_hashes->get(), hashes.data(), hashes.size() * 4, s), "htod");
    hy_check(hy_stream_synchronize(s), "sync");
    return d_hashes->as<uint32_t>();
  }
};

JoinSideInput describe_side(const std::shared_ptr<const Table>& table, ColumnID column_id,
                            StringKeys* strings = nullptr) {
  auto chunk_desc = [&](const BaseColumn& column) {
    return strings ? strings->map(column) : device_column(column)->desc;
  };
  JoinSideInput in;
  const bool is_ref = table->type() == TableType::References;
  const auto& chunks = table->chunks();
  const auto ref_column = [&](ChunkID c, ColumnID col) -> const ReferenceColumn& {
    return static_cast<const ReferenceColumn&>(*chunks[c]->columns()[col]);
  };
  if (is_ref) {
    std::map<PosListsVec, int> ids;
    for (ColumnID col = 0; col < table->column_count(); ++col) {
      PosListsVec v;
      v.reserve(chunks.size());
      for (ChunkID c = 0; c < chunks.size(); ++c) v.push_back(ref_column(c, col).pos_list());
      auto it = ids.find(v);
      if (it == ids.end()) {
        it = ids.emplace(v, static_cast<int>(in.groups.size())).first;
        in.groups.push_back(v);
      }
      in.column_group.push_back(it->second);
    }
    in.join_group = in.column_group.at(column_id);
  }
  // The referenced (table, column) pairs of the join column in order of first appearance; their chunks are listed one
  // table after the other in `referenced` (a reference table's chunks may reference different tables: each row is
  // read from its own chunk's table, as the reference's ReferenceColumn iterable does, join_hash.cpp:248-276).
  std::vector<std::pair<const Table*, ColumnID>> ref_tables;
  std::vector<uint32_t> ref_offsets;
  const Table* referenced = nullptr;
  ColumnID rcol = 0;
  in.chunks.reserve(chunks.size());
  for (ChunkID c = 0; c < chunks.size(); ++c) {
    const BaseColumn& column = *chunks[c]->columns().at(column_id);
    hy_join_chunk jc{};
    jc.chunk_id = c;
    jc.single_chunk = HY_MIXED_CHUNKS;
    jc.size = static_cast<uint32_t>(column.size());
    if (is_ref) {
      const auto& rc = static_cast<const ReferenceColumn&>(column);
      const std::pair<const Table*, ColumnID> key{rc.referenced_table().get(), rc.referenced_column_id()};
      auto it = std::find(ref_tables.begin(), ref_tables.end(), key);
      if (it == ref_tables.end()) {
        ref_offsets.push_back(ref_tables.empty() ? 0u
                                                 : ref_offsets.back() + static_cast<uint32_t>(
                                                                            ref_tables.back().first->chunk_count()));
        ref_tables.push_back(key);
        it = ref_tables.end() - 1;
      }
      jc.referenced_offset = ref_offsets[it - ref_tables.begin()];
      const PosList& pl = *rc.pos_list();
      jc.pos_list = device_pos_list(pl)->ptr();
      if (pl.single_chunk_id() != INVALID_CHUNK_ID) jc.single_chunk = jc.referenced_offset + pl.single_chunk_id();
    } else {
      jc.column = chunk_desc(column);
    }
    in.chunks.push_back(jc);
  }
  in.n_referenced_tables = static_cast<uint32_t>(ref_tables.size());
  if (!ref_tables.empty()) {
    referenced = ref_tables[0].first;
    rcol = ref_tables[0].second;
    for (const auto& [table, col] : ref_tables)
      for (const auto& rch : table->chunks()) in.referenced.push_back(chunk_desc(*rch->columns().at(col)));
  }
  if (referenced) {
    // fuse the dereference when every column shares the join column's PosLists and its one referenced table
    bool fuse = ref_tables.size() == 1;
    for (ColumnID col = 0; col < table->column_count() && fuse; ++col) {
      if (in.column_group[col] != in.join_group) fuse = false;
      for (ChunkID c = 0; c < chunks.size() && fuse; ++c)
        if (ref_column(c, col).referenced_table().get() != referenced) fuse = false;
    }
    in.fuse = fuse ? 1 : 0;
  }
  return in;
}

std::shared_ptr<Table> column_comparison_scan(const std::shared_ptr<const Table>& in_table, ColumnID left_column_id,
                                              PredicateCondition cond, ColumnID right_column_id,
                                              const std::vector<bool>& excluded) {
  auto output = std::make_shared<Table>(in_table->column_definitions(), TableType::References);
  const auto lt = in_table->column_data_type(left_column_id);
  const auto rt = in_table->column_data_type(right_column_id);
  Assert((lt == DataType::String) == (rt == DataType::String), "Invalid column combination detected!");
  require_device();
  hy_stream_t s = operator_stream();
  JoinSideInput l = describe_side(in_table, left_column_id);
  JoinSideInput r = describe_side(in_table, right_column_id);
  Assert(l.n_referenced_tables <= 1 && r.n_referenced_tables <= 1,
         "hyrise-amd: a column comparison over columns referencing several tables is not supported");
  std::vector<hy_join_chunk> lc, rc;
  for (ChunkID c = 0; c < in_table->chunk_count(); ++c) {
    if (excluded[c]) continue;
    lc.push_back(l.chunks[c]);
    rc.push_back(r.chunks[c]);
  }
  if (lc.empty()) return output;
  // string columns: packed strings on the device (value chunks and dictionaries), compared as std::string's operators
  const auto dtype = [](DataType t) { return t == DataType::String ? int32_t{HY_TYPE_STRING} : hy_type_of(t); };
  hy_join_side ls{lc.data(), static_cast<uint32_t>(lc.size()), dtype(lt), l.referenced.data(),
                  static_cast<uint32_t>(l.referenced.size()), 0, 0};
  hy_join_side rs{rc.data(), static_cast<uint32_t>(rc.size()), dtype(rt), r.referenced.data(),
                  static_cast<uint32_t>(r.referenced.size()), 0, 0};
  const bool is_ref = in_table->type() == TableType::References;
  size_t ws_bytes = 0;
  hy_check(hy_column_compare_scan_workspace_size(&ls, &rs, is_ref ? 0 : 1, &ws_bytes),
           "hy_column_compare_scan_workspace_size");
  DeviceBuffer ws(ws_bytes, s);
  uint64_t total_rows = 0;
  for (const auto& c : lc) total_rows += c.size;
  // data input: output RowIDs {chunk id, offset} (the PosLists); reference input: chunk offsets (positions to filter
  // the input PosLists with, table_scan.cpp:104-145)
  auto items = std::make_shared<DeviceBuffer>(std::max<uint64_t>(total_rows, 1) * (is_ref ? 4 : sizeof(RowID)));
  DeviceBuffer counts(lc.size() * 4, s), n_out(8, s);
  hy_check(hy_column_compare_scan(&ls, &rs, value_op(cond), is_ref ? nullptr : items->as<hy_row_id>(),
                                  is_ref ? items->as<uint32_t>() : nullptr, counts.as<uint32_t>(), n_out.as<uint64_t>(),
                                  ws.get(), ws_bytes, s),
           "hy_column_compare_scan");
  std::vector<uint32_t> h_counts(lc.size());
  hy_check(hy_memcpy_dtoh(h_counts.data(), counts.get(), 4 * lc.size(), s), "dtoh");
  hy_check(hy_stream_synchronize(s), "sync");
  uint64_t begin = 0;
  for (size_t k = 0; k < lc.size(); ++k) {
    const uint32_t n = h_counts[k];
    const ChunkID chunk_id = lc[k].chunk_id;
    if (n == 0) continue;  // no empty output chunks (table_scan.cpp:99)
    ChunkColumns cols;
    if (!is_ref) {
      auto pl = pos_list_from_device(items, begin, n);
      pl->set_single_chunk_id(chunk_id);
      for (ColumnID col = 0; col < in_table->column_count(); ++col)
        cols.push_back(std::make_shared<ReferenceColumn>(in_table, col, pl));
    } else {
      const auto chunk = in_table->get_chunk(chunk_id);
      std::map<const PosList*, std::shared_ptr<PosList>> filtered;
      for (ColumnID col = 0; col < in_table->column_count(); ++col) {
        const auto rcol = std::dynamic_pointer_cast<const ReferenceColumn>(chunk->get_column(col));
        Assert(rcol != nullptr, "All columns should be of type ReferenceColumn.");
        auto& f = filtered[rcol->pos_list().get()];
        if (!f) {
          const auto src = device_pos_list(*rcol->pos_list());
          auto rows = std::make_shared<DeviceBuffer>(static_cast<uint64_t>(n) * sizeof(RowID));
          hy_check(hy_gather_row_ids(src->ptr(), items->as<uint32_t>() + begin, n, rows->as<hy_row_id>(), s),
                   "hy_gather_row_ids");
          hy_check(hy_stream_synchronize(s), "sync");
          f = pos_list_from_device(rows, 0, n);
          f->set_single_chunk_id(rcol->pos_list()->single_chunk_id());
        }
        cols.push_back(std::make_shared<ReferenceColumn>(rcol->referenced_table(), rcol->referenced_column_id(), f));
      }
    }
    output->append_chunk(cols);
    begin += n;
  }
  return output;
}

int32_t join_mode(JoinMode m) {
  switch (m) {
    case JoinMode::Inner:
    case JoinMode::Outer:  // the reference's probe emits only matches for Outer (join_hash.cpp:405-435)
    case JoinMode::Cross:
      return HY_JOIN_INNER;
    case JoinMode::Left:
      return HY_JOIN_LEFT;
    case JoinMode::Right:
      return HY_JOIN_RIGHT;
    case JoinMode::Semi:
      return HY_JOIN_SEMI;
    case JoinMode::Anti:
      return HY_JOIN_ANTI;
  }
  return HY_JOIN_INNER;
}

// write_output_columns (join_hash.cpp:564-613), prepared once per side before the join runs: which table / column
// every output column references, and which device RowID array its PosList views - the join's output RowIDs (data
// tables, the fused dereference, an input without chunks), or that side's RowIDs dereferenced through one PosList
// group (reference inputs; computed for all partitions by a single launch once the join has run). Columns of one
// group share one PosList per chunk.
struct OutCol {
  const Table* table;
  ColumnID column;
  int group;  // -1: the side's one PosList (data-like side)
};
struct SideOut {
  std::vector<OutCol> cols;
  const DeviceBuffer* rows = nullptr;                  // data-like side
  std::vector<std::shared_ptr<DeviceBuffer>> deref;   // per group: dereferenced rows (allocated after the join)
  std::vector<std::shared_ptr<DeviceBuffer>> ptr_arrays;  // per group: the group's device PosList pointers
  int n_lists = 0;                                     // distinct PosLists per output chunk
};

// What one builder thread's output objects hold: aliasing pointers into this object's control block instead of
// copies of the tables' / buffers' own (shared by every thread: their reference counts would be contended).
struct OutRefs {
  std::vector<std::shared_ptr<const Table>> tables;
  std::vector<std::shared_ptr<DeviceBuffer>> buffers;
};

SideOut describe_output(const std::shared_ptr<const Table>& input_table, const JoinSideInput& side,
                        const std::shared_ptr<DeviceBuffer>& rows, OutRefs& refs, std::shared_ptr<Table>& dummy_table) {
  SideOut o;
  refs.buffers.push_back(rows);
  if (input_table->type() == TableType::Data || input_table->chunk_count() == 0) {
    std::shared_ptr<const Table> t = input_table;
    if (input_table->chunk_count() == 0 && input_table->type() != TableType::Data) {
      if (!dummy_table) dummy_table = Table::create_dummy_table(input_table->column_definitions());
      t = dummy_table;
    }
    refs.tables.push_back(t);
    o.rows = rows.get();
    for (ColumnID col = 0; col < input_table->column_count(); ++col) o.cols.push_back(OutCol{t.get(), col, -1});
    o.n_lists = 1;
    return o;
  }
  if (side.fuse) {
    o.rows = rows.get();
    o.n_lists = 1;
  } else {
    o.deref.assign(side.groups.size(), nullptr);
    o.ptr_arrays.assign(side.groups.size(), nullptr);
  }
  hy_stream_t s = operator_stream();
  for (ColumnID col = 0; col < input_table->column_count(); ++col) {
    const auto rc = std::static_pointer_cast<const ReferenceColumn>(input_table->get_chunk(0)->get_column(col));
    refs.tables.push_back(rc->referenced_table());
    const int g = side.fuse ? -1 : side.column_group[col];
    o.cols.push_back(OutCol{rc->referenced_table().get(), rc->referenced_column_id(), g});
    if (g < 0 || o.deref[g]) continue;
    std::vector<const hy_row_id*> ptrs;
    for (const auto& p : side.groups[g]) ptrs.push_back(device_pos_list(*p)->ptr());
    auto ptr_array = std::make_shared<DeviceBuffer>(ptrs.size() * sizeof(void*));
    hy_check(hy_memcpy_htod(ptr_array->get(), ptrs.data(), ptrs.size() * sizeof(void*), s), "htod");
    hy_check(hy_stream_synchronize(s), "sync");  // `ptrs` is pageable host memory
    o.ptr_arrays[g] = ptr_array;
    o.deref[g] = std::make_shared<DeviceBuffer>();  // (sized once the join's output range is known)
    refs.buffers.push_back(ptr_array);  // (freed with the outputs: the dereference launch may still read it)
    refs.buffers.push_back(o.deref[g]);
    ++o.n_lists;
  }
  return o;
}

// The dereferenced rows of a side's PosList groups, once the join has written `used` RowIDs.
void dereference_groups(SideOut& o, const DeviceBuffer& rows, uint64_t used) {
  hy_stream_t s = operator_stream();
  for (size_t g = 0; g < o.deref.size(); ++g) {
    if (!o.deref[g]) continue;
    DeviceBuffer d(std::max<uint64_t>(used, 1) * sizeof(RowID));
    o.deref[g]->swap(d);
    hy_check(hy_dereference_row_ids(rows.as<hy_row_id>(), used, o.ptr_arrays[g]->as<const hy_row_id* const>(),
                                    o.deref[g]->as<hy_row_id>(), s),
             "hy_dereference_row_ids");
  }
}

// The columns of one output chunk from a builder's arena, with empty PosLists whose views are set once the join's
// partition ranges are known; the chunk's distinct PosLists and mirrors go to lists / mirrors (side.n_lists each).
void write_chunk_columns(ChunkColumns& out, OutputArena& arena, const std::shared_ptr<OutRefs>& refs,
                         const SideOut& side, PosList** lists, DevicePosList** mirrors) {
  std::shared_ptr<PosList> own;
  std::shared_ptr<PosList> grp[8];
  std::vector<std::shared_ptr<PosList>> more;  // (more than 8 PosList groups: rare)
  int k = 0;
  for (const auto& c : side.cols) {
    std::shared_ptr<PosList>* slot;
    if (c.group < 0) {
      slot = &own;
    } else if (c.group < 8) {
      slot = &grp[c.group];
    } else {
      if (more.size() <= static_cast<size_t>(c.group)) more.resize(c.group + 1);
      slot = &more[c.group];
    }
    if (!*slot) {
      const DeviceBuffer* b = c.group < 0 ? side.rows : side.deref[c.group].get();
      *slot = pos_list_from_device(arena, std::shared_ptr<DeviceBuffer>(refs, const_cast<DeviceBuffer*>(b)), 0, 0,
                                   &mirrors[k]);
      lists[k++] = slot->get();
    }
    out.push_back(arena_reference_column(arena, std::shared_ptr<const Table>(refs, c.table), c.column, *slot));
  }
}

// Prepared plans (hy_scan_join_plan_*) of JoinHash executions over data tables, kept for re-executions of the same
// shape - a prepared statement executed again, or a plan re-run by the scheduler - so that the side and predicate
// descriptors are validated and staged to HBM once per shape (SF100's fused TableScan -> JoinHash: 9,155 + 1,500 chunk
// and 6,000 predicate descriptors) instead of once per execution. A plan matches an execution whose descriptors are
// byte-identical (device pointers of every column chunk included: the staged copies are then exactly what the call
// would stage) under the same HY_* knobs. A plan is used by one execution at a time (taken out of the cache, put back
// after the execution's stream synchronised); each execution rebinds it to its own TableScan output buffers.
// HY_OP_PLAN_CACHE = plans kept (default 0: off; opt-in). Join inputs with PosLists change per execution and do not use
// the cache. Off by default because of an unexplained failure under concurrent operators: with 2 plans kept,
// tests/test_operator_surface_gpu.py::test_concurrent_operators (4 threads, a new plan shape per execution, so every
// execution creates a plan - hipMalloc of its workspace - and evicts one - hipFree) aborted in 1 of 6 runs and returned
// a wrong TableScan PosList in one full-suite run; with the cache off it passed 12 of 12 runs (round 6).
struct CachedJoinPlan {
  std::vector<hy_join_chunk> bchunks, pchunks;
  hy_join_side bside{}, pside{};
  std::vector<hy_scan_chunk> filter;
  hy_join_filter pf{};
  ScanConstant constant;
  bool filtered = false;
  hy_join_params prm{};
  std::string knobs;
  hy_join_plan_t plan = nullptr;
  ~CachedJoinPlan() {
    if (plan) (void)hy_scan_join_plan_destroy(plan);
  }
};

std::string join_knobs() {  // the HY_* environment a plan was created under (its knobs snapshot)
  std::string k;
  for (char** e = ::environ; e && *e; ++e)
    if (std::strncmp(*e, "HY_", 3) == 0) k.append(*e).push_back('\n');
  return k;
}

bool same_side(const hy_join_side& a, const std::vector<hy_join_chunk>& ac, const hy_join_side& b) {
  return a.n_chunks == b.n_chunks && a.value_type == b.value_type && a.n_referenced == b.n_referenced &&
         a.fuse_dereference == b.fuse_dereference && a.referenced_chunk_base == b.referenced_chunk_base &&
         (b.n_chunks == 0 || std::memcmp(ac.data(), b.chunks, sizeof(hy_join_chunk) * b.n_chunks) == 0);
}

class JoinPlanCache {
 public:
  static JoinPlanCache& get() {
    static JoinPlanCache* c = new JoinPlanCache();  // (never destroyed: no HIP call after the runtime's teardown)
    return *c;
  }
  static std::atomic<size_t>& capacity_ref() {
    static std::atomic<size_t> v{[] {
      const char* e = std::getenv("HY_OP_PLAN_CACHE");
      return e ? static_cast<size_t>(std::max(0L, std::strtol(e, nullptr, 10))) : size_t{0};
    }()};
    return v;
  }
  static size_t capacity() { return capacity_ref().load(std::memory_order_relaxed); }
  // the plan for this execution: a cached one of the same shape, or a new one (nullptr when the cache is off)
  std::unique_ptr<CachedJoinPlan> take(const hy_join_side& b, const hy_join_side& p, const hy_join_filter* pf,
                                       const ScanConstant* constant, const hy_join_params& prm) {
    if (capacity() == 0) return nullptr;
    const std::string knobs = join_knobs();
    {
      std::lock_guard<std::mutex> lock(_m);
      for (auto it = _idle.begin(); it != _idle.end(); ++it) {
        const CachedJoinPlan& e = **it;
        if (e.knobs != knobs || std::memcmp(&e.prm, &prm, sizeof(prm)) != 0 || e.filtered != (pf != nullptr) ||
            !same_side(e.bside, e.bchunks, b) || !same_side(e.pside, e.pchunks, p))
          continue;
        if (pf && (e.pf.value_type != pf->value_type || e.pf.n_chunks != pf->n_chunks ||
                   std::memcmp(e.constant.bytes, constant->bytes, sizeof(e.constant.bytes)) != 0 ||
                   (pf->n_chunks && std::memcmp(e.filter.data(), pf->chunks, sizeof(hy_scan_chunk) * pf->n_chunks))))
          continue;
        auto found = std::move(*it);
        _idle.erase(it);
        ++_hits;
        return found;
      }
      ++_misses;
    }
    auto e = std::make_unique<CachedJoinPlan>();
    e->bchunks.assign(b.chunks, b.chunks + b.n_chunks);
    e->pchunks.assign(p.chunks, p.chunks + p.n_chunks);
    e->bside = b;
    e->bside.chunks = e->bchunks.data();
    e->pside = p;
    e->pside.chunks = e->pchunks.data();
    e->prm = prm;
    e->knobs = knobs;
    e->filtered = pf != nullptr;
    if (pf) {
      e->filter.assign(pf->chunks, pf->chunks + pf->n_chunks);
      e->constant = *constant;
      e->pf = *pf;
      e->pf.chunks = e->filter.data();
      e->pf.constant = e->constant.bytes;
    }
    hy_check(hy_scan_join_plan_create(&e->bside, nullptr, &e->pside, pf ? &e->pf : nullptr, &e->prm, &e->plan),
             "hy_scan_join_plan_create");
    return e;
  }
  // back into the cache once the execution's stream has synchronised (the oldest plan beyond the capacity is freed)
  void put(std::unique_ptr<CachedJoinPlan> e) {
    std::unique_ptr<CachedJoinPlan> evicted;
    {
      std::lock_guard<std::mutex> lock(_m);
      _idle.push_back(std::move(e));
      if (_idle.size() > capacity()) {
        evicted = std::move(_idle.front());
        _idle.erase(_idle.begin());
      }
    }
  }
  std::pair<uint64_t, uint64_t> stats() {
    std::lock_guard<std::mutex> lock(_m);
    return {_hits, _misses};
  }
  void clear() {
    std::vector<std::unique_ptr<CachedJoinPlan>> gone;
    std::lock_guard<std::mutex> lock(_m);
    gone.swap(_idle);
  }

 private:
  std::mutex _m;
  std::vector<std::unique_ptr<CachedJoinPlan>> _idle;
  uint64_t _hits = 0, _misses = 0;
};

bool scan_rowids_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("HY_OP_SCAN_ROWIDS");
    return e && std::strtol(e, nullptr, 10) != 0;
  }();
  return v;
}

bool data_side(const hy_join_side& s) {
  if (s.n_referenced) return false;
  for (uint32_t i = 0; i < s.n_chunks; ++i)
    if (s.chunks[i].pos_list) return false;
  return true;
}

}  // namespace

std::pair<uint64_t, uint64_t> join_plan_cache_stats() { return JoinPlanCache::get().stats(); }
void join_plan_cache_clear() { JoinPlanCache::get().clear(); }
void join_plan_cache_set_capacity(size_t plans) {
  JoinPlanCache::capacity_ref().store(plans);
  if (plans == 0) JoinPlanCache::get().clear();
}

std::shared_ptr<const Table> JoinHash::_on_execute() {
  const auto left_in = input_table_left();
  const auto right_in = input_table_right();
  const bool string_keys =
      join_hashed_type(left_in->column_data_type(_column_ids.first), right_in->column_data_type(_column_ids.second)) ==
      DataType::String;
  // A deferred TableScan input (DataScan) whose predicate the join's first radix pass can evaluate: its output's row
  // count comes from a count-only scan (the swap rule below needs it), and if it becomes the probe side the scan runs
  // fused into the join (hy_scan_join_hash) and its output is built from the join's by-product.
  const bool fuse_modes = _mode == JoinMode::Inner || _mode == JoinMode::Outer;
  auto fusable_scan = [&](const std::shared_ptr<const Table>& t) -> std::shared_ptr<DataScan> {
    if (!scan_fusion_enabled() || string_keys || !fuse_modes) return nullptr;
    auto scan = std::dynamic_pointer_cast<DataScan>(t->pending());
    return scan && scan->fusable() ? scan : nullptr;
  };
  const auto left_scan = fusable_scan(left_in), right_scan = fusable_scan(right_in);
  const uint64_t left_rows = left_scan ? left_scan->count_matches() : left_in->row_count();
  const uint64_t right_rows = right_scan ? right_scan->count_matches() : right_in->row_count();
  // reference join_hash.cpp:55-76
  bool inputs_swapped = (_mode == JoinMode::Left || _mode == JoinMode::Anti || _mode == JoinMode::Semi);
  if (!inputs_swapped && left_rows > right_rows) inputs_swapped = true;
  const auto build_table = inputs_swapped ? right_in : left_in;
  const auto probe_table = inputs_swapped ? left_in : right_in;
  const uint64_t build_rows = inputs_swapped ? right_rows : left_rows;
  const uint64_t probe_rows = inputs_swapped ? left_rows : right_rows;
  const ColumnID build_col = inputs_swapped ? _column_ids.second : _column_ids.first;
  const ColumnID probe_col = inputs_swapped ? _column_ids.first : _column_ids.second;
  const DataType build_type = build_table->column_data_type(build_col);
  const DataType probe_type = probe_table->column_data_type(probe_col);
  const DataType hashed = join_hashed_type(build_type, probe_type);
  // the probe side's scan runs fused when this join takes it over (a build-side scan is produced when it is read)
  std::shared_ptr<DataScan> fused_scan = inputs_swapped ? left_scan : right_scan;
  if (fused_scan && std::const_pointer_cast<Table>(probe_table)->take_pending() != fused_scan) fused_scan = nullptr;
  // (if the join fails before the scan's output is built, the scan goes back to being produced on access)
  struct Untake {
    std::shared_ptr<Table> table;
    std::shared_ptr<DataScan> scan;
    ~Untake() {
      if (scan) table->set_pending(scan);
    }
  } untake{fused_scan ? std::const_pointer_cast<Table>(probe_table) : nullptr, fused_scan};

  const bool semi_anti = _mode == JoinMode::Semi || _mode == JoinMode::Anti;
  TableColumnDefinitions defs;
  if (inputs_swapped) {
    defs = probe_table->column_definitions();
    if (!semi_anti)
      for (const auto& d : build_table->column_definitions()) defs.push_back(d);
  } else {
    defs = build_table->column_definitions();
    for (const auto& d : probe_table->column_definitions()) defs.push_back(d);
  }
  auto output = std::make_shared<Table>(defs, TableType::References);
  require_device();
  hy_stream_t s = operator_stream();
  _performance_data.rows_in = build_rows + probe_rows;
  PhaseTrace tr{"JoinHash"};

  StringKeys strings;
  JoinSideInput bside = describe_side(build_table, build_col, string_keys ? &strings : nullptr);
  // fused: the probe side is the scan's data table, filtered inside the join
  const std::shared_ptr<const Table> probe_data = fused_scan ? fused_scan->in_table : probe_table;
  JoinSideInput pside = describe_side(probe_data, probe_col, string_keys ? &strings : nullptr);
  const int32_t btype = string_keys ? HY_TYPE_INT32 : hy_type_of(build_type);
  const int32_t ptype = string_keys ? HY_TYPE_INT32 : hy_type_of(probe_type);
  hy_join_side b{bside.chunks.data(), static_cast<uint32_t>(bside.chunks.size()), btype,
                 bside.referenced.data(), static_cast<uint32_t>(bside.referenced.size()), bside.fuse};
  hy_join_side p{pside.chunks.data(), static_cast<uint32_t>(pside.chunks.size()), ptype,
                 pside.referenced.data(), static_cast<uint32_t>(pside.referenced.size()), pside.fuse};
  hy_join_params prm{};
  prm.mode = join_mode(_mode);
  prm.hashed_type = string_keys ? HY_TYPE_INT32 : hy_type_of(hashed);
  if (string_keys) prm.key_hash = strings.upload_hashes();
  // the constructor's radix_bits is ignored and recomputed from the build side (join_hash.cpp:640-668)
  // sizeof(LeftType) of the build column's type; a std::string is 32 bytes in libstdc++
  const uint32_t build_size = build_type == DataType::String ? 32u : static_cast<uint32_t>(data_type_size(build_type));
  prm.radix_bits = hy_join_radix_bits(build_rows, build_size);
  prm.seed = 17;
  _used_radix_bits = prm.radix_bits;

  tr.mark("describe sides");
  // the fused scan's filter and its by-product (the scan's matches, chunk by chunk); the scan's output chunks - their
  // sizes known from the count - are built by a job while the join runs, over RowIDs expanded after it
  std::unique_ptr<DeviceBuffer> scan_offsets, scan_begin;
  std::shared_ptr<DeviceBuffer> scan_rows;
  std::vector<std::shared_ptr<Chunk>> scan_chunks;
  JobGroup scan_builder;
  hy_join_filter pf{};
  if (fused_scan) {
    scan_rows = std::make_shared<DeviceBuffer>(std::max<uint64_t>(probe_rows, 1) * sizeof(RowID));
    scan_builder.schedule([&] { scan_chunks = fused_scan->chunks_for(scan_rows); });
    scan_offsets = std::make_unique<DeviceBuffer>(std::max<uint64_t>(fused_scan->total, 1) * 4, s);
    scan_begin = std::make_unique<DeviceBuffer>((fused_scan->descs.size() + 1) * 8, s);
    // HY_OP_SCAN_ROWIDS=1: the scan's PosLists come straight from the join's ranking pass (out_row_ids) instead of an
    // expansion of its offsets after the join (opt-in: see DESIGN.md, round 6 second session)
    pf = hy_join_filter{fused_scan->descs.data(), hy_type_of(fused_scan->col_type), fused_scan->constant.bytes,
                        scan_offsets->as<uint32_t>(), scan_begin->as<uint64_t>(),
                        static_cast<uint32_t>(fused_scan->descs.size()),
                        scan_rowids_enabled() ? scan_rows->as<hy_row_id>() : nullptr};
  }
  // a prepared plan of this shape (data-table sides), rebound to this execution's scan output buffers; else one call
  std::unique_ptr<CachedJoinPlan> cached;
  if (!string_keys && data_side(b) && data_side(p)) {
    cached = JoinPlanCache::get().take(b, p, fused_scan ? &pf : nullptr, fused_scan ? &fused_scan->constant : nullptr,
                                       prm);
    if (cached) hy_check(hy_scan_join_plan_rebind(cached->plan, nullptr, fused_scan ? &pf : nullptr), "rebind");
  }
  size_t ws_bytes = 0;
  if (cached)
    ws_bytes = 0;  // (the plan's own workspace)
  else if (fused_scan)
    hy_check(hy_scan_join_hash_workspace_size(&b, nullptr, &p, &pf, &prm, &ws_bytes),
             "hy_scan_join_hash_workspace_size");
  else
    hy_check(hy_join_hash_workspace_size(&b, &p, &prm, &ws_bytes), "hy_join_hash_workspace_size");
  DeviceBuffer ws(ws_bytes, s);
  tr.mark("plan");
  const uint32_t n_parts = 1u << prm.radix_bits;
  DeviceBuffer part_begin(8 * n_parts, s), part_count(4 * n_parts, s);
  uint64_t capacity = std::max<uint64_t>(probe_rows + build_rows, 16);
  auto out_b = std::make_shared<DeviceBuffer>(capacity * sizeof(RowID));
  auto out_p = std::make_shared<DeviceBuffer>(capacity * sizeof(RowID));
  tr.mark("buffers");

  // One output chunk per non-empty partition (join_hash.cpp:829-855), in partition order. The chunks of all
  // partitions are built while the device runs the join - their columns and PosLists depend only on the inputs -
  // and their PosLists' views are set from the partition ranges afterwards; empty partitions' chunks are dropped.
  // Chunks, columns, PosLists and mirrors come from output arenas (device.hpp), and every pointer a builder hands
  // out aliases its own OutRefs: several threads build without contending on shared reference counts (65,536
  // chunks at SF100).
  OutRefs base_refs;
  std::shared_ptr<Table> dummy, pdummy;
  const bool with_build = !(semi_anti && inputs_swapped);
  SideOut bo = with_build ? describe_output(build_table, bside, out_b, base_refs, dummy) : SideOut{};
  SideOut po = describe_output(probe_data, pside, out_p, base_refs, pdummy);
  const int n_lists = bo.n_lists + po.n_lists;
  std::vector<std::shared_ptr<Chunk>> chunks(n_parts);
  std::vector<PosList*> lists(static_cast<size_t>(n_parts) * n_lists);
  std::vector<DevicePosList*> mirrors(lists.size());
  static const size_t max_workers = [] {  // HY_OP_THREADS caps the builder jobs (A/B)
    const char* e = std::getenv("HY_OP_THREADS");
    return e ? std::max(1L, std::strtol(e, nullptr, 10)) : 16L;
  }();
  std::atomic<size_t> next{0};
  const auto spawn = std::chrono::steady_clock::now();
  std::atomic<int64_t> last_done_us{0};  // (HY_OP_TRACE: when the builders finished)
  auto build = [&]() {
    struct Done {
      std::atomic<int64_t>& last;
      std::chrono::steady_clock::time_point t0;
      ~Done() {
        const int64_t us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                               .count();
        for (int64_t cur = last.load(); cur < us && !last.compare_exchange_weak(cur, us);) {
        }
      }
    } done{last_done_us, spawn};
    OutputArena arena;
    auto refs = std::make_shared<OutRefs>(base_refs);
    constexpr size_t BATCH = 256;
    for (size_t i0; (i0 = next.fetch_add(BATCH)) < n_parts;) {
      for (size_t i = i0; i < std::min<size_t>(n_parts, i0 + BATCH); ++i) {
        ChunkColumns cols;
        cols.reserve(output->column_count());
        PosList** l = &lists[i * n_lists];
        DevicePosList** m = &mirrors[i * n_lists];
        if (inputs_swapped) {
          write_chunk_columns(cols, arena, refs, po, l, m);
          if (with_build) write_chunk_columns(cols, arena, refs, bo, l + po.n_lists, m + po.n_lists);
        } else {
          write_chunk_columns(cols, arena, refs, bo, l, m);
          write_chunk_columns(cols, arena, refs, po, l + bo.n_lists, m + bo.n_lists);
        }
        chunks[i] = arena_chunk(arena, std::move(cols));
      }
    }
  };
  // once the partition ranges are known and every chunk is built, jobs set the PosLists' views
  std::vector<uint64_t> h_begin(n_parts);
  std::vector<uint32_t> h_count(n_parts);
  std::atomic<size_t> next_view{0};
  auto set_views = [&]() {
    constexpr size_t BATCH = 2048;
    for (size_t i0; (i0 = next_view.fetch_add(BATCH)) < n_parts;) {
      for (size_t part = i0; part < std::min<size_t>(n_parts, i0 + BATCH); ++part) {
        const uint32_t n = h_count[part];
        if (!n) continue;
        for (int k = 0; k < n_lists; ++k) {
          const size_t i = part * n_lists + k;
          lists[i]->set_lazy_size(n);
          mirrors[i]->size = n;
          mirrors[i]->view_offset = h_begin[part];
        }
      }
    }
  };
  // The builders are jobs of the host's scheduler (scheduler.hpp; join_hash.cpp:139-182 submits JobTasks and waits in
  // CurrentScheduler::wait_for_tasks), scheduled before the join's kernels so that they run while the device joins;
  // without a registered scheduler each job has a thread of its own. The group is declared after everything the jobs
  // read, so its destructor waits for them also when the join throws.
  JobGroup builders;
  static const size_t parts_per_job = [] {  // at least this many partitions per job (HY_OP_PARTS_PER_JOB: tests)
    const char* e = std::getenv("HY_OP_PARTS_PER_JOB");
    return e ? std::max(1L, std::strtol(e, nullptr, 10)) : 2048L;
  }();
  const unsigned workers = static_cast<unsigned>(std::max<size_t>(
      1, std::min<size_t>({max_workers, builders.concurrency(host_cpu_share()), n_parts / parts_per_job})));
  for (unsigned t = 0; t < workers; ++t) builders.schedule(build);
  tr.mark("output described, builders scheduled");

  hy_join_result res{};
  for (int attempt = 0; attempt < 2; ++attempt) {
    const hy_status st =
        cached ? hy_scan_join_plan_execute(cached->plan, out_b->as<hy_row_id>(), out_p->as<hy_row_id>(), capacity,
                                           part_begin.as<uint64_t>(), part_count.as<uint32_t>(), &res, s)
        : fused_scan
            ? hy_scan_join_hash(&b, nullptr, &p, &pf, &prm, out_b->as<hy_row_id>(), out_p->as<hy_row_id>(), capacity,
                                part_begin.as<uint64_t>(), part_count.as<uint32_t>(), &res, ws.get(), ws_bytes, s)
            : hy_join_hash(&b, &p, &prm, out_b->as<hy_row_id>(), out_p->as<hy_row_id>(), capacity,
                           part_begin.as<uint64_t>(), part_count.as<uint32_t>(), &res, ws.get(), ws_bytes, s);
    if (st == HY_ERR_CAPACITY && attempt == 0) {
      capacity = std::max<uint64_t>(res.capacity_required, 16);
      DeviceBuffer nb(capacity * sizeof(RowID)), np(capacity * sizeof(RowID));
      out_b->swap(nb);  // (the PosLists built so far view these objects, not their allocations)
      out_p->swap(np);
      continue;
    }
    hy_check(st, fused_scan ? "hy_scan_join_hash" : "hy_join_hash");
    break;
  }
  tr.mark("join launched");
  hy_check(hy_memcpy_dtoh(h_begin.data(), part_begin.get(), 8 * n_parts, s), "dtoh");
  hy_check(hy_memcpy_dtoh(h_count.data(), part_count.get(), 4 * n_parts, s), "dtoh");
  std::vector<uint64_t> h_scan_begin(fused_scan ? fused_scan->descs.size() + 1 : 0);
  if (fused_scan)
    hy_check(hy_memcpy_dtoh(h_scan_begin.data(), scan_begin->get(), 8 * h_scan_begin.size(), s), "dtoh");
  hy_check(hy_stream_synchronize(s), "sync");
  if (cached) JoinPlanCache::get().put(std::move(cached));  // (its workspace is idle: the stream synchronised)
  tr.mark("join kernels + partition counts synchronised");
  if (fused_scan) {  // the scan's output: RowIDs written by the join (out_row_ids), or expanded from its offsets here
    uint64_t at = 0;
    for (size_t k = 0; k < fused_scan->counts.size(); ++k) {
      Assert(h_scan_begin[k] == at, "fused TableScan: the join's scan output disagrees with the scan's count");
      at += fused_scan->counts[k];
    }
    if (!pf.out_row_ids) {
      hy_check(hy_expand_chunk_row_ids(scan_offsets->as<uint32_t>(), scan_begin->as<uint64_t>(), nullptr,
                                       static_cast<uint32_t>(fused_scan->descs.size()), scan_rows->as<hy_row_id>(), s),
               "hy_expand_chunk_row_ids");
      hy_check(hy_stream_synchronize(s), "sync");  // (consumers on other threads read scan_rows once published)
    }
    scan_builder.wait();
    // consumers blocked in resolve() on other threads read scan_rows from their own streams as soon as the chunks are
    // published: every write of it was ordered before the stream synchronisation above
    std::const_pointer_cast<Table>(probe_table)->fulfil(std::move(scan_chunks));
    untake.scan = nullptr;
    tr.mark("fused TableScan output");
  }

  uint64_t used = 0;  // the output range the partitions occupy
  for (uint32_t part = 0; part < n_parts; ++part)
    if (h_count[part]) used = std::max<uint64_t>(used, h_begin[part] + h_count[part]);
  {  // algorithmic bytes: both join columns (+ 8 B per row read through a PosList, + the fused scan's predicate ids
     // of every scanned row), 16 B per output pair (+ the fused scan's 8 B RowIDs)
    const uint64_t kb = build_type == DataType::String ? 4 : data_type_size(build_type);
    const uint64_t kp = probe_type == DataType::String ? 4 : data_type_size(probe_type);
    uint64_t rd = build_rows * (kb + (build_table->type() == TableType::References ? 8 : 0));
    if (fused_scan) {
      uint64_t vid = 0;
      for (const auto& d : fused_scan->descs) vid += uint64_t(d.column.size) * d.column.vid_width;
      rd += fused_scan->total * kp + vid;
    } else {
      rd += probe_rows * (kp + (probe_table->type() == TableType::References ? 8 : 0));
    }
    _performance_data.bytes_read = rd;
    _performance_data.bytes_written = res.total_pairs * 2 * sizeof(RowID) + (fused_scan ? probe_rows * sizeof(RowID) : 0);
  }
  if (with_build) dereference_groups(bo, *out_b, used);
  dereference_groups(po, *out_p, used);
  builders.wait();  // (rethrows a builder's exception)
  {
    JobGroup viewers;
    for (unsigned t = 0; t < workers; ++t) viewers.schedule(set_views);
    viewers.wait();
  }
  if (tr.on) tr.note("builders done after start (" + std::to_string(workers) + " jobs)", last_done_us.load() / 1000.0);
  tr.mark("output chunks built, views set");
  std::vector<std::shared_ptr<Chunk>> nonempty;  // join_hash.cpp:835-837: no chunk for an empty partition
  nonempty.reserve(n_parts);
  for (uint32_t part = 0; part < n_parts; ++part)
    if (h_count[part]) nonempty.push_back(std::move(chunks[part]));
  output->append_chunks(std::move(nonempty));
  tr.mark("output chunks");
  {  // the workspace goes back to this thread's block cache (traced: a release that frees device memory is slow)
    DeviceBuffer none;
    ws.swap(none);
  }
  tr.mark("workspace released");
  return output;
}

}  // namespace hyrise
