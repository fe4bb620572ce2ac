// Aggregate::_on_execute on the device (reference src/lib/operators/aggregate.cpp:203-820).
//
// The host describes the input columns to the C-ABI (hy_aggregate), which folds every row into per-group records on
// the GPU in one pass. The host then reproduces the reference's observable output from those records:
//   * group ids: per group-by column, ids 1, 2, ... in order of first appearance, 0 for NULL (aggregate.cpp:341-392);
//     the first appearance of a value is the smallest first-row over the groups holding it;
//   * row order: the iteration order of the reference's std::unordered_map<AggregateKey, ...>, obtained by inserting
//     the composite keys into the same container type, with the same hash, in first-row order (its insertion order);
//   * group values: read with operator[] at each group's last row (_write_groupby_output, :722-733);
//   * output types, names and nullability of aggregate_traits.hpp:15-74 and write_aggregate_output (:756-820).
//
// Strings never reach the device as bytes: a string column is sent as int32 codes (ranks in the sorted set of its
// distinct strings), so grouping, COUNT(DISTINCT) and MIN/MAX on codes equal those on the strings. Group-by columns
// whose dictionaries hold few distinct values are sent as codes too, which selects the dense (LDS) device path.
#include <algorithm>
#include <array>
#include <map>
#include <memory>
#include <numeric>
#include <unordered_map>

#include "operators.hpp"

namespace hyrise {

namespace {

constexpr uint32_t DENSE_MAX_GROUPS = 64;  // hyk::AGG_DENSE_MAX

// boost::hash_range over 64-bit key entries (hash_combine as in Boost < 1.81), used by the reference's
// std::hash<std::array<AggregateKeyEntry, 2>> and std::hash<pmr_vector<AggregateKeyEntry>> (aggregate.hpp:154-169).
template <typename It>
size_t hash_range(It b, It e) {
  size_t seed = 0;
  for (; b != e; ++b) seed ^= static_cast<size_t>(*b) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
  return seed;
}
struct ArrayKeyHash {
  size_t operator()(const std::array<uint64_t, 2>& k) const { return hash_range(k.begin(), k.end()); }
};
struct VectorKeyHash {
  size_t operator()(const std::vector<uint64_t>& k) const { return hash_range(k.begin(), k.end()); }
};

// Iteration order of std::unordered_map<K, ...> after inserting keys[order[0]], keys[order[1]], ...
template <typename K, typename H>
std::vector<size_t> unordered_map_iteration(const std::vector<K>& keys, const std::vector<size_t>& order) {
  std::unordered_map<K, size_t, H> m;
  for (const auto i : order) m.emplace(keys[i], i);
  std::vector<size_t> out;
  out.reserve(m.size());
  for (const auto& kv : m) out.push_back(kv.second);
  return out;
}

// One column as the device reads it.
struct DevColumn {
  ColumnID column_id = 0;
  bool coded = false;                  // values are int32 codes
  DataType type = DataType::Int;       // logical type of the column
  hy_agg_column desc{};
  std::vector<hy_column_chunk> chunks;
  std::vector<std::shared_ptr<DeviceBuffer>> keep;
  std::vector<std::string> string_codes;  // string columns: code -> string
};

// The column chunks the device reads for a column of the input: the input's own chunks (data table) or the
// referenced table's chunks (reference table; all chunks must reference one table).
struct SourceChunks {
  std::vector<std::shared_ptr<const BaseColumn>> columns;
  int32_t pos_group = -1;
};

template <typename T>
void collect_values(const BaseColumn& col, std::vector<T>& out) {
  if (const auto* d = dynamic_cast<const DictionaryColumn<T>*>(&col)) {
    out.insert(out.end(), d->dictionary().begin(), d->dictionary().end());
    return;
  }
  const auto& v = static_cast<const ValueColumn<T>&>(col);
  for (size_t i = 0; i < v.size(); ++i)
    if (!v.is_null(i)) out.push_back(v.values()[i]);
}

template <typename T>
int32_t code_of(const std::vector<T>& sorted, const T& v) {
  return static_cast<int32_t>(std::lower_bound(sorted.begin(), sorted.end(), v) - sorted.begin());
}

// Builds the int32 code representation of a column over the given source chunks, codes = ranks in sorted distinct.
template <typename T>
void build_codes(DevColumn& dc, const std::vector<std::shared_ptr<const BaseColumn>>& src, hy_stream_t s) {
  std::vector<T> all;
  for (const auto& c : src) collect_values<T>(*c, all);
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end(), [](const T& a, const T& b) { return a == b; }), all.end());
  dc.desc.domain = static_cast<uint32_t>(all.size());
  if constexpr (std::is_same_v<T, std::string>) dc.string_codes = all;
  for (const auto& c : src) {
    hy_column_chunk ch{};
    ch.size = static_cast<uint32_t>(c->size());
    if (const auto* d = dynamic_cast<const DictionaryColumn<T>*>(c.get())) {
      std::vector<int32_t> codes(d->dictionary().size());
      for (size_t i = 0; i < codes.size(); ++i) codes[i] = code_of(all, d->dictionary()[i]);
      auto buf = std::make_shared<DeviceBuffer>(std::max<size_t>(16, 4 * codes.size()));
      hy_check(hy_memcpy_htod(buf->get(), codes.data(), 4 * codes.size(), s), "htod");
      const auto dev = device_column(*c);  // attribute vector
      ch = dev->desc;
      ch.dictionary = buf->get();
      dc.keep.push_back(buf);
    } else {
      const auto& v = static_cast<const ValueColumn<T>&>(*c);
      std::vector<int32_t> codes(v.size(), 0);
      for (size_t i = 0; i < v.size(); ++i)
        if (!v.is_null(i)) codes[i] = code_of(all, v.values()[i]);
      auto buf = std::make_shared<DeviceBuffer>(std::max<size_t>(16, 4 * codes.size()));
      hy_check(hy_memcpy_htod(buf->get(), codes.data(), 4 * codes.size(), s), "htod");
      dc.keep.push_back(buf);
      ch.kind = HY_COL_VALUE;
      ch.data = buf->get();
      if (v.is_nullable()) {
        auto nb = std::make_shared<DeviceBuffer>(std::max<size_t>(16, v.size()));
        hy_check(hy_memcpy_htod(nb->get(), v.null_values().data(), v.size(), s), "htod");
        dc.keep.push_back(nb);
        ch.nulls = nb->template as<uint8_t>();
      }
    }
    dc.chunks.push_back(ch);
  }
  hy_check(hy_stream_synchronize(s), "sync");
}

// Distinct values of a numeric column over its dictionaries, if every source chunk is dictionary-encoded and there
// are at most `limit` of them (dense group-by candidates).
template <typename T>
bool small_dictionary_domain(const std::vector<std::shared_ptr<const BaseColumn>>& src, size_t limit) {
  std::vector<T> all;
  for (const auto& c : src) {
    const auto* d = dynamic_cast<const DictionaryColumn<T>*>(c.get());
    if (!d) return false;
    all.insert(all.end(), d->dictionary().begin(), d->dictionary().end());
    if (all.size() > 64 * limit) {
      std::sort(all.begin(), all.end());
      all.erase(std::unique(all.begin(), all.end()), all.end());
      if (all.size() > limit) return false;
    }
  }
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end(), [](const T& a, const T& b) { return a == b; }), all.end());
  return all.size() <= limit;
}

double ordered_to_double(uint64_t ordered, DataType t) {
  const uint64_t b = hy_agg_decode_ordered(ordered, hy_type_of(t));
  if (t == DataType::Float) {
    float f;
    const uint32_t u = static_cast<uint32_t>(b);
    std::memcpy(&f, &u, 4);
    return f;
  }
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}

AllTypeVariant ordered_to_variant(uint64_t ordered, const DevColumn& dc) {
  if (dc.type == DataType::String) return dc.string_codes.at(static_cast<uint32_t>(ordered ^ 0x80000000u));
  const uint64_t b = hy_agg_decode_ordered(ordered, hy_type_of(dc.type));
  switch (dc.type) {
    case DataType::Int:
      return static_cast<int32_t>(static_cast<uint32_t>(b));
    case DataType::Long:
      return static_cast<int64_t>(b);
    case DataType::Float:
      return static_cast<float>(ordered_to_double(ordered, dc.type));
    default:
      return ordered_to_double(ordered, dc.type);
  }
}

}  // namespace

std::shared_ptr<const Table> Aggregate::_on_execute() {
  const auto in = input_table_left();
  // reference aggregate.cpp:268-281
  for (const auto& a : _aggregates) {
    if (!a.column) {
      if (a.function != AggregateFunction::Count) Fail("Aggregate: Asterisk is only valid with COUNT");
    } else if (in->column_data_type(*a.column) == DataType::String &&
               (a.function == AggregateFunction::Sum || a.function == AggregateFunction::Avg)) {
      Fail("Aggregate: Cannot calculate SUM or AVG on string column");
    }
  }
  require_device();
  hy_stream_t s = operator_stream();
  const bool is_ref = in->type() == TableType::References;
  const uint32_t n_chunks = in->chunk_count();
  _performance_data.rows_in = in->row_count();

  // ---- input shape: chunk sizes, PosList groups (columns sharing the same PosLists, join_hash.cpp:533-562 style)
  std::vector<uint32_t> chunk_sizes(n_chunks);
  for (ChunkID c = 0; c < n_chunks; ++c) chunk_sizes[c] = static_cast<uint32_t>(in->get_chunk(c)->size());
  std::vector<std::vector<const PosList*>> pos_groups;
  std::vector<std::vector<std::shared_ptr<const PosList>>> pos_group_lists;
  auto source_of = [&](ColumnID col) {
    SourceChunks sc;
    if (!is_ref) {
      for (ChunkID c = 0; c < n_chunks; ++c) sc.columns.push_back(in->get_chunk(c)->get_column(col));
      return sc;
    }
    std::vector<const PosList*> key;
    std::vector<std::shared_ptr<const PosList>> lists;
    std::shared_ptr<const Table> referenced;
    ColumnID rcol = 0;
    for (ChunkID c = 0; c < n_chunks; ++c) {
      const auto rc = std::dynamic_pointer_cast<const ReferenceColumn>(in->get_chunk(c)->get_column(col));
      Assert(rc != nullptr, "All columns should be of type ReferenceColumn.");
      if (!referenced) {
        referenced = rc->referenced_table();
        rcol = rc->referenced_column_id();
      }
      Assert(rc->referenced_table() == referenced && rc->referenced_column_id() == rcol,
             "hyrise-amd: an aggregate column referencing several tables is not supported");
      key.push_back(rc->pos_list().get());
      lists.push_back(rc->pos_list());
    }
    auto it = std::find(pos_groups.begin(), pos_groups.end(), key);
    if (it == pos_groups.end()) {
      pos_groups.push_back(key);
      pos_group_lists.push_back(lists);
      it = pos_groups.end() - 1;
    }
    sc.pos_group = static_cast<int32_t>(it - pos_groups.begin());
    if (referenced)
      for (ChunkID r = 0; r < referenced->chunk_count(); ++r)
        sc.columns.push_back(referenced->get_chunk(r)->get_column(rcol));
    return sc;
  };

  // ---- device columns: group-by (codes when every group-by column has a small domain, or for strings), aggregates
  std::vector<std::unique_ptr<DevColumn>> columns;
  auto add_column = [&](ColumnID col, bool coded) -> int32_t {
    for (size_t i = 0; i < columns.size(); ++i)
      if (columns[i]->column_id == col && columns[i]->coded == coded) return static_cast<int32_t>(i);
    auto dc = std::make_unique<DevColumn>();
    dc->column_id = col;
    dc->coded = coded;
    dc->type = in->column_data_type(col);
    const auto src = source_of(col);
    dc->desc.pos_group = src.pos_group;
    if (coded) {
      resolve_data_type(dc->type, [&](auto tag) { build_codes<decltype(tag)>(*dc, src.columns, s); });
      dc->desc.value_type = HY_TYPE_INT32;
    } else {
      for (const auto& c : src.columns) dc->chunks.push_back(device_column(*c)->desc);
      dc->desc.value_type = hy_type_of(dc->type);
    }
    dc->desc.chunks = dc->chunks.data();
    dc->desc.n_chunks = static_cast<uint32_t>(dc->chunks.size());
    columns.push_back(std::move(dc));
    Assert(columns.size() <= HY_AGG_MAX_COLUMNS, "hyrise-amd: too many columns for the device Aggregate");
    return static_cast<int32_t>(columns.size() - 1);
  };

  // dense device path: every group-by column has a small code domain (its dictionaries' distinct values, or strings)
  bool dense = !_groupby_column_ids.empty();
  for (const auto& a : _aggregates) dense = dense && a.function != AggregateFunction::CountDistinct;
  for (const auto g : _groupby_column_ids) {
    if (!dense) break;
    const auto src = source_of(g);
    resolve_data_type(in->column_data_type(g), [&](auto tag) {
      using T = decltype(tag);
      if constexpr (!std::is_same_v<T, std::string>) dense = small_dictionary_domain<T>(src.columns, DENSE_MAX_GROUPS - 1);
    });
  }
  std::vector<int32_t> gb_entries;
  for (const auto g : _groupby_column_ids)
    gb_entries.push_back(add_column(g, dense || in->column_data_type(g) == DataType::String));
  if (dense) {
    uint64_t product = 1;
    for (const auto e : gb_entries) product *= uint64_t(columns[e]->desc.domain) + 1;
    if (product > DENSE_MAX_GROUPS) dense = false;
  }
  if (!dense)  // non-string group-by columns read raw values; their domains must not claim dense codes
    for (size_t j = 0; j < gb_entries.size(); ++j) {
      auto& dc = *columns[gb_entries[j]];
      if (dc.type != DataType::String && dc.coded) gb_entries[j] = add_column(dc.column_id, false);
    }
  std::vector<hy_agg_def> defs;
  for (const auto& a : _aggregates) {
    hy_agg_def d{};
    d.function = static_cast<int32_t>(a.function);  // same order as HY_AGG_*
    d.column = a.column ? add_column(*a.column, in->column_data_type(*a.column) == DataType::String) : -1;
    defs.push_back(d);
  }
  std::vector<hy_agg_column> col_descs;
  for (auto& c : columns) {
    c->desc.chunks = c->chunks.data();
    col_descs.push_back(c->desc);
    if (!dense) col_descs.back().domain = 0;  // domains only select the dense path
  }

  std::vector<const hy_row_id*> pos_ptrs;
  for (const auto& lists : pos_group_lists)
    for (const auto& pl : lists) pos_ptrs.push_back(device_pos_list(*pl)->ptr());
  hy_agg_input hin{};
  hin.n_chunks = n_chunks;
  hin.chunk_sizes = chunk_sizes.data();
  hin.pos_lists = pos_ptrs.data();
  hin.n_pos_groups = static_cast<uint32_t>(pos_group_lists.size());
  hin.columns = col_descs.data();
  hin.n_columns = static_cast<uint32_t>(col_descs.size());
  hy_agg_params prm{};
  prm.groupby = gb_entries.data();
  prm.n_groupby = static_cast<uint32_t>(gb_entries.size());
  prm.aggregates = defs.data();
  prm.n_aggregates = static_cast<uint32_t>(defs.size());
  prm.group_bound = 0;
  Assert(prm.n_groupby <= HY_AGG_MAX_GROUPBY, "hyrise-amd: too many group-by columns for the device Aggregate");
  Assert(prm.n_aggregates <= HY_AGG_MAX_AGGREGATES, "hyrise-amd: too many aggregates for the device Aggregate");
  Assert(hin.n_pos_groups <= HY_AGG_MAX_POS_GROUPS, "hyrise-amd: too many PosList groups for the device Aggregate");

  hy_agg_layout layout{};
  hy_check(hy_aggregate_layout(&hin, &prm, &layout), "hy_aggregate_layout");
  _used_dense_path = layout.dense != 0;
  size_t ws_bytes = 0;
  hy_check(hy_aggregate_workspace_size(&hin, &prm, &ws_bytes), "hy_aggregate_workspace_size");
  auto ws = std::make_unique<DeviceBuffer>(ws_bytes, s);
  uint64_t capacity = std::max<uint64_t>(1, std::min<uint64_t>(in->row_count(), layout.dense ? 64 : 1u << 16));
  uint64_t n_groups = 0;
  std::vector<uint64_t> rec;
  // retries: a larger output capacity (HY_ERR_CAPACITY) or a larger hash table (HY_ERR_GROUP_BOUND: the device
  // table is sized for params.group_bound groups, derived from the inputs when 0, and grows 4x per retry)
  bool done = false;
  for (int attempt = 0; attempt < 16 && !done; ++attempt) {
    DeviceBuffer out(capacity * layout.words * 8, s);
    const hy_status st =
        hy_aggregate(&hin, &prm, out.as<uint64_t>(), capacity, &n_groups, ws->get(), ws_bytes, s);
    if (st == HY_ERR_CAPACITY) {
      capacity = n_groups;
      continue;
    }
    if (st == HY_ERR_GROUP_BOUND) {
      prm.group_bound = n_groups;
      hy_check(hy_aggregate_workspace_size(&hin, &prm, &ws_bytes), "hy_aggregate_workspace_size");
      ws = std::make_unique<DeviceBuffer>(ws_bytes, s);
      continue;
    }
    hy_check(st, "hy_aggregate");
    rec.resize(n_groups * layout.words);
    hy_check(hy_memcpy_dtoh(rec.data(), out.get(), rec.size() * 8, s), "dtoh");
    hy_check(hy_stream_synchronize(s), "sync");
    done = true;
  }
  if (!done) Fail("hyrise-amd: hy_aggregate did not converge on an output capacity / group bound");

  // ---- reference row order
  const uint32_t W = layout.words, NG = prm.n_groupby;
  auto word = [&](size_t g, uint32_t w) { return rec[g * W + w]; };
  auto first_row = [&](size_t g) { return word(g, NG + 1); };
  std::vector<size_t> by_first(n_groups);
  std::iota(by_first.begin(), by_first.end(), size_t{0});
  std::sort(by_first.begin(), by_first.end(), [&](size_t a, size_t b) { return first_row(a) < first_row(b); });
  // per group-by column: first-appearance ids (0 = NULL)
  std::vector<std::vector<uint64_t>> ids(NG, std::vector<uint64_t>(n_groups, 0));
  for (uint32_t j = 0; j < NG; ++j) {
    std::map<uint64_t, uint64_t> first_seen;  // key word -> smallest first row
    for (size_t g = 0; g < n_groups; ++g) {
      if ((word(g, NG) >> j) & 1u) continue;
      auto it = first_seen.find(word(g, j));
      if (it == first_seen.end())
        first_seen.emplace(word(g, j), first_row(g));
      else
        it->second = std::min(it->second, first_row(g));
    }
    std::vector<std::pair<uint64_t, uint64_t>> order;  // (first row, key word)
    for (const auto& kv : first_seen) order.emplace_back(kv.second, kv.first);
    std::sort(order.begin(), order.end());
    std::unordered_map<uint64_t, uint64_t> id_of;
    for (size_t i = 0; i < order.size(); ++i) id_of[order[i].second] = i + 1;
    for (size_t g = 0; g < n_groups; ++g)
      ids[j][g] = ((word(g, NG) >> j) & 1u) ? 0 : id_of.at(word(g, j));
  }
  std::vector<size_t> out_order;
  if (NG <= 1) {
    std::vector<uint64_t> keys(n_groups, 0);
    if (NG == 1) keys = ids[0];
    out_order = unordered_map_iteration<uint64_t, std::hash<uint64_t>>(keys, by_first);
  } else if (NG == 2) {
    std::vector<std::array<uint64_t, 2>> keys(n_groups);
    for (size_t g = 0; g < n_groups; ++g) keys[g] = {ids[0][g], ids[1][g]};
    out_order = unordered_map_iteration<std::array<uint64_t, 2>, ArrayKeyHash>(keys, by_first);
  } else {
    std::vector<std::vector<uint64_t>> keys(n_groups, std::vector<uint64_t>(NG));
    for (size_t g = 0; g < n_groups; ++g)
      for (uint32_t j = 0; j < NG; ++j) keys[g][j] = ids[j][g];
    out_order = unordered_map_iteration<std::vector<uint64_t>, VectorKeyHash>(keys, by_first);
  }

  // ---- output (aggregate.cpp:543-566, 756-820)
  TableColumnDefinitions out_defs;
  ChunkColumns out_cols;
  // group rows as RowIDs of the input (last row of each group)
  std::vector<uint64_t> chunk_begin(n_chunks + 1, 0);
  for (ChunkID c = 0; c < n_chunks; ++c) chunk_begin[c + 1] = chunk_begin[c] + chunk_sizes[c];
  auto row_id_of = [&](uint64_t row) {
    const auto it = std::upper_bound(chunk_begin.begin(), chunk_begin.end(), row);
    const ChunkID c = static_cast<ChunkID>(it - chunk_begin.begin() - 1);
    return RowID{c, static_cast<ChunkOffset>(row - chunk_begin[c])};
  };
  for (const auto g : _groupby_column_ids) {
    out_defs.emplace_back(in->column_name(g), in->column_data_type(g), false);
    auto col = make_value_column(in->column_data_type(g), true);
    for (const auto gi : out_order) {
      const RowID r = row_id_of(word(gi, NG + 2));
      col->append((*in->get_chunk(r.chunk_id)->get_column(g))[r.chunk_offset]);
    }
    out_cols.push_back(col);
  }
  static const char* fn_names[] = {"MIN", "MAX", "SUM", "AVG", "COUNT", "COUNT"};
  for (size_t ai = 0; ai < _aggregates.size(); ++ai) {
    const auto& a = _aggregates[ai];
    const DataType in_type = a.column ? in->column_data_type(*a.column) : DataType::Int;
    DataType out_type = in_type;
    switch (a.function) {
      case AggregateFunction::Count:
      case AggregateFunction::CountDistinct:
        out_type = DataType::Long;
        break;
      case AggregateFunction::Avg:
        out_type = DataType::Double;
        break;
      case AggregateFunction::Sum:
        out_type = (in_type == DataType::Float || in_type == DataType::Double) ? DataType::Double : DataType::Long;
        break;
      default:
        break;
    }
    std::string name = a.function == AggregateFunction::CountDistinct ? "COUNT(DISTINCT "
                                                                       : std::string(fn_names[int(a.function)]) + "(";
    name += a.column ? in->column_name(*a.column) : "*";
    name += ")";
    const bool nullable = !(a.function == AggregateFunction::Count || a.function == AggregateFunction::CountDistinct);
    out_defs.emplace_back(name, out_type, nullable);
    auto col = make_value_column(out_type, nullable);
    const uint32_t w0 = layout.agg_word[ai];
    const DevColumn* dc = defs[ai].column >= 0 ? columns[defs[ai].column].get() : nullptr;
    auto float_sum = [&](size_t gi) {
      double v = 0;
      hy_check(hy_agg_float_sum(&rec[gi * W + w0 + 2], layout.agg_limbs[ai], layout.agg_emin[ai], word(gi, w0 + 1), &v),
               "hy_agg_float_sum");
      return v;
    };
    for (const auto gi : out_order) {
      if (!a.column) {  // COUNT(*)
        col->append(static_cast<int64_t>(word(gi, NG + 3)));
        continue;
      }
      const uint64_t count = word(gi, w0);
      switch (a.function) {
        case AggregateFunction::Count:
        case AggregateFunction::CountDistinct:
          col->append(static_cast<int64_t>(count));
          break;
        case AggregateFunction::Min:
        case AggregateFunction::Max:
          col->append(count ? ordered_to_variant(word(gi, w0 + 1), *dc) : AllTypeVariant{NullValue{}});
          break;
        case AggregateFunction::Sum:
          if (!count)
            col->append(NullValue{});
          else if (layout.agg_limbs[ai])
            col->append(float_sum(gi));
          else
            col->append(static_cast<int64_t>(word(gi, w0 + 1)));
          break;
        case AggregateFunction::Avg:
          if (!count) {
            col->append(NullValue{});
          } else {
            const double sum = layout.agg_limbs[ai] ? float_sum(gi)
                                                    : static_cast<double>(static_cast<int64_t>(word(gi, w0 + 1)));
            col->append(sum / static_cast<double>(count));
          }
          break;
      }
    }
    // aggregate.cpp:811-817: no groups and no group-by -> one row (NULL, or 0 for COUNT)
    if (n_groups == 0 && _groupby_column_ids.empty()) {
      if (a.function == AggregateFunction::Count || a.function == AggregateFunction::CountDistinct)
        col->append(int64_t{0});
      else
        col->append(NullValue{});
    }
    out_cols.push_back(col);
  }
  auto output = std::make_shared<Table>(out_defs, TableType::Data);
  output->append_chunk(out_cols);
  return output;
}

}  // namespace hyrise
