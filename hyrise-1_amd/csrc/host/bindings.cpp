// Python bindings of the host operator layer (tests, bench, smoke). Mirrors the reference's C++ test vocabulary:
// load_table, ChunkEncoder, TableWrapper, TableScan, JoinHash, Aggregate, ReferenceColumn, PosList.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "device.hpp"
#include "operators.hpp"
#include "scheduler.hpp"
#include "storage.hpp"

namespace py = pybind11;
using namespace hyrise;

namespace {

AllTypeVariant to_variant(const py::handle& o) {
  if (o.is_none()) return NullValue{};
  if (py::isinstance<py::bool_>(o)) return static_cast<int32_t>(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) {
    const auto v = o.cast<long long>();
    if (v >= INT32_MIN && v <= INT32_MAX) return static_cast<int32_t>(v);
    return static_cast<int64_t>(v);
  }
  if (py::isinstance<py::float_>(o)) return o.cast<double>();
  if (py::isinstance<py::str>(o)) return o.cast<std::string>();
  // typed wrappers from Python: (type_name, value)
  if (py::isinstance<py::tuple>(o) && py::len(o) == 2) {
    const auto t = o[py::int_(0)].cast<std::string>();
    const py::handle v = o[py::int_(1)];
    if (t == "int") return v.cast<int32_t>();
    if (t == "long") return v.cast<int64_t>();
    if (t == "float") return v.cast<float>();
    if (t == "double") return v.cast<double>();
    if (t == "string") return v.cast<std::string>();
  }
  throw std::invalid_argument("cannot convert Python object to AllTypeVariant");
}

py::object to_py(const AllTypeVariant& v) {
  switch (v.index()) {
    case 0:
      return py::none();
    case 1:
      return py::int_(std::get<int32_t>(v));
    case 2:
      return py::int_(std::get<int64_t>(v));
    case 3:
      return py::float_(static_cast<double>(std::get<float>(v)));
    case 4:
      return py::float_(std::get<double>(v));
    default:
      return py::str(std::get<std::string>(v));
  }
}

py::object parameter_to_py(const AllParameterVariant& p);

ParameterMap to_parameter_map(const py::dict& d) {
  ParameterMap m;
  for (const auto& kv : d) m.emplace(ParameterID{kv.first.cast<size_t>()}, to_variant(kv.second));
  return m;
}

py::array_t<uint32_t> pos_list_array(const PosList& pl) {
  py::array_t<uint32_t> a({static_cast<py::ssize_t>(pl.size()), static_cast<py::ssize_t>(2)});
  if (!pl.empty()) std::memcpy(a.mutable_data(), pl.data(), pl.size() * sizeof(RowID));
  return a;
}

std::shared_ptr<PosList> pos_list_from_array(py::array_t<uint32_t, py::array::c_style | py::array::forcecast> a) {
  Assert(a.ndim() == 2 && a.shape(1) == 2, "PosList array must have shape (n, 2)");
  auto pl = std::make_shared<PosList>(a.shape(0));
  if (a.shape(0)) std::memcpy(pl->data(), a.data(), a.shape(0) * sizeof(RowID));
  return pl;
}

// Builds a data table from numpy columns (one array per column), split into chunks of chunk_size rows.
std::shared_ptr<Table> table_from_arrays(const std::vector<std::tuple<std::string, DataType, bool>>& defs_in,
                                         const std::vector<py::array>& arrays, const std::vector<py::object>& nulls,
                                         uint32_t chunk_size) {
  TableColumnDefinitions defs;
  for (const auto& [n, t, nl] : defs_in) defs.emplace_back(n, t, nl);
  auto table = std::make_shared<Table>(defs, TableType::Data, chunk_size);
  Assert(arrays.size() == defs.size(), "one array per column");
  const size_t rows = arrays.empty() ? 0 : static_cast<size_t>(arrays[0].shape(0));
  for (size_t begin = 0; begin < rows; begin += chunk_size) {
    const size_t n = std::min<size_t>(chunk_size, rows - begin);
    ChunkColumns cols;
    for (size_t c = 0; c < defs.size(); ++c) {
      Assert(static_cast<size_t>(arrays[c].shape(0)) == rows, "columns must have equal length");
      std::optional<std::vector<uint8_t>> nv;
      if (defs[c].nullable) {
        nv.emplace(n, 0);
        if (c < nulls.size() && !nulls[c].is_none()) {
          auto na = nulls[c].cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
          std::memcpy(nv->data(), na.data() + begin, n);
        }
      }
      resolve_data_type(defs[c].data_type, [&](auto tag) {
        using T = decltype(tag);
        if constexpr (std::is_same_v<T, std::string>) {
          std::vector<std::string> v;
          for (size_t i = 0; i < n; ++i) v.push_back(py::str(arrays[c][py::int_(begin + i)]).cast<std::string>());
          cols.push_back(std::make_shared<ValueColumn<std::string>>(std::move(v), std::move(nv)));
        } else {
          auto a = py::array_t<T, py::array::c_style | py::array::forcecast>(arrays[c]);
          std::vector<T> v(a.data() + begin, a.data() + begin + n);
          cols.push_back(std::make_shared<ValueColumn<T>>(std::move(v), std::move(nv)));
        }
      });
    }
    table->append_chunk(cols);
  }
  return table;
}

py::list table_rows(const Table& t) {
  py::list rows;
  for (const auto& chunk : t.chunks()) {
    for (ChunkOffset o = 0; o < chunk->size(); ++o) {
      py::tuple row(chunk->column_count());
      for (ColumnID c = 0; c < chunk->column_count(); ++c) row[c] = to_py((*chunk->get_column(c))[o]);
      rows.append(row);
    }
  }
  return rows;
}

py::object parameter_to_py(const AllParameterVariant& p) {
  switch (p.index()) {
    case 0:
      return to_py(std::get<AllTypeVariant>(p));
    case 1:
      return py::cast(std::get<ColumnParameter>(p));
    default:
      return py::cast(std::get<ParameterID>(p));
  }
}

}  // namespace

PYBIND11_MODULE(_hyrise_host, m) {
  m.doc() = "Hyrise MI355X operator layer (host side)";

  py::register_exception<std::logic_error>(m, "LogicError", PyExc_RuntimeError);

  py::enum_<DataType>(m, "DataType")
      .value("Null", DataType::Null)
      .value("Int", DataType::Int)
      .value("Long", DataType::Long)
      .value("Float", DataType::Float)
      .value("Double", DataType::Double)
      .value("String", DataType::String);
  py::enum_<PredicateCondition>(m, "PredicateCondition")
      .value("Equals", PredicateCondition::Equals)
      .value("NotEquals", PredicateCondition::NotEquals)
      .value("LessThan", PredicateCondition::LessThan)
      .value("LessThanEquals", PredicateCondition::LessThanEquals)
      .value("GreaterThan", PredicateCondition::GreaterThan)
      .value("GreaterThanEquals", PredicateCondition::GreaterThanEquals)
      .value("Between", PredicateCondition::Between)
      .value("In", PredicateCondition::In)
      .value("Like", PredicateCondition::Like)
      .value("NotLike", PredicateCondition::NotLike)
      .value("IsNull", PredicateCondition::IsNull)
      .value("IsNotNull", PredicateCondition::IsNotNull);
  py::enum_<JoinMode>(m, "JoinMode")
      .value("Inner", JoinMode::Inner)
      .value("Left", JoinMode::Left)
      .value("Right", JoinMode::Right)
      .value("Outer", JoinMode::Outer)
      .value("Cross", JoinMode::Cross)
      .value("Semi", JoinMode::Semi)
      .value("Anti", JoinMode::Anti);
  py::enum_<TableType>(m, "TableType").value("References", TableType::References).value("Data", TableType::Data);
  py::enum_<EncodingType>(m, "EncodingType")
      .value("Unencoded", EncodingType::Unencoded)
      .value("Dictionary", EncodingType::Dictionary)
      .value("RunLength", EncodingType::RunLength)
      .value("FixedStringDictionary", EncodingType::FixedStringDictionary)
      .value("FrameOfReference", EncodingType::FrameOfReference);
  py::enum_<VectorCompressionType>(m, "VectorCompressionType")
      .value("FixedSizeByteAligned", VectorCompressionType::FixedSizeByteAligned)
      .value("SimdBp128", VectorCompressionType::SimdBp128);
  py::enum_<AggregateFunction>(m, "AggregateFunction")
      .value("Min", AggregateFunction::Min)
      .value("Max", AggregateFunction::Max)
      .value("Sum", AggregateFunction::Sum)
      .value("Avg", AggregateFunction::Avg)
      .value("Count", AggregateFunction::Count)
      .value("CountDistinct", AggregateFunction::CountDistinct);

  py::class_<BaseColumn, std::shared_ptr<BaseColumn>>(m, "BaseColumn")
      .def("size", &BaseColumn::size)
      .def("__len__", &BaseColumn::size)
      .def("data_type", &BaseColumn::data_type)
      .def("encoding_type", &BaseColumn::encoding_type)
      .def("is_reference", &BaseColumn::is_reference)
      .def("__getitem__", [](const BaseColumn& c, uint32_t o) {
        if (o >= c.size()) throw py::index_error();
        return to_py(c[o]);
      })
      .def("values", [](const BaseColumn& c) {
        py::list l;
        for (ChunkOffset o = 0; o < c.size(); ++o) l.append(to_py(c[o]));
        return l;
      })
      .def("attribute_vector_width", [](const BaseColumn& c) -> int {
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        return d->attribute_vector().width();
      })
      .def("attribute_vector_compression", [](const BaseColumn& c) {
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        return d->attribute_vector().compression();
      })
      .def("attribute_vector_bytes", [](const BaseColumn& c) {  // FSBA ids or the SIMD-BP128 words
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        const auto& b = d->attribute_vector().bytes();
        return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
      })
      .def("attribute_vector_ids", [](const BaseColumn& c) {  // every id through the vector's own decoder
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        const auto& av = d->attribute_vector();
        std::vector<uint32_t> out(av.size());
        for (size_t i = 0; i < out.size(); ++i) out[i] = av.get(i);
        return out;
      })
      .def("lower_bound", [](const BaseColumn& c, py::object v) {
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        return d->lower_bound(to_variant(v));
      })
      .def("upper_bound", [](const BaseColumn& c, py::object v) {
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        return d->upper_bound(to_variant(v));
      })
      .def("unique_values_count", [](const BaseColumn& c) {
        const auto* d = dynamic_cast<const BaseDictionaryColumn*>(&c);
        Assert(d != nullptr, "not a dictionary column");
        return d->unique_values_count();
      });

  py::class_<ReferenceColumn, BaseColumn, std::shared_ptr<ReferenceColumn>>(m, "ReferenceColumn")
      .def(py::init([](std::shared_ptr<Table> t, ColumnID c, py::array_t<uint32_t> pl) {
             return std::make_shared<ReferenceColumn>(t, c, pos_list_from_array(pl));
           }),
           py::arg("referenced_table"), py::arg("referenced_column_id"), py::arg("pos_list"))
      .def("pos_list",
           [](const ReferenceColumn& c) {
             const auto& pl = *c.pos_list();
             {
               py::gil_scoped_release release;  // (a lazy list's first host access copies it down)
               static_cast<void>(pl.data());
             }
             return pos_list_array(pl);
           })
      .def("pos_list_id", [](const ReferenceColumn& c) { return reinterpret_cast<uintptr_t>(c.pos_list().get()); })
      .def("referenced_table", [](const ReferenceColumn& c) { return std::const_pointer_cast<Table>(c.referenced_table()); })
      .def("referenced_column_id", &ReferenceColumn::referenced_column_id)
      .def("referenced_table_id",
           [](const ReferenceColumn& c) { return reinterpret_cast<uintptr_t>(c.referenced_table().get()); });

  py::class_<Chunk, std::shared_ptr<Chunk>>(m, "Chunk")
      .def("set_mvcc_columns",
           [](Chunk& c, py::array_t<uint32_t> tids, py::array_t<uint32_t> begin, py::array_t<uint32_t> end) {
             auto m = std::make_shared<MvccColumns>();
             auto copy = [](py::array_t<uint32_t>& a, std::vector<uint32_t>& v) {
               auto r = a.unchecked<1>();
               v.resize(r.shape(0));
               for (py::ssize_t i = 0; i < r.shape(0); ++i) v[i] = r(i);
             };
             copy(tids, m->tids);
             copy(begin, m->begin_cids);
             copy(end, m->end_cids);
             c.set_mvcc_columns(m);
           },
           py::arg("tids"), py::arg("begin_cids"), py::arg("end_cids"))
      .def("has_mvcc_columns", &Chunk::has_mvcc_columns)
      .def("size", &Chunk::size)
      .def("column_count", &Chunk::column_count)
      .def("get_column", &Chunk::get_column);

  py::class_<Table, std::shared_ptr<Table>>(m, "Table")
      .def(py::init([](const std::vector<std::tuple<std::string, DataType, bool>>& defs, TableType type,
                       uint32_t chunk_size) {
             TableColumnDefinitions d;
             for (const auto& [n, t, nl] : defs) d.emplace_back(n, t, nl);
             return std::make_shared<Table>(d, type, chunk_size);
           }),
           py::arg("column_definitions"), py::arg("type") = TableType::Data, py::arg("chunk_size") = CHUNK_MAX_SIZE)
      .def_static("from_arrays", &table_from_arrays, py::arg("column_definitions"), py::arg("arrays"),
                  py::arg("nulls") = std::vector<py::object>{}, py::arg("chunk_size") = CHUNK_MAX_SIZE)
      .def("id", [](const Table& t) { return reinterpret_cast<uintptr_t>(&t); })
      .def("type", &Table::type)
      .def("column_count", &Table::column_count)
      .def("row_count", &Table::row_count)
      .def("chunk_count", &Table::chunk_count)
      .def("max_chunk_size", &Table::max_chunk_size)
      .def("column_name", &Table::column_name)
      .def("column_names", &Table::column_names)
      .def("column_data_type", &Table::column_data_type)
      .def("column_is_nullable", &Table::column_is_nullable)
      .def("column_id_by_name", &Table::column_id_by_name)
      .def("get_chunk", &Table::get_chunk)
      .def("append", [](Table& t, const py::list& values) {
        std::vector<AllTypeVariant> v;
        for (auto o : values) v.push_back(to_variant(o));
        t.append(v);
      })
      .def("append_chunk", [](Table& t, const std::vector<std::shared_ptr<BaseColumn>>& cols) { t.append_chunk(cols); })
      .def("get_value", [](const Table& t, ColumnID c, uint64_t r) { return to_py(t.get_value(c, r)); })
      .def("rows", [](const Table& t) { return table_rows(t); })
      .def("column_definitions", [](const Table& t) {
        py::list l;
        for (const auto& d : t.column_definitions()) l.append(py::make_tuple(d.name, d.data_type, d.nullable));
        return l;
      });

  m.def("load_table", &load_table, py::arg("file_name"), py::arg("chunk_size") = CHUNK_MAX_SIZE);
  m.def("import_binary", &import_binary, py::arg("filename"));
  m.def("export_binary", [](std::shared_ptr<Table> t, const std::string& f) { export_binary(t, f); },
        py::arg("table"), py::arg("filename"));
  m.def("load_to_device", [](std::shared_ptr<Table> t) { load_to_device(t); }, py::arg("table"));
  // the attribute-vector compressor on its own (SIMD-BP128 / FixedSizeByteAligned): (bytes, meta offsets, ids read
  // back through the vector's decoder) - for the parity tests of the packing
  m.def("compress_vector", [](const std::vector<uint32_t>& ids, uint32_t max_value, VectorCompressionType c) {
    const AttributeVector av(ids, max_value, c);
    std::vector<uint32_t> back(av.size());
    for (size_t i = 0; i < back.size(); ++i) back[i] = av.get(i);
    const auto& b = av.bytes();
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(b.data()), b.size()), av.meta_offsets(), back,
                          av.width());
  });
  m.def("encode_chunks", &ChunkEncoder::encode_chunks, py::arg("table"), py::arg("chunk_ids"), py::arg("encoding"),
        py::arg("vector_compression") = VectorCompressionType::FixedSizeByteAligned);
  m.def("encode_all_chunks", &ChunkEncoder::encode_all_chunks, py::arg("table"), py::arg("encoding"),
        py::arg("vector_compression") = VectorCompressionType::FixedSizeByteAligned);
  m.def("encode_columns", &ChunkEncoder::encode_columns, py::arg("table"), py::arg("column_ids"), py::arg("encoding"),
        py::arg("vector_compression") = VectorCompressionType::FixedSizeByteAligned);
  m.def("synchronize", []() { hy_check(hy_stream_synchronize(operator_stream()), "hy_stream_synchronize"); },
        "Waits for the calling thread's operator stream (operator outputs are produced asynchronously).");
  m.def("join_hashed_type", &join_hashed_type);
  m.def("join_radix_bits", [](uint64_t rows, uint32_t key_bytes) { return hy_join_radix_bits(rows, key_bytes); });
  m.def("device_count", []() {
    int n = 0;
    hy_get_device_count(&n);
    return n;
  });
  m.def("build_info", []() { return std::string(hy_build_info()); });
  m.def("op_trace_enable", &op_trace_enable, py::arg("on"));
  m.def("join_plan_cache_stats", &join_plan_cache_stats);
  m.def("join_plan_cache_clear", &join_plan_cache_clear);
  m.def("join_plan_cache_set_capacity", &join_plan_cache_set_capacity, py::arg("plans"));
  m.def("op_trace_take", []() {
    py::list l;
    for (const auto& r : op_trace_take()) l.append(py::make_tuple(r.op, r.phase, r.ms));
    return l;
  });
  m.def("pool_stats", []() {
    uint64_t reserved = 0, used = 0;
    hy_check(hy_pool_stats(&reserved, &used), "hy_pool_stats");
    return py::make_tuple(reserved, used);
  });
  m.def("host_cpu_share", &host_cpu_share);
  m.def("release_drain", &release_drain, py::call_guard<py::gil_scoped_release>(),
        "wait until the chunks of dropped large tables (destroyed on a background thread) are gone");
  m.def("device_memory", []() {
    uint64_t free_b = 0, total_b = 0;
    hy_check(hy_device_memory(&free_b, &total_b), "hy_device_memory");
    return py::make_tuple(free_b, total_b);
  });

  py::class_<OperatorPerformanceData>(m, "OperatorPerformanceData")
      .def_readonly("walltime_ns", &OperatorPerformanceData::walltime_ns)
      .def_readonly("rows_in", &OperatorPerformanceData::rows_in)
      .def_readonly("device_ns", &OperatorPerformanceData::device_ns)
      .def_readonly("bytes_read", &OperatorPerformanceData::bytes_read)
      .def_readonly("bytes_written", &OperatorPerformanceData::bytes_written);

  // the host scheduler the operators submit their jobs to (scheduler.hpp): "pool" (n workers fed from one queue),
  // "inline" (jobs run when scheduled) or None (a thread per job)
  m.def(
      "set_job_scheduler",
      [](py::object kind, unsigned workers) {
        if (kind.is_none()) return set_job_scheduler(nullptr);
        const std::string k = kind.cast<std::string>();
        if (k == "pool") return set_job_scheduler(make_pool_scheduler(workers));
        if (k == "inline") return set_job_scheduler(make_inline_scheduler());
        throw std::invalid_argument("job scheduler kind: pool, inline or None");
      },
      py::arg("kind"), py::arg("workers") = 4);

  py::enum_<DescriptionMode>(m, "DescriptionMode")
      .value("SingleLine", DescriptionMode::SingleLine)
      .value("MultiLine", DescriptionMode::MultiLine);

  py::class_<AbstractOperator, std::shared_ptr<AbstractOperator>>(m, "AbstractOperator")
      .def("execute", &AbstractOperator::execute, py::call_guard<py::gil_scoped_release>())
      .def("get_output", [](const AbstractOperator& o) { return std::const_pointer_cast<Table>(o.get_output()); })
      .def("name", &AbstractOperator::name)
      .def("description", &AbstractOperator::description, py::arg("description_mode") = DescriptionMode::SingleLine)
      .def("performance_data", &AbstractOperator::performance_data)
      .def("deep_copy", &AbstractOperator::deep_copy)
      .def("set_parameters",
           [](AbstractOperator& o, const py::dict& parameters) { o.set_parameters(to_parameter_map(parameters)); },
           py::arg("parameters"))
      .def("input_left", [](const AbstractOperator& o) { return o.mutable_input_left(); })
      .def("input_right", [](const AbstractOperator& o) { return o.mutable_input_right(); })
      .def(
          "set_transaction_context_recursively",
          [](AbstractOperator& o, std::shared_ptr<TransactionContext> c) { o.set_transaction_context_recursively(c); },
          py::keep_alive<1, 2>())
      // the operator holds its context weakly (abstract_operator.cpp:95-98); Python keeps it alive with the operator
      .def(
          "set_transaction_context",
          [](AbstractOperator& o, std::shared_ptr<TransactionContext> c) { o.set_transaction_context(c); },
          py::keep_alive<1, 2>())
      .def("transaction_context", &AbstractOperator::transaction_context);

  py::class_<TableWrapper, AbstractOperator, std::shared_ptr<TableWrapper>>(m, "TableWrapper")
      .def(py::init<std::shared_ptr<const Table>>());

  py::class_<ColumnParameter>(m, "ColumnParameter")
      .def(py::init([](ColumnID c) { return ColumnParameter{c}; }), py::arg("column_id"))
      .def_readonly("column_id", &ColumnParameter::column_id)
      .def("__eq__", [](const ColumnParameter& a, const ColumnParameter& b) { return a == b; })
      .def("__repr__", [](const ColumnParameter& c) { return "ColumnParameter(" + std::to_string(c.column_id) + ")"; });
  py::class_<ParameterID>(m, "ParameterID")
      .def(py::init([](size_t id) { return ParameterID{id}; }), py::arg("id"))
      .def_readonly("id", &ParameterID::t)
      .def("__eq__", [](const ParameterID& a, const ParameterID& b) { return a == b; })
      .def("__hash__", [](const ParameterID& p) { return ParameterIDHash{}(p); })
      .def("__repr__", [](const ParameterID& p) { return "ParameterID(" + std::to_string(p.t) + ")"; });
  py::class_<TableScan, AbstractOperator, std::shared_ptr<TableScan>>(m, "TableScan")
      .def(py::init([](std::shared_ptr<AbstractOperator> in, ColumnID col, PredicateCondition cond, py::object value) {
             if (py::isinstance<ColumnParameter>(value))
               return std::make_shared<TableScan>(in, col, cond, value.cast<ColumnParameter>());
             if (py::isinstance<ParameterID>(value))
               return std::make_shared<TableScan>(in, col, cond, value.cast<ParameterID>());
             return std::make_shared<TableScan>(in, col, cond, to_variant(value));
           }),
           py::arg("input"), py::arg("column_id"), py::arg("predicate_condition"), py::arg("value"))
      .def("left_column_id", &TableScan::left_column_id)
      .def("predicate_condition", &TableScan::predicate_condition)
      .def("right_parameter", [](const TableScan& t) { return parameter_to_py(t.right_parameter()); })
      .def("set_excluded_chunk_ids", &TableScan::set_excluded_chunk_ids);

  py::class_<TransactionContext, std::shared_ptr<TransactionContext>>(m, "TransactionContext")
      .def(py::init<uint32_t, uint32_t>(), py::arg("transaction_id"), py::arg("snapshot_commit_id"))
      .def("transaction_id", &TransactionContext::transaction_id)
      .def("snapshot_commit_id", &TransactionContext::snapshot_commit_id)
      .def("aborted", &TransactionContext::aborted)
      .def("set_aborted", &TransactionContext::set_aborted);
  py::class_<Validate, AbstractOperator, std::shared_ptr<Validate>>(m, "Validate")
      .def(py::init<std::shared_ptr<AbstractOperator>>(), py::arg("input"));
  m.attr("MAX_COMMIT_ID") = MvccColumns::MAX_COMMIT_ID;
  py::class_<JoinHash, AbstractOperator, std::shared_ptr<JoinHash>>(m, "JoinHash")
      .def(py::init([](std::shared_ptr<AbstractOperator> l, std::shared_ptr<AbstractOperator> r, JoinMode mode,
                       std::pair<ColumnID, ColumnID> cols, PredicateCondition cond, size_t radix_bits) {
             return std::make_shared<JoinHash>(l, r, mode, cols, cond, radix_bits);
           }),
           py::arg("left"), py::arg("right"), py::arg("mode"), py::arg("column_ids"), py::arg("predicate_condition"),
           py::arg("radix_bits") = 9)
      .def("used_radix_bits", &JoinHash::used_radix_bits)
      .def("mode", &JoinHash::mode)
      .def("column_ids", &JoinHash::column_ids)
      .def("predicate_condition", &JoinHash::predicate_condition);

  py::class_<AggregateColumnDefinition>(m, "AggregateColumnDefinition")
      .def(py::init<std::optional<ColumnID>, AggregateFunction>(), py::arg("column"), py::arg("function"))
      .def_readonly("column", &AggregateColumnDefinition::column)
      .def_readonly("function", &AggregateColumnDefinition::function);

  py::class_<Aggregate, AbstractOperator, std::shared_ptr<Aggregate>>(m, "Aggregate")
      .def(py::init<std::shared_ptr<const AbstractOperator>, std::vector<AggregateColumnDefinition>,
                    std::vector<ColumnID>>(),
           py::arg("input"), py::arg("aggregates"), py::arg("groupby_column_ids"))
      .def("used_dense_path", &Aggregate::used_dense_path)
      .def("aggregates", &Aggregate::aggregates)
      .def("groupby_column_ids", &Aggregate::groupby_column_ids);

  // ---- Projection and its expressions (reference expression/*.hpp, operators/projection.hpp)
  py::enum_<ArithmeticOperator>(m, "ArithmeticOperator")
      .value("Addition", ArithmeticOperator::Addition)
      .value("Subtraction", ArithmeticOperator::Subtraction)
      .value("Multiplication", ArithmeticOperator::Multiplication)
      .value("Division", ArithmeticOperator::Division)
      .value("Modulo", ArithmeticOperator::Modulo);
  py::class_<AbstractExpression, std::shared_ptr<AbstractExpression>>(m, "AbstractExpression")
      .def("data_type", &AbstractExpression::data_type)
      .def("is_nullable", &AbstractExpression::is_nullable)
      .def("as_column_name", &AbstractExpression::as_column_name)
      .def("deep_copy", &AbstractExpression::deep_copy);
  py::class_<PQPColumnExpression, AbstractExpression, std::shared_ptr<PQPColumnExpression>>(m, "PQPColumnExpression")
      .def(py::init<ColumnID, DataType, bool, std::string>(), py::arg("column_id"), py::arg("data_type"),
           py::arg("nullable"), py::arg("column_name"))
      .def_static("from_table", &PQPColumnExpression::from_table, py::arg("table"), py::arg("column_id"))
      .def_readonly("column_id", &PQPColumnExpression::column_id);
  py::class_<ValueExpression, AbstractExpression, std::shared_ptr<ValueExpression>>(m, "ValueExpression")
      .def(py::init([](py::object v) { return std::make_shared<ValueExpression>(to_variant(v)); }), py::arg("value"))
      .def(py::init([](py::object v, DataType t) {
             // a literal of an explicit type (Python numbers are int32/int64/double otherwise)
             AllTypeVariant var = to_variant(v);
             if (!variant_is_null(var)) resolve_data_type(t, [&](auto tag) { var = type_cast<decltype(tag)>(var); });
             return std::make_shared<ValueExpression>(var);
           }),
           py::arg("value"), py::arg("data_type"))
      .def_property_readonly("value", [](const ValueExpression& e) { return to_py(e.value); });
  py::class_<ParameterExpression, AbstractExpression, std::shared_ptr<ParameterExpression>>(m, "ParameterExpression")
      .def(py::init([](size_t id) { return std::make_shared<ParameterExpression>(ParameterID{id}); }),
           py::arg("parameter_id"))
      .def_property_readonly("parameter_id", [](const ParameterExpression& e) { return e.parameter_id.t; })
      .def_property_readonly("value", [](const ParameterExpression& e) -> py::object {
        return e.value() ? to_py(*e.value()) : py::object(py::none());
      })
      .def_property_readonly("has_value", [](const ParameterExpression& e) { return e.value().has_value(); });
  py::class_<ArithmeticExpression, AbstractExpression, std::shared_ptr<ArithmeticExpression>>(m, "ArithmeticExpression")
      .def(py::init<ArithmeticOperator, std::shared_ptr<AbstractExpression>, std::shared_ptr<AbstractExpression>>(),
           py::arg("arithmetic_operator"), py::arg("left_operand"), py::arg("right_operand"))
      .def_readonly("arithmetic_operator", &ArithmeticExpression::arithmetic_operator)
      .def("left_operand", &ArithmeticExpression::left_operand)
      .def("right_operand", &ArithmeticExpression::right_operand);
  m.def("expression_common_type", &expression_common_type);
  py::class_<Projection, AbstractOperator, std::shared_ptr<Projection>>(m, "Projection")
      .def(py::init<std::shared_ptr<const AbstractOperator>, std::vector<std::shared_ptr<AbstractExpression>>>(),
           py::arg("input"), py::arg("expressions"))
      .def_readonly("expressions", &Projection::expressions);
}
