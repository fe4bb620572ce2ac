// Projection operator (reference src/lib/operators/projection.cpp:39-87) and the expression properties it needs.
// Arithmetic is evaluated on the device through hy_projection (include/hyrise_amd.h); the host compiles each
// expression tree into the C-ABI's postfix program with the reference's type rules and builds the Data table.
#include <algorithm>
#include <cstring>
#include <map>

#include "operators.hpp"

namespace hyrise {

// ================================================================================================================
// Expressions
// ================================================================================================================
DataType expression_common_type(DataType lhs, DataType rhs) {
  Assert(lhs != DataType::Null || rhs != DataType::Null, "Can't deduce common type if both sides are NULL");
  Assert((lhs == DataType::String) == (rhs == DataType::String), "Strings only compatible with strings");
  if (lhs == DataType::Null) return rhs;
  if (rhs == DataType::Null) return lhs;
  if (lhs == DataType::String) return DataType::String;
  auto is_float = [](DataType t) { return t == DataType::Float || t == DataType::Double; };
  if (lhs == DataType::Double || rhs == DataType::Double) return DataType::Double;
  if (lhs == DataType::Long) return is_float(rhs) ? DataType::Double : DataType::Long;
  if (rhs == DataType::Long) return is_float(lhs) ? DataType::Double : DataType::Long;
  if (lhs == DataType::Float || rhs == DataType::Float) return DataType::Float;
  return DataType::Int;
}

DataType cpp_common_type(DataType lhs, DataType rhs) {
  auto rank = [](DataType t) {
    switch (t) {
      case DataType::Int:
        return 0;
      case DataType::Long:
        return 1;
      case DataType::Float:
        return 2;
      case DataType::Double:
        return 3;
      default:
        return -1;
    }
  };
  if (lhs == DataType::Null) return rhs;
  if (rhs == DataType::Null) return lhs;
  return rank(lhs) >= rank(rhs) ? lhs : rhs;
}

DataType data_type_of_variant(const AllTypeVariant& v) {
  switch (v.index()) {
    case 1:
      return DataType::Int;
    case 2:
      return DataType::Long;
    case 3:
      return DataType::Float;
    case 4:
      return DataType::Double;
    case 5:
      return DataType::String;
    default:
      return DataType::Null;
  }
}

std::string arithmetic_operator_to_string(ArithmeticOperator op) {  // arithmetic_expression.cpp:10-28
  switch (op) {
    case ArithmeticOperator::Addition:
      return "+";
    case ArithmeticOperator::Subtraction:
      return "-";
    case ArithmeticOperator::Multiplication:
      return "*";
    case ArithmeticOperator::Division:
      return "/";
    default:
      return "%";
  }
}

std::shared_ptr<PQPColumnExpression> PQPColumnExpression::from_table(const Table& table, ColumnID column_id) {
  return std::make_shared<PQPColumnExpression>(column_id, table.column_data_type(column_id),
                                               table.column_is_nullable(column_id), table.column_name(column_id));
}

DataType ValueExpression::data_type() const { return data_type_of_variant(value); }

std::string ValueExpression::as_column_name() const {  // value_expression.cpp:19-29: operator<< of the value
  std::ostringstream stream;
  std::visit(
      [&](const auto& v) {
        using V = std::decay_t<decltype(v)>;
        if constexpr (std::is_same_v<V, NullValue>)
          stream << "NULL";
        else if constexpr (std::is_same_v<V, std::string>)
          stream << "'" << v << "'";
        else
          stream << v;
      },
      value);
  return stream.str();
}

DataType ParameterExpression::data_type() const {
  Assert(_value.has_value(), "Can't obtain type of unset ValuePlaceholder");
  return data_type_of_variant(*_value);
}

bool ParameterExpression::is_nullable() const {
  Assert(_value.has_value(), "Can't obtain nullability of unset ValuePlaceholder");
  return variant_is_null(*_value);
}

std::string ParameterExpression::as_column_name() const {
  std::ostringstream stream;
  stream << "Parameter[id=" << parameter_id.t << "]";
  if (_value) {
    stream << "=";
    std::visit(
        [&](const auto& v) {
          if constexpr (std::is_same_v<std::decay_t<decltype(v)>, NullValue>)
            stream << "NULL";
          else
            stream << v;
        },
        *_value);
  }
  return stream.str();
}

void expressions_set_parameters(const std::vector<std::shared_ptr<AbstractExpression>>& expressions,
                                const std::unordered_map<ParameterID, AllTypeVariant, ParameterIDHash>& parameters) {
  for (const auto& e : expressions) {
    if (e->type == ExpressionType::Parameter) {
      auto& p = static_cast<ParameterExpression&>(*e);
      const auto it = parameters.find(p.parameter_id);
      if (it != parameters.end()) p.set_value(it->second);
    } else {
      expressions_set_parameters(e->arguments, parameters);
    }
  }
}

std::vector<std::shared_ptr<AbstractExpression>> expressions_deep_copy(
    const std::vector<std::shared_ptr<AbstractExpression>>& expressions) {
  std::vector<std::shared_ptr<AbstractExpression>> out;
  out.reserve(expressions.size());
  for (const auto& e : expressions) out.push_back(e->deep_copy());
  return out;
}

DataType ArithmeticExpression::data_type() const {
  return expression_common_type(left_operand()->data_type(), right_operand()->data_type());
}

std::string ArithmeticExpression::as_column_name() const {
  return enclose_argument_as_column_name(*left_operand()) + " " + arithmetic_operator_to_string(arithmetic_operator) +
         " " + enclose_argument_as_column_name(*right_operand());
}

// ================================================================================================================
// Projection
// ================================================================================================================
namespace {

int32_t expr_kind(ArithmeticOperator op) {
  switch (op) {
    case ArithmeticOperator::Addition:
      return HY_EXPR_ADD;
    case ArithmeticOperator::Subtraction:
      return HY_EXPR_SUB;
    case ArithmeticOperator::Multiplication:
      return HY_EXPR_MUL;
    case ArithmeticOperator::Division:
      return HY_EXPR_DIV;
    default:
      return HY_EXPR_MOD;
  }
}

// Device input of one expression: the input columns its leaves reference (hy_agg_input column model).
struct ExprInput {
  std::vector<ColumnID> column_ids;                    // input column of each device column
  std::vector<std::vector<hy_column_chunk>> chunks;    // per device column
  std::vector<hy_agg_column> columns;
  std::vector<std::vector<const PosList*>> group_keys;  // PosList groups (reference input)
  std::vector<std::vector<std::shared_ptr<const PosList>>> group_lists;
};

int32_t add_input_column(ExprInput& ei, const Table& in, ColumnID col) {
  for (size_t i = 0; i < ei.column_ids.size(); ++i)
    if (ei.column_ids[i] == col) return static_cast<int32_t>(i);
  Assert(in.column_data_type(col) != DataType::String, "hyrise-amd: arithmetic on a string column");
  hy_agg_column desc{};
  desc.value_type = hy_type_of(in.column_data_type(col));
  desc.pos_group = -1;
  std::vector<hy_column_chunk> chunks;
  if (in.type() == TableType::Data) {
    for (ChunkID c = 0; c < in.chunk_count(); ++c) chunks.push_back(device_column(*in.get_chunk(c)->get_column(col))->desc);
  } else {
    std::vector<const PosList*> key;
    std::vector<std::shared_ptr<const PosList>> lists;
    std::shared_ptr<const Table> referenced;
    ColumnID rcol = 0;
    for (ChunkID c = 0; c < in.chunk_count(); ++c) {
      const auto rc = std::dynamic_pointer_cast<const ReferenceColumn>(in.get_chunk(c)->get_column(col));
      Assert(rc != nullptr, "All columns should be of type ReferenceColumn.");
      if (!referenced) {
        referenced = rc->referenced_table();
        rcol = rc->referenced_column_id();
      }
      Assert(rc->referenced_table() == referenced && rc->referenced_column_id() == rcol,
             "hyrise-amd: a projection column referencing several tables is not supported");
      key.push_back(rc->pos_list().get());
      lists.push_back(rc->pos_list());
    }
    auto it = std::find(ei.group_keys.begin(), ei.group_keys.end(), key);
    if (it == ei.group_keys.end()) {
      ei.group_keys.push_back(key);
      ei.group_lists.push_back(lists);
      it = ei.group_keys.end() - 1;
    }
    desc.pos_group = static_cast<int32_t>(it - ei.group_keys.begin());
    if (referenced)
      for (ChunkID r = 0; r < referenced->chunk_count(); ++r)
        chunks.push_back(device_column(*referenced->get_chunk(r)->get_column(rcol))->desc);
  }
  ei.column_ids.push_back(col);
  ei.chunks.push_back(std::move(chunks));
  ei.columns.push_back(desc);
  Assert(ei.columns.size() <= HY_AGG_MAX_COLUMNS, "hyrise-amd: too many columns in one projection expression");
  return static_cast<int32_t>(ei.columns.size() - 1);
}

// Postfix program of an expression tree (left operand, right operand, operator).
void compile(const AbstractExpression& e, const Table& in, ExprInput& ei, std::vector<hy_expr_node>& prog) {
  hy_expr_node n{};
  switch (e.type) {
    case ExpressionType::PQPColumn: {
      const auto& c = static_cast<const PQPColumnExpression&>(e);
      n.kind = HY_EXPR_COLUMN;
      n.column = add_input_column(ei, in, c.column_id);
      n.type = hy_type_of(in.column_data_type(c.column_id));
      break;
    }
    case ExpressionType::Value:
    case ExpressionType::Parameter: {
      // a set placeholder evaluates as a literal of its value (the reference's evaluator reads value())
      const AllTypeVariant& value = e.type == ExpressionType::Value
                                        ? static_cast<const ValueExpression&>(e).value
                                        : [&]() -> const AllTypeVariant& {
        const auto& p = static_cast<const ParameterExpression&>(e);
        Assert(p.value().has_value(), "ParameterExpression: Parameter not set, cannot evaluate");
        return *p.value();
      }();
      n.kind = HY_EXPR_VALUE;
      n.type = hy_type_of(data_type_of_variant(value));  // 0 for NULL
      Assert(data_type_of_variant(value) != DataType::String, "hyrise-amd: arithmetic on a string literal");
      std::visit(
          [&](const auto& x) {
            using V = std::decay_t<decltype(x)>;
            if constexpr (std::is_arithmetic_v<V>) std::memcpy(&n.value, &x, sizeof(V));
          },
          value);
      break;
    }
    case ExpressionType::Arithmetic: {
      const auto& a = static_cast<const ArithmeticExpression&>(e);
      compile(*a.left_operand(), in, ei, prog);
      compile(*a.right_operand(), in, ei, prog);
      n.kind = expr_kind(a.arithmetic_operator);
      n.type = hy_type_of(a.data_type());
      n.calc_type = hy_type_of(cpp_common_type(a.left_operand()->data_type(), a.right_operand()->data_type()));
      break;
    }
  }
  prog.push_back(n);
  Assert(prog.size() <= HY_EXPR_MAX_NODES, "hyrise-amd: expression has too many nodes for the device projection");
}

// Distinct input columns an expression's leaves reference, beyond those already in `ei`.
void new_columns(const AbstractExpression& e, const ExprInput& ei, std::vector<ColumnID>& seen) {
  if (e.type == ExpressionType::PQPColumn) {
    const ColumnID c = static_cast<const PQPColumnExpression&>(e).column_id;
    if (std::find(ei.column_ids.begin(), ei.column_ids.end(), c) == ei.column_ids.end() &&
        std::find(seen.begin(), seen.end(), c) == seen.end())
      seen.push_back(c);
  } else if (e.type == ExpressionType::Arithmetic) {
    const auto& a = static_cast<const ArithmeticExpression&>(e);
    new_columns(*a.left_operand(), ei, seen);
    new_columns(*a.right_operand(), ei, seen);
  }
}

// Evaluates expressions over all chunks of `in` into one ValueColumn per chunk each: one hy_projection_multi launch
// per batch (the batch's expressions share the input columns, at most HY_AGG_MAX_COLUMNS, and RowID reads), one
// stream synchronisation per batch.
std::vector<std::vector<std::shared_ptr<BaseColumn>>> evaluate_on_device(
    const std::vector<const AbstractExpression*>& exprs, const Table& in) {
  hy_stream_t s = operator_stream();
  const uint32_t n_chunks = in.chunk_count();
  std::vector<uint32_t> sizes(n_chunks);
  std::vector<uint64_t> row_begin(n_chunks + 1, 0);
  for (ChunkID c = 0; c < n_chunks; ++c) {
    sizes[c] = static_cast<uint32_t>(in.get_chunk(c)->size());
    row_begin[c + 1] = row_begin[c] + sizes[c];
  }
  const uint64_t rows = row_begin[n_chunks];
  std::vector<std::vector<std::shared_ptr<BaseColumn>>> result(exprs.size());
  size_t next = 0;
  while (next < exprs.size()) {
    // the batch: expressions while their input columns fit one hy_agg_input
    ExprInput ei;
    std::vector<std::vector<hy_expr_node>> progs;
    const size_t first = next;
    while (next < exprs.size() && progs.size() < HY_PROJ_MAX_OUTPUTS) {
      std::vector<ColumnID> extra;
      new_columns(*exprs[next], ei, extra);
      if (!progs.empty() && ei.columns.size() + extra.size() > HY_AGG_MAX_COLUMNS) break;
      progs.emplace_back();
      compile(*exprs[next], in, ei, progs.back());
      ++next;
    }
    for (size_t j = 0; j < ei.columns.size(); ++j) {
      ei.columns[j].chunks = ei.chunks[j].data();
      ei.columns[j].n_chunks = static_cast<uint32_t>(ei.chunks[j].size());
    }
    std::vector<const hy_row_id*> pos_ptrs;
    for (const auto& lists : ei.group_lists)
      for (const auto& pl : lists) pos_ptrs.push_back(device_pos_list(*pl)->ptr());
    hy_agg_input hin{};
    hin.n_chunks = n_chunks;
    hin.chunk_sizes = sizes.data();
    hin.pos_lists = pos_ptrs.data();
    hin.n_pos_groups = static_cast<uint32_t>(ei.group_lists.size());
    hin.columns = ei.columns.data();
    hin.n_columns = static_cast<uint32_t>(ei.columns.size());
    Assert(hin.n_pos_groups <= HY_AGG_MAX_POS_GROUPS, "hyrise-amd: too many PosList groups for the device projection");

    const size_t n = progs.size();
    std::vector<std::shared_ptr<DeviceBuffer>> values(n), nulls(n);
    std::vector<const hy_expr_node*> prog_ptrs(n);
    std::vector<uint32_t> prog_lens(n);
    std::vector<void*> outs(n);
    std::vector<uint8_t*> out_nulls(n);
    for (size_t i = 0; i < n; ++i) {
      const AbstractExpression& e = *exprs[first + i];
      values[i] = std::make_shared<DeviceBuffer>(std::max<uint64_t>(rows, 1) * data_type_size(e.data_type()) + 16);
      nulls[i] = e.is_nullable() ? std::make_shared<DeviceBuffer>(std::max<uint64_t>(rows, 1) + 16) : nullptr;
      prog_ptrs[i] = progs[i].data();
      prog_lens[i] = static_cast<uint32_t>(progs[i].size());
      outs[i] = values[i]->get();
      out_nulls[i] = nulls[i] ? nulls[i]->as<uint8_t>() : nullptr;
    }
    size_t ws_bytes = 0;
    hy_check(hy_projection_workspace_size(&hin, &ws_bytes), "hy_projection_workspace_size");
    DeviceBuffer ws(ws_bytes, s);
    hy_check(hy_projection_multi(&hin, prog_ptrs.data(), prog_lens.data(), static_cast<uint32_t>(n), outs.data(),
                                 out_nulls.data(), ws.get(), ws_bytes, s),
             "hy_projection_multi");

    for (size_t i = 0; i < n; ++i) {
      const AbstractExpression& e = *exprs[first + i];
      const bool nullable = e.is_nullable();
      auto& out = result[first + i];
      resolve_data_type(e.data_type(), [&](auto tag) {
        using T = decltype(tag);
        if constexpr (!std::is_same_v<T, std::string>) {
          std::vector<T> all(rows);
          std::vector<uint8_t> all_nulls(nullable ? rows : 0);
          if (rows) hy_check(hy_memcpy_dtoh(all.data(), values[i]->get(), rows * sizeof(T), s), "dtoh");
          if (nullable && rows) hy_check(hy_memcpy_dtoh(all_nulls.data(), nulls[i]->get(), rows, s), "dtoh");
          hy_check(hy_stream_synchronize(s), "sync");
          for (ChunkID c = 0; c < n_chunks; ++c) {
            std::vector<T> v(all.begin() + row_begin[c], all.begin() + row_begin[c + 1]);
            std::optional<std::vector<uint8_t>> nv;
            if (nullable) {
              nv.emplace(all_nulls.begin() + row_begin[c], all_nulls.begin() + row_begin[c + 1]);
              for (size_t r = 0; r < v.size(); ++r)
                if ((*nv)[r]) v[r] = T{};  // NULL rows hold T{} (the device leaves them unspecified)
            }
            auto col = std::make_shared<ValueColumn<T>>(std::move(v), std::move(nv));
            // the result already is in HBM: its slice becomes the column's device mirror when 16-byte aligned
            const uint64_t off = row_begin[c] * sizeof(T);
            if (!nullable && off % 16 == 0) {
              auto d = std::make_shared<DeviceColumn>();
              d->data = values[i];
              d->desc.data = static_cast<char*>(values[i]->get()) + off;
              d->desc.size = sizes[c];
              d->desc.kind = HY_COL_VALUE;
              col->set_device_mirror(d);
            }
            out.push_back(col);
          }
        }
      });
    }
  }
  return result;
}

// A column of a reference table materialized on the host (string columns, which the device holds only as
// dictionary codes): the reference's evaluate_expression_to_column of a PQPColumnExpression.
std::vector<std::shared_ptr<BaseColumn>> materialize_on_host(const Table& in, ColumnID col) {
  std::vector<std::shared_ptr<BaseColumn>> out;
  const bool nullable = in.column_is_nullable(col);
  resolve_data_type(in.column_data_type(col), [&](auto tag) {
    using T = decltype(tag);
    for (ChunkID c = 0; c < in.chunk_count(); ++c) {
      const auto src = in.get_chunk(c)->get_column(col);
      auto dst = std::make_shared<ValueColumn<T>>(nullable);
      for (ChunkOffset o = 0; o < src->size(); ++o) dst->append((*src)[o]);
      out.push_back(dst);
    }
  });
  return out;
}

}  // namespace

void Projection::_on_set_parameters(const ParameterMap& parameters) { expressions_set_parameters(expressions, parameters); }

std::shared_ptr<AbstractOperator> Projection::_on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                            const std::shared_ptr<AbstractOperator>&) const {
  return std::make_shared<Projection>(copied_input_left, expressions_deep_copy(expressions));
}

std::shared_ptr<const Table> Projection::_on_execute() {
  const auto in = input_table_left();
  TableColumnDefinitions defs;
  for (const auto& e : expressions) defs.emplace_back(e->as_column_name(), e->data_type(), e->is_nullable());
  const bool only_columns = std::all_of(expressions.begin(), expressions.end(),
                                        [](const auto& e) { return e->type == ExpressionType::PQPColumn; });
  const auto output_type = only_columns ? in->type() : TableType::Data;
  const bool forward = in->type() == output_type;
  auto output = std::make_shared<Table>(defs, output_type, in->max_chunk_size());
  _performance_data.rows_in = in->row_count();

  std::vector<std::vector<std::shared_ptr<BaseColumn>>> computed(expressions.size());
  std::vector<const AbstractExpression*> on_device;
  std::vector<size_t> device_index;
  for (size_t i = 0; i < expressions.size(); ++i) {
    const auto& e = *expressions[i];
    if (e.type == ExpressionType::PQPColumn && forward) continue;
    if (e.type == ExpressionType::PQPColumn &&
        in->column_data_type(static_cast<const PQPColumnExpression&>(e).column_id) == DataType::String) {
      computed[i] = materialize_on_host(*in, static_cast<const PQPColumnExpression&>(e).column_id);
      continue;
    }
    Assert(e.data_type() != DataType::String, "hyrise-amd: string-valued expressions are not supported");
    on_device.push_back(&e);
    device_index.push_back(i);
  }
  if (!on_device.empty()) {
    require_device();
    auto cols = evaluate_on_device(on_device, *in);
    for (size_t k = 0; k < cols.size(); ++k) computed[device_index[k]] = std::move(cols[k]);
  }
  for (ChunkID c = 0; c < in->chunk_count(); ++c) {
    ChunkColumns cols;
    for (size_t i = 0; i < expressions.size(); ++i) {
      const auto& e = *expressions[i];
      if (e.type == ExpressionType::PQPColumn && forward)
        cols.push_back(std::const_pointer_cast<BaseColumn>(
            in->get_chunk(c)->get_column(static_cast<const PQPColumnExpression&>(e).column_id)));
      else
        cols.push_back(computed[i][c]);
    }
    output->append_chunk(cols);
  }
  return output;
}

}  // namespace hyrise
