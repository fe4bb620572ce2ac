// Operator layer: the reference's AbstractOperator surface with GPU-backed TableScan / JoinHash / Aggregate.
//
//   AbstractOperator::execute / get_output / _on_execute   reference src/lib/operators/abstract_operator.cpp:25-67
//   AbstractReadOnlyOperator                               reference src/lib/operators/abstract_read_only_operator.hpp:12-33
//   AbstractJoinOperator (mode, column ids, predicate, description)
//                                                          reference src/lib/operators/abstract_join_operator.hpp:25-53
//   TableWrapper                                           reference src/lib/operators/table_wrapper.cpp
//   deep_copy / set_parameters / _on_deep_copy / _on_set_parameters
//                                                          reference src/lib/operators/abstract_operator.hpp:107-155
//   TableScan(in, ColumnID, PredicateCondition, AllParameterVariant)
//                                                          reference src/lib/operators/table_scan.hpp:22-23
//   JoinHash(l, r, JoinMode, ColumnIDPair, PredicateCondition, radix_bits = 9)
//                                                          reference src/lib/operators/join_hash.hpp:26-28
//   Aggregate(in, aggregates, groupby_column_ids)          reference src/lib/operators/aggregate.hpp:87-88
//
// The compute of TableScan / JoinHash / Aggregate runs in the gfx950 kernels behind include/hyrise_amd.h; there is
// no CPU fallback: without a device these operators throw.
#pragma once

#include <chrono>
#include <map>
#include <optional>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "device.hpp"
#include "expression.hpp"
#include "storage.hpp"

namespace hyrise {

enum class OperatorType { TableWrapper, TableScan, JoinHash, Aggregate, Projection, Validate, Mock };

// types.hpp:197 of the reference: how description() lays out an operator's parameters
enum class DescriptionMode { SingleLine, MultiLine };

// reference operator_performance_data.hpp:10-15 (walltime), extended at that documented extension point with what
// ran on the device: the time between the first and the last command the operator issued on its stream (device_ns:
// 0 when it issued none - a TableScan deferred into the JoinHash that consumes it is timed in that JoinHash), and the
// algorithmic HBM bytes its kernels read and wrote (SURVEY.md 8(d) per-unit figures: inputs' column bytes, output
// RowIDs / values), so that bytes / device_ns is the operator's achieved bandwidth.
struct OperatorPerformanceData {
  uint64_t walltime_ns = 0;  // reference operator_performance_data.hpp:15
  uint64_t rows_in = 0;
  uint64_t device_ns = 0;
  uint64_t bytes_read = 0;
  uint64_t bytes_written = 0;
};

// The part of the reference's TransactionContext (concurrency/transaction_context.hpp) the hot path reads: the
// transaction's id, its snapshot commit id and whether it aborted (AbstractOperator::execute skips the operator then,
// abstract_operator.cpp:32-48). Commit / rollback live in the out-of-scope transaction manager.
class TransactionContext {
 public:
  TransactionContext(uint32_t transaction_id, uint32_t snapshot_commit_id)
      : _transaction_id(transaction_id), _snapshot_commit_id(snapshot_commit_id) {}
  uint32_t transaction_id() const { return _transaction_id; }
  uint32_t snapshot_commit_id() const { return _snapshot_commit_id; }
  bool aborted() const { return _aborted; }
  void set_aborted() { _aborted = true; }

 private:
  uint32_t _transaction_id, _snapshot_commit_id;
  bool _aborted = false;
};

// A parameter's values by id: what set_parameters hands down a plan (reference abstract_operator.hpp:129).
using ParameterMap = std::unordered_map<ParameterID, AllTypeVariant, ParameterIDHash>;

// abstract_operator.hpp:70-172. Operators are not copyable (Noncopyable in the reference); deep_copy() makes a fresh,
// unexecuted plan of the same configuration.
class AbstractOperator : public std::enable_shared_from_this<AbstractOperator> {
 public:
  AbstractOperator(OperatorType type, std::shared_ptr<const AbstractOperator> left = nullptr,
                   std::shared_ptr<const AbstractOperator> right = nullptr)
      : _type(type), _input_left(std::move(left)), _input_right(std::move(right)) {}
  AbstractOperator(const AbstractOperator&) = delete;
  AbstractOperator& operator=(const AbstractOperator&) = delete;
  virtual ~AbstractOperator() = default;

  void execute();
  std::shared_ptr<const Table> get_output() const { return _output; }
  void clear_output() { _output.reset(); }

  OperatorType type() const { return _type; }
  virtual const std::string name() const = 0;
  // abstract_operator.hpp:93, abstract_operator.cpp:76
  virtual const std::string description(DescriptionMode description_mode = DescriptionMode::SingleLine) const {
    (void)description_mode;
    return name();
  }

  std::shared_ptr<const AbstractOperator> input_left() const { return _input_left; }
  std::shared_ptr<const AbstractOperator> input_right() const { return _input_right; }
  // abstract_operator.cpp:121-127: the inputs with const cast away
  std::shared_ptr<AbstractOperator> mutable_input_left() const {
    return std::const_pointer_cast<AbstractOperator>(_input_left);
  }
  std::shared_ptr<AbstractOperator> mutable_input_right() const {
    return std::const_pointer_cast<AbstractOperator>(_input_right);
  }
  std::shared_ptr<const Table> input_table_left() const { return _input_left->get_output(); }
  std::shared_ptr<const Table> input_table_right() const { return _input_right->get_output(); }
  const OperatorPerformanceData& performance_data() const { return _performance_data; }

  // abstract_operator.cpp:87-119: the operator's transaction (held weakly, as the reference does)
  bool transaction_context_is_set() const { return _transaction_context.has_value(); }
  void set_transaction_context(const std::weak_ptr<TransactionContext>& context) { _transaction_context = context; }
  std::shared_ptr<TransactionContext> transaction_context() const {
    return _transaction_context ? _transaction_context->lock() : nullptr;
  }
  void set_transaction_context_recursively(const std::weak_ptr<TransactionContext>& context);

  // abstract_operator.cpp:77-81, 157-173: a new instance of the same operator with the same configuration, inputs
  // copied recursively; an input shared by two consumers (a diamond) is copied once.
  std::shared_ptr<AbstractOperator> deep_copy() const;

  // abstract_operator.cpp:147-151: parameters set in this operator, then in both inputs
  void set_parameters(const ParameterMap& parameters);

 protected:
  // execute() calls the context overload (abstract_operator.cpp:47); AbstractReadOnlyOperator forwards it to the plain one
  virtual std::shared_ptr<const Table> _on_execute(std::shared_ptr<TransactionContext> transaction_context) = 0;
  virtual void _on_cleanup() {}
  virtual void _on_set_parameters(const ParameterMap& parameters) = 0;
  virtual std::shared_ptr<AbstractOperator> _on_deep_copy(
      const std::shared_ptr<AbstractOperator>& copied_input_left,
      const std::shared_ptr<AbstractOperator>& copied_input_right) const = 0;
  std::shared_ptr<AbstractOperator> _deep_copy_impl(
      std::unordered_map<const AbstractOperator*, std::shared_ptr<AbstractOperator>>& copied_ops) const;

  std::optional<std::weak_ptr<TransactionContext>> _transaction_context;

  const OperatorType _type;
  std::shared_ptr<const AbstractOperator> _input_left, _input_right;
  std::shared_ptr<const Table> _output;
  OperatorPerformanceData _performance_data;
};

// abstract_read_only_operator.hpp:12-33: the operators that do not write their inputs; only Validate reads the
// transaction context, the others implement the plain _on_execute().
class AbstractReadOnlyOperator : public AbstractOperator {
 public:
  using AbstractOperator::AbstractOperator;

 protected:
  std::shared_ptr<const Table> _on_execute(std::shared_ptr<TransactionContext>) override { return _on_execute(); }
  virtual std::shared_ptr<const Table> _on_execute() = 0;
};

// abstract_join_operator.hpp:25-53 / abstract_join_operator.cpp:9-45: a join of two inputs on one column pair; owns the
// mode, the column pair and the predicate, and the description every join shares.
class AbstractJoinOperator : public AbstractReadOnlyOperator {
 public:
  AbstractJoinOperator(OperatorType type, std::shared_ptr<const AbstractOperator> left,
                       std::shared_ptr<const AbstractOperator> right, JoinMode mode,
                       std::pair<ColumnID, ColumnID> column_ids, PredicateCondition predicate_condition)
      : AbstractReadOnlyOperator(type, std::move(left), std::move(right)),
        _mode(mode),
        _column_ids(column_ids),
        _predicate_condition(predicate_condition) {
    Assert(mode != JoinMode::Cross, "Specified JoinMode not supported by an AbstractJoin, use Product etc. instead.");
  }
  JoinMode mode() const { return _mode; }
  const std::pair<ColumnID, ColumnID>& column_ids() const { return _column_ids; }
  PredicateCondition predicate_condition() const { return _predicate_condition; }
  const std::string description(DescriptionMode description_mode = DescriptionMode::SingleLine) const override;

 protected:
  const JoinMode _mode;
  const std::pair<ColumnID, ColumnID> _column_ids;
  const PredicateCondition _predicate_condition;
  void _on_set_parameters(const ParameterMap&) override {}  // abstract_join_operator.cpp:45
};

class TableWrapper final : public AbstractReadOnlyOperator {
 public:
  explicit TableWrapper(std::shared_ptr<const Table> table)
      : AbstractReadOnlyOperator(OperatorType::TableWrapper), _table(std::move(table)) {}
  const std::string name() const override { return "TableWrapper"; }

 protected:
  std::shared_ptr<const Table> _on_execute() override { return _table; }
  void _on_set_parameters(const ParameterMap&) override {}
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>&,
                                                  const std::shared_ptr<AbstractOperator>&) const override {
    return std::make_shared<TableWrapper>(_table);  // table_wrapper.cpp:14-18
  }
  std::shared_ptr<const Table> _table;
};

class TableScan final : public AbstractReadOnlyOperator {
 public:
  // table_scan.cpp:32-37: the right side is a value, a column of the input (ColumnParameter) or a ParameterID
  // placeholder that set_parameters replaces by its value before execution.
  TableScan(std::shared_ptr<const AbstractOperator> in, ColumnID left_column_id, PredicateCondition predicate_condition,
            AllParameterVariant right_parameter)
      : AbstractReadOnlyOperator(OperatorType::TableScan, std::move(in)),
        _left_column_id(left_column_id),
        _predicate_condition(predicate_condition),
        _right_parameter(std::move(right_parameter)) {}

  const std::string name() const override { return "TableScan"; }
  const std::string description(DescriptionMode description_mode = DescriptionMode::SingleLine) const override;
  ColumnID left_column_id() const { return _left_column_id; }
  PredicateCondition predicate_condition() const { return _predicate_condition; }
  const AllParameterVariant& right_parameter() const { return _right_parameter; }
  void set_excluded_chunk_ids(const std::vector<ChunkID>& ids) { _excluded_chunk_ids = ids; }

 protected:
  std::shared_ptr<const Table> _on_execute() override;
  void _on_set_parameters(const ParameterMap& parameters) override;
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                  const std::shared_ptr<AbstractOperator>&) const override;

 private:
  ColumnID _left_column_id;
  PredicateCondition _predicate_condition;
  AllParameterVariant _right_parameter;
  std::vector<ChunkID> _excluded_chunk_ids;
};

// Validate (reference operators/validate.cpp:36-95): the input rows visible to one transaction. The reference's
// TransactionContext enters as its two fields, the transaction id and the snapshot commit id.
// validate.hpp:18-36: Validate(in), visibility from the operator's TransactionContext (set_transaction_context, as the
// SQL pipeline does for every operator); without one, _on_execute() fails like the reference's (validate.cpp:45-47).
class Validate final : public AbstractReadOnlyOperator {
 public:
  explicit Validate(std::shared_ptr<const AbstractOperator> in)
      : AbstractReadOnlyOperator(OperatorType::Validate, std::move(in)) {}
  const std::string name() const override { return "Validate"; }

 protected:
  std::shared_ptr<const Table> _on_execute(std::shared_ptr<TransactionContext> transaction_context) override;
  std::shared_ptr<const Table> _on_execute() override;
  void _on_set_parameters(const ParameterMap&) override {}  // validate.cpp:44
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                  const std::shared_ptr<AbstractOperator>&) const override {
    return std::make_shared<Validate>(copied_input_left);  // validate.cpp:38-42
  }
};

// join_hash.hpp:24-30: JoinHash : AbstractJoinOperator
class JoinHash final : public AbstractJoinOperator {
 public:
  JoinHash(std::shared_ptr<const AbstractOperator> left, std::shared_ptr<const AbstractOperator> right, JoinMode mode,
           std::pair<ColumnID, ColumnID> column_ids, PredicateCondition predicate_condition, size_t radix_bits = 9)
      : AbstractJoinOperator(OperatorType::JoinHash, std::move(left), std::move(right), mode, column_ids,
                             predicate_condition),
        _radix_bits(radix_bits) {
    Assert(predicate_condition == PredicateCondition::Equals, "Operator not supported by Hash Join.");
  }
  const std::string name() const override { return "JoinHash"; }
  // radix bits actually used by the last execution (the constructor argument is ignored, as in the reference)
  uint32_t used_radix_bits() const { return _used_radix_bits; }

 protected:
  std::shared_ptr<const Table> _on_execute() override;
  // join_hash.cpp:41-45: the copy gets the default radix_bits (the argument is ignored by execution anyway)
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                  const std::shared_ptr<AbstractOperator>& copied_input_right) const override {
    return std::make_shared<JoinHash>(copied_input_left, copied_input_right, _mode, _column_ids, _predicate_condition);
  }

 private:
  size_t _radix_bits;
  uint32_t _used_radix_bits = 0;
};

struct AggregateColumnDefinition {
  AggregateColumnDefinition(std::optional<ColumnID> c, AggregateFunction f) : column(c), function(f) {}
  std::optional<ColumnID> column;
  AggregateFunction function;
};

class Aggregate final : public AbstractReadOnlyOperator {
 public:
  Aggregate(std::shared_ptr<const AbstractOperator> in, std::vector<AggregateColumnDefinition> aggregates,
            std::vector<ColumnID> groupby_column_ids)
      : AbstractReadOnlyOperator(OperatorType::Aggregate, std::move(in)),
        _aggregates(std::move(aggregates)),
        _groupby_column_ids(std::move(groupby_column_ids)) {
    Assert(!(_aggregates.empty() && _groupby_column_ids.empty()),
           "Neither aggregate nor groupby columns have been specified");
  }
  const std::string name() const override { return "Aggregate"; }
  const std::vector<AggregateColumnDefinition>& aggregates() const { return _aggregates; }
  const std::vector<ColumnID>& groupby_column_ids() const { return _groupby_column_ids; }
  // device path of the last execution: true = dense (code-indexed LDS records), false = hash table in HBM
  bool used_dense_path() const { return _used_dense_path; }

 protected:
  std::shared_ptr<const Table> _on_execute() override;
  void _on_set_parameters(const ParameterMap&) override {}  // aggregate.cpp:78
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                  const std::shared_ptr<AbstractOperator>&) const override {
    return std::make_shared<Aggregate>(copied_input_left, _aggregates, _groupby_column_ids);  // aggregate.cpp:70-74
  }

 private:
  std::vector<AggregateColumnDefinition> _aggregates;
  std::vector<ColumnID> _groupby_column_ids;
  bool _used_dense_path = false;
};

// Projection(in, expressions): reference src/lib/operators/projection.hpp:20-50, projection.cpp:39-87. One output
// column per expression; PQPColumn expressions forward the input column when the output table type equals the
// input's (a projection of columns only keeps the input's type; anything computed makes a Data table). Arithmetic
// expressions are evaluated on the device (hy_projection), one launch per expression over all chunks.
class Projection final : public AbstractReadOnlyOperator {
 public:
  Projection(std::shared_ptr<const AbstractOperator> in, std::vector<std::shared_ptr<AbstractExpression>> expressions)
      : AbstractReadOnlyOperator(OperatorType::Projection, std::move(in)), expressions(std::move(expressions)) {}
  const std::string name() const override { return "Projection"; }

  const std::vector<std::shared_ptr<AbstractExpression>> expressions;

 protected:
  std::shared_ptr<const Table> _on_execute() override;
  // projection.cpp:25-33: placeholders in the expressions get their values; a copy deep-copies the expressions
  void _on_set_parameters(const ParameterMap& parameters) override;
  std::shared_ptr<AbstractOperator> _on_deep_copy(const std::shared_ptr<AbstractOperator>& copied_input_left,
                                                  const std::shared_ptr<AbstractOperator>&) const override;
};

// Operator phase timings (host wall time): recorded while enabled, taken (and cleared) by op_trace_take.
struct OpTraceRecord {
  std::string op, phase;
  double ms;
};
void op_trace_enable(bool on);
std::vector<OpTraceRecord> op_trace_take();

// JoinHash's prepared-plan cache (operators.cpp, JoinPlanCache): {hits, misses} since the start, and freeing the
// cached plans (their workspaces).
std::pair<uint64_t, uint64_t> join_plan_cache_stats();
void join_plan_cache_clear();
// plans kept (HY_OP_PLAN_CACHE at start, default 0 = off)
void join_plan_cache_set_capacity(size_t plans);

// JoinHashTraits (reference src/lib/operators/join_hash/hash_traits.hpp:9-42) over data types.
DataType join_hashed_type(DataType left, DataType right);

// Binary table files (reference ImportBinary / ExportBinary, import_binary.cpp / export_binary.cpp): chunks keep their
// stored encoding; load_to_device creates every numeric column chunk's HBM mirror (the file's bytes).
std::shared_ptr<Table> import_binary(const std::string& filename);
void export_binary(const std::shared_ptr<const Table>& table, const std::string& filename);
void load_to_device(const std::shared_ptr<const Table>& table);

}  // namespace hyrise
