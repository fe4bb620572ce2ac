// Expressions of the Projection operator: the reference's PQPColumnExpression, ValueExpression and
// ArithmeticExpression (src/lib/expression/pqp_column_expression.hpp, value_expression.hpp,
// arithmetic_expression.hpp) with the properties the Projection's output relies on: data type
// (expression_common_type, expression/expression_utils.cpp:116-136), nullability (abstract_expression.cpp:20-23,
// arithmetic_expression.cpp:58-62) and column name (as_column_name with precedence-based parentheses,
// abstract_expression.cpp:46-56, arithmetic_expression.cpp:50-56).
#pragma once

#include <memory>
#include <optional>
#include <sstream>
#include <string>
#include <unordered_map>
#include <variant>
#include <vector>

#include "storage.hpp"

namespace hyrise {

// ParameterID: reference expression/parameter_expression.hpp:14 (STRONG_TYPEDEF(size_t, ParameterID)).
struct ParameterID {
  size_t t;
  bool operator==(const ParameterID& o) const { return t == o.t; }
  bool operator!=(const ParameterID& o) const { return t != o.t; }
};
struct ParameterIDHash {
  size_t operator()(const ParameterID& p) const { return std::hash<size_t>{}(p.t); }
};

// The ColumnID alternative of the reference's AllParameterVariant (all_parameter_variant.hpp:21-26): TableScan
// compares two columns of its input (ColumnComparisonTableScanImpl, table_scan.cpp:191-199). A struct, because this
// layer's ColumnID is a plain integer and would be ambiguous with an int value.
struct ColumnParameter {
  ColumnID column_id;
  bool operator==(const ColumnParameter& o) const { return column_id == o.column_id; }
};

// AllParameterVariant (all_parameter_variant.hpp:21-33) without the LQP's column reference, which only the optimizer
// builds: a value, a column of the input, or a placeholder for a prepared statement's parameter.
using AllParameterVariant = std::variant<AllTypeVariant, ColumnParameter, ParameterID>;
inline bool is_variant(const AllParameterVariant& v) { return v.index() == 0; }
inline bool is_column_id(const AllParameterVariant& v) { return v.index() == 1; }
inline bool is_parameter_id(const AllParameterVariant& v) { return v.index() == 2; }

enum class ExpressionType { PQPColumn, Value, Arithmetic, Parameter };
enum class ArithmeticOperator { Addition, Subtraction, Multiplication, Division, Modulo };

// reference expression_precedence.hpp:8-15 (lower binds tighter; 0 for leaves)
enum class ExpressionPrecedence : uint32_t {
  Highest = 0,
  UnaryPredicate,
  MultiplicationDivision,
  AdditionSubtraction,
  BinaryTernaryPredicate,
  Logical
};

class AbstractExpression {
 public:
  AbstractExpression(ExpressionType type, std::vector<std::shared_ptr<AbstractExpression>> arguments)
      : type(type), arguments(std::move(arguments)) {}
  virtual ~AbstractExpression() = default;

  virtual DataType data_type() const = 0;
  virtual bool is_nullable() const {
    for (const auto& a : arguments)
      if (a->is_nullable()) return true;
    return false;
  }
  virtual std::string as_column_name() const = 0;
  // abstract_expression.hpp: a copy of the whole tree
  virtual std::shared_ptr<AbstractExpression> deep_copy() const = 0;

  const ExpressionType type;
  const std::vector<std::shared_ptr<AbstractExpression>> arguments;

 protected:
  virtual ExpressionPrecedence precedence() const { return ExpressionPrecedence::Highest; }
  std::string enclose_argument_as_column_name(const AbstractExpression& argument) const {
    if (static_cast<uint32_t>(argument.precedence()) >= static_cast<uint32_t>(precedence()))
      return "(" + argument.as_column_name() + ")";
    return argument.as_column_name();
  }
};

// A column of the operator's input table (reference pqp_column_expression.hpp:12-41).
class PQPColumnExpression final : public AbstractExpression {
 public:
  PQPColumnExpression(ColumnID column_id, DataType data_type, bool nullable, std::string column_name)
      : AbstractExpression(ExpressionType::PQPColumn, {}),
        column_id(column_id),
        _data_type(data_type),
        _nullable(nullable),
        _column_name(std::move(column_name)) {}
  static std::shared_ptr<PQPColumnExpression> from_table(const Table& table, ColumnID column_id);

  DataType data_type() const override { return _data_type; }
  bool is_nullable() const override { return _nullable; }
  std::string as_column_name() const override { return _column_name; }
  std::shared_ptr<AbstractExpression> deep_copy() const override {
    return std::make_shared<PQPColumnExpression>(column_id, _data_type, _nullable, _column_name);
  }

  const ColumnID column_id;

 private:
  const DataType _data_type;
  const bool _nullable;
  const std::string _column_name;
};

// A literal (reference value_expression.cpp:19-39).
class ValueExpression final : public AbstractExpression {
 public:
  explicit ValueExpression(AllTypeVariant value) : AbstractExpression(ExpressionType::Value, {}), value(std::move(value)) {}

  DataType data_type() const override;
  bool is_nullable() const override { return variant_is_null(value); }
  std::string as_column_name() const override;
  std::shared_ptr<AbstractExpression> deep_copy() const override { return std::make_shared<ValueExpression>(value); }

  const AllTypeVariant value;
};

// A value placeholder of a prepared statement (reference parameter_expression.hpp:24-70, ValuePlaceholder kind):
// no type until set_parameters gives it a value; evaluated like a literal of that value.
class ParameterExpression final : public AbstractExpression {
 public:
  explicit ParameterExpression(ParameterID parameter_id)
      : AbstractExpression(ExpressionType::Parameter, {}), parameter_id(parameter_id) {}

  // parameter_expression.cpp:60-76: type and nullability of an unset placeholder are an error
  DataType data_type() const override;
  bool is_nullable() const override;
  std::string as_column_name() const override;  // parameter_expression.cpp:41-56
  // parameter_expression.cpp:31-37: the copy is an unset placeholder of the same id (a plan cache copies the
  // prepared plan, then sets the execution's parameters in the copy)
  std::shared_ptr<AbstractExpression> deep_copy() const override {
    return std::make_shared<ParameterExpression>(parameter_id);
  }
  const std::optional<AllTypeVariant>& value() const { return _value; }
  void set_value(const std::optional<AllTypeVariant>& value) { _value = value; }

  const ParameterID parameter_id;

 private:
  std::optional<AllTypeVariant> _value;
};

class ArithmeticExpression final : public AbstractExpression {
 public:
  ArithmeticExpression(ArithmeticOperator op, std::shared_ptr<AbstractExpression> left,
                       std::shared_ptr<AbstractExpression> right)
      : AbstractExpression(ExpressionType::Arithmetic, {std::move(left), std::move(right)}), arithmetic_operator(op) {}

  const std::shared_ptr<AbstractExpression>& left_operand() const { return arguments[0]; }
  const std::shared_ptr<AbstractExpression>& right_operand() const { return arguments[1]; }

  DataType data_type() const override;
  // division / modulo by 0 yield NULL (arithmetic_expression.cpp:58-62)
  bool is_nullable() const override {
    return AbstractExpression::is_nullable() || arithmetic_operator == ArithmeticOperator::Division ||
           arithmetic_operator == ArithmeticOperator::Modulo;
  }
  std::string as_column_name() const override;
  std::shared_ptr<AbstractExpression> deep_copy() const override {
    return std::make_shared<ArithmeticExpression>(arithmetic_operator, left_operand()->deep_copy(),
                                                  right_operand()->deep_copy());
  }

  const ArithmeticOperator arithmetic_operator;

 protected:
  ExpressionPrecedence precedence() const override {
    return (arithmetic_operator == ArithmeticOperator::Addition ||
            arithmetic_operator == ArithmeticOperator::Subtraction)
               ? ExpressionPrecedence::AdditionSubtraction
               : ExpressionPrecedence::MultiplicationDivision;
  }
};

// reference expression_utils.cpp:116-136
DataType expression_common_type(DataType lhs, DataType rhs);
// The type std::common_type gives the C++ operands (the type an arithmetic functor computes in,
// expression_functors.hpp:121-123): int32 < int64 < float < double by the usual arithmetic conversions.
DataType cpp_common_type(DataType lhs, DataType rhs);
// data_type_from_all_type_variant (reference all_type_variant.hpp)
DataType data_type_of_variant(const AllTypeVariant& v);
std::string arithmetic_operator_to_string(ArithmeticOperator op);
// expression_utils.cpp:166-193: every placeholder of the trees whose id has a value gets that value
void expressions_set_parameters(const std::vector<std::shared_ptr<AbstractExpression>>& expressions,
                                const std::unordered_map<ParameterID, AllTypeVariant, ParameterIDHash>& parameters);
// expression_utils.cpp:49-57
std::vector<std::shared_ptr<AbstractExpression>> expressions_deep_copy(
    const std::vector<std::shared_ptr<AbstractExpression>>& expressions);

}  // namespace hyrise
