"""The operator surface a Hyrise plan cache and prepared statements use, without a GPU: deep_copy / _on_deep_copy,
set_parameters / _on_set_parameters with ParameterID placeholders, set_transaction_context_recursively, and execute()
under an aborted transaction (reference abstract_operator.hpp:70-172, abstract_operator.cpp:25-173,
table_scan.cpp:63-78, join_hash.cpp:41-47, aggregate.cpp:70-78, projection.cpp:25-33, validate.cpp:38-44,
table_wrapper.cpp:14-20). Executing the compute needs the device (test_operator_surface_gpu.py)."""
import pytest

from helpers import tbl, wrap


def int_int(hy):
    t = hy.load_table(tbl("int_int_shuffled.tbl"), 7)
    hy.encode_chunks(t, [0, 1], hy.EncodingType.Dictionary)
    return wrap(hy, t)


def test_set_parameters(hy):
    """table_scan_test.cpp:632-655 (OperatorsTableScanTest.SetParameters)."""
    parameters = {3: 5, 2: 6}
    w = int_int(hy)
    ge = hy.PredicateCondition.GreaterThanEquals

    scan_a = hy.TableScan(w, 0, ge, 4)
    scan_a.set_parameters(parameters)
    assert scan_a.left_column_id() == 0
    assert scan_a.right_parameter() == 4

    scan_b = hy.TableScan(w, 0, ge, hy.ParameterID(2))
    scan_b.set_parameters(parameters)
    assert scan_b.left_column_id() == 0
    assert scan_b.right_parameter() == 6

    scan_c = hy.TableScan(w, 0, ge, hy.ParameterID(4))
    scan_c.set_parameters(parameters)
    assert scan_c.left_column_id() == 0
    assert scan_c.right_parameter() == hy.ParameterID(4)


def test_set_parameters_reaches_inputs(hy):
    """abstract_operator.cpp:147-151: the operator first, then both inputs, recursively."""
    w = int_int(hy)
    lt, ge = hy.PredicateCondition.LessThan, hy.PredicateCondition.GreaterThanEquals
    inner = hy.TableScan(w, 1, lt, hy.ParameterID(7))
    outer = hy.TableScan(inner, 0, ge, hy.ParameterID(8))
    join = hy.JoinHash(w, outer, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    join.set_parameters({7: 108, 8: ("float", 2.5)})
    assert inner.right_parameter() == 108
    assert outer.right_parameter() == 2.5
    # a value, a column or an unmatched placeholder is left as it is
    col = hy.TableScan(w, 0, lt, hy.ColumnParameter(1))
    col.set_parameters({1: 3})
    assert col.right_parameter() == hy.ColumnParameter(1)


def test_unset_parameter_fails_before_any_work(hy):
    w = int_int(hy)
    scan = hy.TableScan(w, 0, hy.PredicateCondition.Equals, hy.ParameterID(1))
    with pytest.raises(RuntimeError, match="parameter 1 has no value"):
        scan.execute()
    assert scan.get_output() is None


def test_deep_copy_keeps_configuration(hy):
    w = int_int(hy)
    lt = hy.PredicateCondition.LessThan
    scan = hy.TableScan(w, 1, lt, hy.ParameterID(3))
    join = hy.JoinHash(w, scan, hy.JoinMode.Semi, (0, 0), hy.PredicateCondition.Equals, 11)
    agg = hy.Aggregate(join, [hy.AggregateColumnDefinition(1, hy.AggregateFunction.Sum),
                              hy.AggregateColumnDefinition(None, hy.AggregateFunction.Count)], [0])
    copy = agg.deep_copy()
    assert copy is not agg and copy.name() == "Aggregate"
    assert [(d.column, d.function) for d in copy.aggregates()] == [(1, hy.AggregateFunction.Sum),
                                                                   (None, hy.AggregateFunction.Count)]
    assert copy.groupby_column_ids() == [0]
    cjoin = copy.input_left()
    assert cjoin is not join and cjoin.name() == "JoinHash"
    assert cjoin.mode() == hy.JoinMode.Semi and cjoin.column_ids() == (0, 0)
    assert cjoin.predicate_condition() == hy.PredicateCondition.Equals
    cscan = cjoin.input_right()
    assert cscan is not scan and cscan.name() == "TableScan"
    assert (cscan.left_column_id(), cscan.predicate_condition(), cscan.right_parameter()) == (1, lt, hy.ParameterID(3))
    # copies are unexecuted, except the TableWrapper's table, which it holds (table_wrapper.cpp:14-18)
    assert copy.get_output() is None and cjoin.get_output() is None and cscan.get_output() is None
    # parameters set in the copy leave the original's placeholder alone (a plan cache's prepared plan)
    copy.set_parameters({3: 100})
    assert cscan.right_parameter() == 100
    assert scan.right_parameter() == hy.ParameterID(3)


def test_deep_copy_of_a_diamond_copies_the_shared_input_once(hy):
    """abstract_operator.cpp:157-173: an input two operators share is copied once and shared by the copies."""
    w = int_int(hy)
    scan = hy.TableScan(w, 0, hy.PredicateCondition.GreaterThanEquals, 0)
    left = hy.TableScan(scan, 1, hy.PredicateCondition.LessThan, 200)
    right = hy.TableScan(scan, 1, hy.PredicateCondition.GreaterThanEquals, 200)
    join = hy.JoinHash(left, right, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    copy = join.deep_copy()
    cl, cr = copy.input_left(), copy.input_right()
    assert cl is not left and cr is not right
    assert cl.input_left() is cr.input_left()
    assert cl.input_left() is not scan
    assert cl.input_left().input_left() is cr.input_left().input_left()


def test_deep_copy_keeps_the_transaction_context(hy):
    w = int_int(hy)
    ctx = hy.TransactionContext(5, 3)
    v = hy.Validate(w)
    scan = hy.TableScan(v, 0, hy.PredicateCondition.Equals, 1)
    scan.set_transaction_context_recursively(ctx)
    assert v.transaction_context() is not None and w.transaction_context().transaction_id() == 5
    copy = scan.deep_copy()
    assert copy.transaction_context().transaction_id() == 5
    assert copy.input_left().name() == "Validate"
    assert copy.input_left().transaction_context().snapshot_commit_id() == 3


def test_projection_placeholders(hy):
    """projection.cpp:25-33: set_parameters fills the expressions' placeholders; deep_copy copies the expressions
    and a copied placeholder is unset again (parameter_expression.cpp:31-37)."""
    w = int_int(hy)
    t = w.get_output()
    a = hy.PQPColumnExpression.from_table(t, 0)
    p = hy.ParameterExpression(4)
    expr = hy.ArithmeticExpression(hy.ArithmeticOperator.Addition, a, p)
    proj = hy.Projection(w, [expr])
    with pytest.raises(RuntimeError, match="unset ValuePlaceholder"):
        p.data_type()
    proj.set_parameters({4: 10})
    assert p.has_value and p.value == 10
    assert p.as_column_name() == "Parameter[id=4]=10"
    assert expr.as_column_name() == "a + Parameter[id=4]=10"
    assert expr.data_type() == hy.DataType.Int
    copy = proj.deep_copy()
    cp = copy.expressions[0].right_operand()
    assert cp is not p and cp.parameter_id == 4 and not cp.has_value
    copy.set_parameters({4: ("float", 1.5)})
    assert cp.value == 1.5 and p.value == 10
    assert copy.expressions[0].data_type() == hy.DataType.Float


def test_aborted_transaction_leaves_output_unset(hy):
    """abstract_operator.cpp:32-41: an operator of an aborted transaction does not run and its output stays unset;
    a join over it therefore cannot execute either."""
    w = int_int(hy)
    ctx = hy.TransactionContext(1, 1)
    ctx.set_aborted()
    scan = hy.TableScan(w, 0, hy.PredicateCondition.Equals, 1)
    join = hy.JoinHash(w, w, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    agg = hy.Aggregate(w, [hy.AggregateColumnDefinition(None, hy.AggregateFunction.Count)], [])
    for op in (scan, join, agg):
        op.set_transaction_context(ctx)
        op.execute()
        assert op.get_output() is None
        assert op.performance_data().walltime_ns == 0
    downstream = hy.TableScan(scan, 0, hy.PredicateCondition.Equals, 1)
    with pytest.raises(RuntimeError, match="Left input has not been executed"):
        downstream.execute()


def test_descriptions_and_layering(hy):
    """description(DescriptionMode) of TableScan (table_scan.cpp:51-61) and of every join (AbstractJoinOperator,
    abstract_join_operator.cpp:30-43): executed inputs lend their column names (else "Col #i"), the predicate and the
    parameter follow; MultiLine breaks after the name. JoinHash keeps AbstractJoinOperator's mode / column ids /
    predicate accessors (join_hash.hpp:24, abstract_join_operator.hpp:34-37)."""
    w = int_int(hy)
    a, b = w.get_output().column_names()
    lt, ge, eq = hy.PredicateCondition.LessThan, hy.PredicateCondition.GreaterThanEquals, hy.PredicateCondition.Equals
    scan = hy.TableScan(w, 1, lt, 24)
    assert scan.description() == f"TableScan ({b} < 24)"
    assert scan.description(hy.DescriptionMode.MultiLine) == f"TableScan\n({b} < 24)"
    assert hy.TableScan(w, 0, ge, hy.ParameterID(3)).description() == f"TableScan ({a} >= Placeholder #3)"
    assert hy.TableScan(w, 0, lt, hy.ColumnParameter(1)).description() == f"TableScan ({a} < Col #1)"
    assert hy.TableScan(w, 0, lt, ("float", 2.5)).description() == f"TableScan ({a} < 2.5)"
    join = hy.JoinHash(w, scan, hy.JoinMode.Inner, (0, 1), eq)  # the scan has not run: its column by index
    assert join.description() == f"JoinHash (Inner Join where {a} = Col #1)"
    assert join.description(hy.DescriptionMode.MultiLine) == f"JoinHash\n(Inner Join where {a} = Col #1)"
    assert hy.JoinHash(w, w, hy.JoinMode.Semi, (1, 0), eq).description() == f"JoinHash (Semi Join where {b} = {a})"
    assert join.mode() == hy.JoinMode.Inner and join.column_ids() == (0, 1) and join.predicate_condition() == eq
    with pytest.raises(Exception):
        hy.JoinHash(w, w, hy.JoinMode.Cross, (0, 0), eq)  # abstract_join_operator.cpp:16-17
