"""Projection host logic and the oracle's restatement, without a GPU: expression data types / nullability / column
names as the reference computes them (expression_utils.cpp:116-136, arithmetic_expression.cpp:45-62,
abstract_expression.cpp:46-56), the oracle against the reference's Projection fixture
(projection_test.cpp:50-54, tables/projection/int_float_add.tbl), and the oracle's arithmetic against numpy's IEEE /
C semantics for every operator and operand type pair."""
import numpy as np
import pytest

from helpers import assert_table_eq_unordered, tbl, wrap


def E(hy):
    return hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator, hy.ValueExpression


def test_types_names_nullability(hy):
    P, A, O, V = E(hy)
    t = hy.Table.from_arrays([("i", hy.DataType.Int, False), ("l", hy.DataType.Long, False),
                              ("f", hy.DataType.Float, True), ("d", hy.DataType.Double, False)],
                             [np.zeros(2, np.int32), np.zeros(2, np.int64), np.zeros(2, np.float32), np.zeros(2)],
                             [None, None, np.zeros(2, np.uint8), None], 2)
    i, l, f, d = (P(t, c) for c in range(4))
    DT = hy.DataType
    cases = [(A(O.Addition, i, i), DT.Int), (A(O.Addition, i, l), DT.Long), (A(O.Multiplication, i, f), DT.Float),
             (A(O.Multiplication, l, f), DT.Double), (A(O.Subtraction, f, d), DT.Double),
             (A(O.Division, i, V(2)), DT.Int), (A(O.Modulo, l, V(3)), DT.Long)]
    for e, want in cases:
        assert e.data_type() == want, e.as_column_name()
    assert not A(O.Addition, i, l).is_nullable() and A(O.Addition, i, f).is_nullable()
    assert A(O.Division, i, l).is_nullable() and A(O.Modulo, i, l).is_nullable()
    q1 = A(O.Multiplication, A(O.Multiplication, d, A(O.Subtraction, V(1), f)), A(O.Addition, V(1), d))
    assert q1.as_column_name() == "(d * (1 - f)) * (1 + d)"
    assert A(O.Subtraction, A(O.Subtraction, i, l), i).as_column_name() == "(i - l) - i"
    assert A(O.Multiplication, A(O.Addition, i, l), i).as_column_name() == "(i + l) * i"
    assert A(O.Addition, A(O.Multiplication, i, l), i).as_column_name() == "i * l + i"


def test_oracle_matches_reference_fixture(hy, oracle):
    P, A, O, V = E(hy)
    t = hy.load_table(tbl("int_float.tbl"), 2)
    out = oracle.projection(t, [A(O.Addition, P(t, 0), P(t, 1))])
    assert_table_eq_unordered(out, hy.load_table(tbl("projection/int_float_add.tbl")))
    # ForwardsIfPossibleDataTable: a projection of columns only forwards the input columns
    fwd = oracle.projection(t, [P(t, 1), P(t, 0)])
    assert fwd.type() == hy.TableType.Data and fwd.column_names() == ["b", "a"]


NP = {"Int": np.int32, "Long": np.int64, "Float": np.float32, "Double": np.float64}


def np_common(a, b):
    # C++ std::common_type of the operands (int32 < int64 < float < double)
    order = ["Int", "Long", "Float", "Double"]
    return order[max(order.index(a), order.index(b))]


@pytest.mark.parametrize("op", ["Addition", "Subtraction", "Multiplication", "Division", "Modulo"])
@pytest.mark.parametrize("ta,tb", [("Int", "Int"), ("Int", "Long"), ("Long", "Float"), ("Float", "Float"),
                                   ("Int", "Double"), ("Float", "Double")])
def test_oracle_arithmetic_matches_numpy(hy, oracle, op, ta, tb):
    P, A, O, V = E(hy)
    rng = np.random.default_rng(7)
    n = 500
    a = rng.integers(-1000, 1000, n).astype(NP[ta]) if ta in ("Int", "Long") else (rng.random(n) * 200 - 100).astype(NP[ta])
    b = rng.integers(-9, 9, n).astype(NP[tb]) if tb in ("Int", "Long") else np.round(rng.random(n) * 20 - 10, 1).astype(NP[tb])
    b[::17] = 0  # division / modulo by zero -> NULL
    na = (rng.random(n) < 0.1).astype(np.uint8)
    t = hy.Table.from_arrays([("a", getattr(hy.DataType, ta), True), ("b", getattr(hy.DataType, tb), False)], [a, b],
                             [na, None], 128)
    e = A(getattr(O, op), P(t, 0), P(t, 1))
    out = oracle.projection(t, [e])
    got = np.array([v if v is not None else np.nan for v in sum((out.get_chunk(c).get_column(0).values()
                                                                    for c in range(out.chunk_count())), [])], dtype=float)
    C = NP[np_common(ta, tb)]
    x, y = a.astype(C), b.astype(C)
    with np.errstate(all="ignore"):
        if op == "Addition":
            r = x + y
        elif op == "Subtraction":
            r = x - y
        elif op == "Multiplication":
            r = x * y
        elif op == "Division":
            r = (np.trunc(x / np.where(y == 0, 1, y)).astype(C) if np.issubdtype(C, np.integer)
                 else x / np.where(y == 0, 1, y))
        else:
            r = np.fmod(x, np.where(y == 0, 1, y))
    want = r.astype(NP[e.data_type().name]).astype(float)
    null = (na == 1) | ((y == 0) & (op in ("Division", "Modulo")))
    want[null] = np.nan
    assert np.array_equal(got, want, equal_nan=True)
