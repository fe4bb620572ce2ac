"""Device Projection (hy_projection behind the Projection operator) against the oracle's restatement of the
reference Projection / ExpressionEvaluator: identical output tables (schema, chunking, every value and NULL flag, bit
for bit) for every arithmetic operator and operand type pair, literals of each type and NULL, division / modulo by
zero, data and reference inputs (one and two PosList groups), dictionary-encoded inputs, and column forwarding
(reference projection_test.cpp:50-104)."""
import numpy as np
import pytest

from helpers import assert_identical, wrap

pytestmark = pytest.mark.gpu

NP = {"Int": np.int32, "Long": np.int64, "Float": np.float32, "Double": np.float64}


def table(hy, rng, n, chunk, types, nullable=True):
    arrays, nulls, defs = [], [], []
    for k, t in enumerate(types):
        if t in ("Int", "Long"):
            v = rng.integers(-5000, 5000, n).astype(NP[t])
        else:
            v = (rng.random(n) * 400 - 200).astype(NP[t])
        v[::23] = 0
        arrays.append(v)
        nulls.append((rng.random(n) < 0.05).astype(np.uint8) if nullable else None)
        defs.append((f"c{k}", getattr(hy.DataType, t), nullable))
    return hy.Table.from_arrays(defs, arrays, nulls, chunk)


def run(hy, oracle, src_op, src_table, exprs):
    p = hy.Projection(src_op, exprs)
    p.execute()
    assert_identical(p.get_output(), oracle.projection(src_table, exprs))
    return p


@pytest.mark.parametrize("op", ["Addition", "Subtraction", "Multiplication", "Division", "Modulo"])
def test_all_type_pairs(hy, oracle, op):
    rng = np.random.default_rng(len(op))
    types = ["Int", "Long", "Float", "Double"]
    t = table(hy, rng, 20_000, 7_000, types)
    P, A, O = hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator
    exprs = [A(getattr(O, op), P(t, i), P(t, j)) for i in range(4) for j in range(4)]
    run(hy, oracle, wrap(hy, t), t, exprs[:8])
    run(hy, oracle, wrap(hy, t), t, exprs[8:])


def test_literals_and_tpch_expressions(hy, oracle):
    rng = np.random.default_rng(3)
    t = table(hy, rng, 30_000, 10_000, ["Float", "Float", "Float", "Long", "Int"])
    P, A, O, V = (hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator,
                  hy.ValueExpression)
    price, disc, tax, lng, i = (P(t, c) for c in range(5))
    disc_price = A(O.Multiplication, price, A(O.Subtraction, V(1), disc))          # TPC-H 1 / 3
    charge = A(O.Multiplication, disc_price, A(O.Addition, V(1), tax))             # TPC-H 1
    exprs = [disc_price, charge, A(O.Multiplication, price, disc),                  # TPC-H 6
             A(O.Addition, i, V(7)), A(O.Multiplication, lng, V(0.5)), A(O.Subtraction, i, V(2**40)),
             A(O.Division, lng, V(3)), A(O.Modulo, i, V(7)), A(O.Addition, i, V(None)),
             A(O.Multiplication, lng, price), A(O.Division, V(1.0), A(O.Subtraction, price, price))]
    run(hy, oracle, wrap(hy, t), t, exprs)


def test_reference_inputs_and_forwarding(hy, oracle):
    rng = np.random.default_rng(9)
    t = table(hy, rng, 25_000, 6_000, ["Int", "Float", "Double"], nullable=False)
    hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
    P, A, O, V = (hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator,
                  hy.ValueExpression)
    w = wrap(hy, t)
    # forwarding: columns only keeps the input (data) columns themselves
    p = run(hy, oracle, w, t, [P(t, 1), P(t, 0)])
    assert p.get_output().type() == hy.TableType.Data
    # reference input (one PosList group): a TableScan's output
    s = hy.TableScan(w, 0, hy.PredicateCondition.GreaterThan, 0)
    s.execute()
    st = s.get_output()
    run(hy, oracle, s, st, [P(st, 2), A(O.Multiplication, P(st, 1), A(O.Subtraction, V(1), P(st, 2)))])
    fwd = run(hy, oracle, s, st, [P(st, 1), P(st, 0)])
    assert fwd.get_output().type() == hy.TableType.References
    # two PosList groups: a JoinHash output over two tables
    u = table(hy, rng, 9_000, 4_000, ["Int", "Double"], nullable=False)
    j = hy.JoinHash(w, wrap(hy, u), hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    jt = j.get_output()
    run(hy, oracle, j, jt, [A(O.Multiplication, P(jt, 1), P(jt, 4)), A(O.Addition, P(jt, 0), P(jt, 3))])
