"""TPC-H 1 (all eight aggregates), 3 and 6 (revenue) as operator chains on the dbgen SF0.01 fixture.

The chains follow the query texts (reference src/benchmarklib/tpch/tpch_queries.cpp:36-44 Q1, :101-106 Q3,
:206-210 Q6) the way the reference plans them: TableScans over the base tables, JoinHash on the key equalities,
a Projection computing the arithmetic (projection.cpp:39-87), then the Aggregate. The CPU tests pin the oracle's
chain to the SQLite known answers (tests/golden/tpch_sf0.01_answers.json, made by make_tpch_fixture.py); the GPU
tests run the device operators and compare every stage with the oracle: scans, joins and projections bit-exact,
group keys and counts exact, and float SUM/AVG equal to the exactly rounded sum of the group's values (math.fsum),
with the ULP distance to the oracle's sequential sum (aggregate.cpp:168-179) bounded and reported.
"""
import math

import numpy as np
import pytest

import agg_cases as ac
import tpch_fixture as tf
from helpers import assert_identical, wrap

Q3_DATE = "1995-03-15"


def exprs(hy):
    return hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator, hy.ValueExpression


def disc_price(hy, t, price, disc):
    P, A, O, V = exprs(hy)
    return A(O.Multiplication, P(t, price), A(O.Subtraction, V(1), P(t, disc)))


def q1_projection(hy, t):
    """SELECT list inputs of Q1 over the lineitem scan: flags, quantity, price, disc_price, charge, discount."""
    P, A, O, V = exprs(hy)
    dp = disc_price(hy, t, 2, 3)
    return [P(t, 5), P(t, 6), P(t, 1), P(t, 2), dp, A(O.Multiplication, dp, A(O.Addition, V(1), P(t, 4))), P(t, 3)]


Q1_AGGS = [(2, "Sum"), (3, "Sum"), (4, "Sum"), (5, "Sum"), (2, "Avg"), (3, "Avg"), (6, "Avg"), (None, "Count")]
# Q3 join chain: (customer scan) ⋈ c_custkey = o_custkey (orders scan) ⋈ o_orderkey = l_orderkey (lineitem scan);
# the join output holds customer (0-1), orders (2-5) and lineitem (6-13) columns
Q3_J1 = (0, 1)
Q3_J2 = (2, 0)


def q3_projection(hy, t):
    P = hy.PQPColumnExpression.from_table
    return [P(t, 6), P(t, 4), P(t, 5), disc_price(hy, t, 8, 9)]


def q6_projection(hy, t):
    P, A, O, V = exprs(hy)
    return [A(O.Multiplication, P(t, 2), P(t, 3))]


def oracle_scan(hy, oracle, t, col, cond, value):
    return oracle.table_scan(t, col, getattr(hy.PredicateCondition, cond), value, [])


def oracle_q1(hy, oracle, lineitem):
    s = oracle_scan(hy, oracle, lineitem, 7, "LessThanEquals", "1998-12-01")
    p = oracle.projection(s, q1_projection(hy, s))
    return p, oracle.aggregate(p, ac.agg_defs(hy, Q1_AGGS), [0, 1])


def oracle_q3(hy, oracle, customer, orders, lineitem):
    c = oracle_scan(hy, oracle, customer, 1, "Equals", "BUILDING")
    o = oracle_scan(hy, oracle, orders, 2, "LessThan", Q3_DATE)
    l = oracle_scan(hy, oracle, lineitem, 7, "GreaterThan", Q3_DATE)
    j1, _ = oracle.join_hash(c, o, hy.JoinMode.Inner, Q3_J1)
    j2, _ = oracle.join_hash(j1, l, hy.JoinMode.Inner, Q3_J2)
    p = oracle.projection(j2, q3_projection(hy, j2))
    return [c, o, l, j1, j2, p], oracle.aggregate(p, ac.agg_defs(hy, [(3, "Sum")]), [0, 1, 2])


def oracle_q6(hy, oracle, lineitem):
    t = lineitem
    for col, cond, val in tf.Q6_SCANS:
        t = oracle_scan(hy, oracle, t, col, cond, val)
    p = oracle.projection(t, q6_projection(hy, t))
    return t, p, oracle.aggregate(p, ac.agg_defs(hy, [(0, "Sum")]), [])


def q3_sorted(rows):
    """Q3's ORDER BY revenue DESC, o_orderdate, l_orderkey."""
    return sorted(rows, key=lambda r: (-r[3], r[1], r[0]))


def test_oracle_q1_full_known_answer(hy, oracle):
    orders, lineitem = tf.tables(hy)
    _, agg = oracle_q1(hy, oracle, lineitem)
    got, want = sorted(agg.rows()), tf.answers()["q1_full"]
    assert [(r[0], r[1], r[9]) for r in got] == [(w[0], w[1], w[9]) for w in want]
    for r, w in zip(got, want):
        assert r[2] == w[2]  # SUM(l_quantity): integer-valued, exact
        assert math.isclose(r[3], w[3], rel_tol=1e-12)  # SUM(l_extendedprice): both sum the float inputs in double
        # disc_price / charge: Hyrise multiplies in float (the columns' common type), SQLite in double
        assert math.isclose(r[4], w[4], rel_tol=1e-7) and math.isclose(r[5], w[5], rel_tol=1e-7)
        for k in (6, 7, 8):
            assert math.isclose(r[k], w[k], rel_tol=1e-12)


def test_oracle_q3_known_answer(hy, oracle):
    orders, lineitem = tf.tables(hy)
    customer = tf.customer_table(hy)
    assert customer.row_count() == tf.answers()["customer_rows"]
    _, agg = oracle_q3(hy, oracle, customer, orders, lineitem)
    got, want = q3_sorted(agg.rows()), tf.answers()["q3"]
    assert len(got) == len(want)
    assert sorted((r[0], r[1], r[2]) for r in got) == sorted((w[0], w[2], w[3]) for w in want)
    by_key = {(w[0], w[2], w[3]): w[1] for w in want}
    for r in got:
        assert math.isclose(r[3], by_key[(r[0], r[1], r[2])], rel_tol=1e-6)


def test_oracle_q6_revenue(hy, oracle):
    orders, lineitem = tf.tables(hy)
    t, _, agg = oracle_q6(hy, oracle, lineitem)
    ans = tf.answers()
    assert t.row_count() == ans["q6_rows"]
    # l_extendedprice * l_discount is a float product in Hyrise, a double product in SQLite
    assert math.isclose(agg.rows()[0][0], ans["q6_revenue"], rel_tol=1e-7)


def ulps(a, b):
    ia, ib = (int(np.array(x, np.float64).view(np.int64)) for x in (a, b))
    return abs(ia - ib)


def check_float_aggregates(got, want, proj_rows, keys, aggs, n_group_cols, report):
    """Device float SUM/AVG == exactly rounded result over the group's projected values; ULPs to the oracle."""
    groups = {}
    for r in proj_rows:
        groups.setdefault(tuple(r[k] for k in keys), []).append(r)
    got, want = sorted(got, key=repr), sorted(want, key=repr)
    assert len(got) == len(want)
    worst = 0
    for g, w in zip(got, want):
        members = groups[tuple(g[:n_group_cols])]
        for j, (col, fn) in enumerate(aggs):
            out = n_group_cols + j
            if col is None or fn not in ("Sum", "Avg"):
                assert g[out] == w[out]
                continue
            vals = [r[col] for r in members if r[col] is not None]
            exact = math.fsum(vals)
            expect = exact if fn == "Sum" else exact / len(vals)
            if all(float(v).is_integer() for v in vals):
                assert g[out] == w[out]  # integer-valued inputs: the sequential sum is exact too
            assert g[out] == expect, (g, fn, col)
            worst = max(worst, ulps(g[out], w[out]))
    report.append(worst)
    return worst


@pytest.mark.gpu
def test_device_q1_full(hy, oracle):
    orders, lineitem = tf.tables(hy)
    exp_proj, exp = oracle_q1(hy, oracle, lineitem)
    s = hy.TableScan(wrap(hy, lineitem), 7, hy.PredicateCondition.LessThanEquals, "1998-12-01")
    s.execute()
    p = hy.Projection(s, q1_projection(hy, s.get_output()))
    p.execute()
    assert_identical(p.get_output(), exp_proj)
    a = hy.Aggregate(p, ac.agg_defs(hy, Q1_AGGS), [0, 1])
    a.execute()
    report = []
    worst = check_float_aggregates(a.get_output().rows(), exp.rows(), exp_proj.rows(), [0, 1], Q1_AGGS, 2, report)
    print(f"Q1 SF0.01: worst ULP distance device vs sequential oracle sum = {worst}")
    assert worst <= 1  # the north star's bar (BASELINE.json); measured: 0


@pytest.mark.gpu
def test_device_q3(hy, oracle):
    orders, lineitem = tf.tables(hy)
    customer = tf.customer_table(hy)
    stages, exp = oracle_q3(hy, oracle, customer, orders, lineitem)
    c = hy.TableScan(wrap(hy, customer), 1, hy.PredicateCondition.Equals, "BUILDING")
    o = hy.TableScan(wrap(hy, orders), 2, hy.PredicateCondition.LessThan, Q3_DATE)
    l = hy.TableScan(wrap(hy, lineitem), 7, hy.PredicateCondition.GreaterThan, Q3_DATE)
    j1 = hy.JoinHash(c, o, hy.JoinMode.Inner, Q3_J1, hy.PredicateCondition.Equals)
    j2 = hy.JoinHash(j1, l, hy.JoinMode.Inner, Q3_J2, hy.PredicateCondition.Equals)
    ops = [c, o, l, j1, j2]
    for op in ops:
        op.execute()
    p = hy.Projection(j2, q3_projection(hy, j2.get_output()))
    p.execute()
    ops.append(p)
    for op, e in zip(ops, stages):
        assert_identical(op.get_output(), e)
    a = hy.Aggregate(p, ac.agg_defs(hy, [(3, "Sum")]), [0, 1, 2])
    a.execute()
    report = []
    worst = check_float_aggregates(a.get_output().rows(), exp.rows(), stages[-1].rows(), [0, 1, 2], [(3, "Sum")], 3,
                                   report)
    print(f"Q3 SF0.01: worst ULP distance device vs sequential oracle sum = {worst}")
    assert worst <= 1  # the north star's bar (BASELINE.json); measured: 0
    want = {(w[0], w[2], w[3]): w[1] for w in tf.answers()["q3"]}
    got = a.get_output().rows()
    assert sorted((r[0], r[1], r[2]) for r in got) == sorted(want)
    assert all(math.isclose(r[3], want[(r[0], r[1], r[2])], rel_tol=1e-6) for r in got)


@pytest.mark.gpu
def test_device_q6_revenue(hy, oracle):
    orders, lineitem = tf.tables(hy)
    exp_scan, exp_proj, exp = oracle_q6(hy, oracle, lineitem)
    op = wrap(hy, lineitem)
    for col, cond, val in tf.Q6_SCANS:
        op = hy.TableScan(op, col, getattr(hy.PredicateCondition, cond), val)
        op.execute()
    p = hy.Projection(op, q6_projection(hy, op.get_output()))
    p.execute()
    assert_identical(p.get_output(), exp_proj)
    a = hy.Aggregate(p, ac.agg_defs(hy, [(0, "Sum")]), [])
    a.execute()
    got = a.get_output().rows()[0][0]
    assert got == math.fsum(r[0] for r in exp_proj.rows())
    print(f"Q6 SF0.01: ULP distance device vs sequential oracle sum = {ulps(got, exp.rows()[0][0])}")
    assert ulps(got, exp.rows()[0][0]) <= 1  # the north star's bar (BASELINE.json); measured: 0
