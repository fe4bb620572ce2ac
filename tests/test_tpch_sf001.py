"""TPC-H SF0.01 plumbing (BASELINE.json configs[0]) on dbgen data: the oracle reproduces the SQLite known answers
(tests/golden/tpch_sf0.01_answers.json) for the hot-path shapes — TableScan l_quantity < 24, JoinHash
lineitem ⋈ orders, the TPC-H 6 scan chain and the TPC-H 1 aggregate — and the device operators reproduce the
oracle's outputs bit-for-bit on the same tables."""
import math

import numpy as np
import pytest

import agg_cases as ac
import tpch_fixture as tf
from helpers import assert_identical, wrap


def q6_revenue(table, arrays):
    rows = table.rows()
    # Hyrise evaluates l_extendedprice * l_discount on float columns; SQLite on their double widening
    return math.fsum(float(r[2]) * float(r[3]) for r in rows)


def test_oracle_tpch_known_answers(hy, oracle):
    ans = tf.answers()
    orders, lineitem = tf.tables(hy)
    assert lineitem.row_count() == ans["lineitem_rows"] and orders.row_count() == ans["orders_rows"]
    scan = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, [])
    assert scan.row_count() == ans["scan_l_quantity_lt_24"]
    join, bits = oracle.join_hash(orders, lineitem, hy.JoinMode.Inner, (0, 0))
    assert join.row_count() == ans["join_lineitem_orders_rows"]
    assert bits == oracle.radix_bits(orders.row_count(), 4)
    join2, _ = oracle.join_hash(orders, scan, hy.JoinMode.Inner, (0, 0))
    assert join2.row_count() == ans["join_scan_lineitem_orders_rows"]
    t = lineitem
    for col, cond, val in tf.Q6_SCANS:
        t = oracle.table_scan(t, col, getattr(hy.PredicateCondition, cond), val, [])
    assert t.row_count() == ans["q6_rows"]
    assert math.isclose(q6_revenue(t, None), ans["q6_revenue"], rel_tol=1e-9)
    q1_in = oracle.table_scan(lineitem, 7, hy.PredicateCondition.LessThanEquals, "1998-12-01", [])
    q1 = oracle.aggregate(q1_in, ac.agg_defs(hy, tf.Q1_AGGS), tf.Q1_GROUPBY)
    got = sorted(q1.rows())
    want = ans["q1"]
    assert [(r[0], r[1], r[5]) for r in got] == [(w[0], w[1], w[2]) for w in want]
    for r, w in zip(got, want):
        assert r[2] == w[3]  # SUM(l_quantity): integers, exact
        assert math.isclose(r[3], w[4], rel_tol=1e-12)
        assert math.isclose(r[4], w[5], rel_tol=1e-12)


@pytest.mark.gpu
def test_device_tpch_matches_oracle(hy, oracle):
    orders, lineitem = tf.tables(hy)
    o, l = wrap(hy, orders), wrap(hy, lineitem)
    scan = hy.TableScan(l, 1, hy.PredicateCondition.LessThan, 24)
    scan.execute()
    exp_scan = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, [])
    assert_identical(scan.get_output(), exp_scan)
    j = hy.JoinHash(o, scan, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    assert_identical(j.get_output(), oracle.join_hash(orders, exp_scan, hy.JoinMode.Inner, (0, 0))[0])
    op, t = l, lineitem
    for col, cond, val in tf.Q6_SCANS:
        op = hy.TableScan(op, col, getattr(hy.PredicateCondition, cond), val)
        op.execute()
        t = oracle.table_scan(t, col, getattr(hy.PredicateCondition, cond), val, [])
        assert_identical(op.get_output(), t)
    q1_scan = hy.TableScan(l, 7, hy.PredicateCondition.LessThanEquals, "1998-12-01")
    q1_scan.execute()
    agg = hy.Aggregate(q1_scan, ac.agg_defs(hy, tf.Q1_AGGS), tf.Q1_GROUPBY)
    agg.execute()
    assert agg.used_dense_path()
    q1_in = oracle.table_scan(lineitem, 7, hy.PredicateCondition.LessThanEquals, "1998-12-01", [])
    exp = oracle.aggregate(q1_in, ac.agg_defs(hy, tf.Q1_AGGS), tf.Q1_GROUPBY)
    got, want = agg.get_output().rows(), exp.rows()
    # group keys, order, counts and integer-valued sums exact; float sums: device = exactly rounded sum
    assert [(r[0], r[1], r[2], r[5]) for r in got] == [(r[0], r[1], r[2], r[5]) for r in want]
    for r, w in zip(got, want):
        assert math.isclose(r[3], w[3], rel_tol=1e-12) and math.isclose(r[4], w[4], rel_tol=1e-12)
