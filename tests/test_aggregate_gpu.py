"""Device Aggregate parity: every aggregate_test.cpp case produces the oracle's output table exactly — same rows in
the same (std::unordered_map) order, same names, types and values — and the reference's expected table; plus
seeded synthetic aggregations over the dense (LDS) and hash (HBM) device paths, with NULLs, strings, float sums,
COUNT(DISTINCT) and reference inputs from device TableScans."""
import math
import struct

import numpy as np
import pytest

import agg_cases as ac
from helpers import assert_identical, assert_table_eq_unordered, tbl, wrap

pytestmark = pytest.mark.gpu


def run_device(hy, table, aggs, groupby):
    op = hy.Aggregate(wrap(hy, table), ac.agg_defs(hy, aggs), groupby)
    op.execute()
    return op.get_output()


@pytest.mark.parametrize("case", ac.CASES, ids=ac.CASE_IDS)
def test_device_aggregate_matches_oracle(hy, oracle, case):
    name, inp, aggs, groupby, expected, on_ref = case
    base = ac.BaseTables(hy)
    table = ac.input_table_oracle(hy, oracle, base, inp)
    exp = hy.load_table(tbl(expected), 1)
    out = run_device(hy, table, aggs, groupby)
    assert_identical(out, oracle.aggregate(table, ac.agg_defs(hy, aggs), groupby))
    assert_table_eq_unordered(out, exp)
    if on_ref:
        ref = oracle.table_scan(table, 0, hy.PredicateCondition.GreaterThanEquals, 0, [])
        out2 = run_device(hy, ref, aggs, groupby)
        assert_identical(out2, oracle.aggregate(ref, ac.agg_defs(hy, aggs), groupby))
        assert_table_eq_unordered(out2, exp)


@pytest.mark.parametrize("case", ac.FAILING, ids=[c[0] for c in ac.FAILING])
def test_device_aggregate_rejects_string_sum_avg(hy, case):
    _, inp, aggs, groupby = case
    base = ac.BaseTables(hy)
    with pytest.raises(RuntimeError):
        run_device(hy, base.table(inp), aggs, groupby)


def q1_like(hy, n, chunk, rng, nulls=False):
    """lineitem-shaped columns: returnflag/linestatus codes, quantity, price (cents), discount, tax, shipdate."""
    rf = rng.integers(0, 3, n).astype(np.int32)
    ls = rng.integers(0, 2, n).astype(np.int32)
    qty = rng.integers(1, 51, n).astype(np.int32)
    price = (qty.astype(np.int64) * rng.integers(90_000, 210_000, n)).astype(np.int64)
    disc = rng.integers(0, 11, n).astype(np.int32)
    tax = rng.integers(0, 9, n).astype(np.int32)
    ship = rng.integers(8000, 10600, n).astype(np.int32)
    null_masks = [None] * 7
    cols = [("l_returnflag", hy.DataType.Int, nulls), ("l_linestatus", hy.DataType.Int, False),
            ("l_quantity", hy.DataType.Int, False), ("l_extendedprice", hy.DataType.Long, False),
            ("l_discount", hy.DataType.Int, nulls), ("l_tax", hy.DataType.Int, False),
            ("l_shipdate", hy.DataType.Int, False)]
    if nulls:
        null_masks[0] = (rng.random(n) < 0.01).astype(np.uint8)
        null_masks[4] = (rng.random(n) < 0.05).astype(np.uint8)
    return hy.Table.from_arrays(cols, [rf, ls, qty, price, disc, tax, ship], null_masks, chunk)


Q1_AGGS = [(2, "Sum"), (3, "Sum"), (4, "Sum"), (5, "Sum"), (2, "Avg"), (3, "Avg"), (4, "Avg"), (None, "Count")]


@pytest.mark.parametrize("nulls", [False, True])
def test_q1_shape_dense_path(hy, oracle, nulls):
    rng = np.random.default_rng(11 + nulls)
    t = q1_like(hy, 300_000, 65_536, rng, nulls)
    hy.encode_chunks(t, list(range(t.chunk_count())), hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    scan = hy.TableScan(w, 6, hy.PredicateCondition.LessThanEquals, 10_471)
    scan.execute()
    agg = hy.Aggregate(scan, ac.agg_defs(hy, Q1_AGGS), [0, 1])
    agg.execute()
    assert agg.used_dense_path()
    ref_in = oracle.table_scan(t, 6, hy.PredicateCondition.LessThanEquals, 10_471, [])
    assert_identical(agg.get_output(), oracle.aggregate(ref_in, ac.agg_defs(hy, Q1_AGGS), [0, 1]))


def test_many_groups_hash_path(hy, oracle):
    rng = np.random.default_rng(5)
    n = 200_000
    key = rng.integers(0, 50_000, n).astype(np.int32)
    key2 = rng.integers(-3, 3, n).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np.int32)
    f = rng.standard_normal(n).astype(np.float32)
    t = hy.Table.from_arrays([("k", hy.DataType.Int, True), ("k2", hy.DataType.Long, False),
                              ("v", hy.DataType.Int, True), ("f", hy.DataType.Float, False)],
                             [key, key2, v, f],
                             [(rng.random(n) < 0.02).astype(np.uint8), None, (rng.random(n) < 0.1).astype(np.uint8), None],
                             30_000)
    aggs = [(2, "Sum"), (2, "Min"), (2, "Max"), (2, "Count"), (2, "CountDistinct"), (3, "Max"), (None, "Count")]
    op = hy.Aggregate(wrap(hy, t), ac.agg_defs(hy, aggs), [0, 1])
    op.execute()
    assert not op.used_dense_path()
    out = op.get_output()
    assert_identical(out, oracle.aggregate(t, ac.agg_defs(hy, aggs), [0, 1]))


def test_float_sums_exact_rounding(hy, oracle):
    """SUM/AVG of floats: the device sum is the exact sum rounded once (<= 0.5 ULP of math.fsum); the reference's
    sequential double sum is compared with a tolerance (its own rounding error), groups and counts exactly."""
    rng = np.random.default_rng(3)
    n = 500_000
    g = rng.integers(0, 5, n).astype(np.int32)
    f = (rng.standard_normal(n) * 1e4).astype(np.float32)
    d = rng.standard_normal(n) * 1e-3
    t = hy.Table.from_arrays([("g", hy.DataType.Int, False), ("f", hy.DataType.Float, False),
                              ("d", hy.DataType.Double, False)], [g, f, d], [], 100_000)
    aggs = [(1, "Sum"), (2, "Sum"), (1, "Avg")]
    out = run_device(hy, t, aggs, [0])
    exp = oracle.aggregate(t, ac.agg_defs(hy, aggs), [0])
    ra, re_ = out.rows(), exp.rows()
    assert [r[0] for r in ra] == [r[0] for r in re_]
    for row in ra:
        sel = g == row[0]
        assert row[1] == math.fsum(f[sel].astype(np.float64))
        assert row[2] == math.fsum(d[sel])
    for x, y in zip(ra, re_):
        assert math.isclose(x[1], y[1], rel_tol=1e-9) and math.isclose(x[2], y[2], rel_tol=1e-9)
        assert math.isclose(x[3], y[3], rel_tol=1e-9)


def test_string_group_and_minmax(hy, oracle):
    base = ac.BaseTables(hy)
    t = base.table("1_1_string")
    hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
    for aggs, gb in (([(1, "Max"), (0, "Min"), (0, "CountDistinct")], [0]), ([(0, "Max"), (0, "Count")], [])):
        out = run_device(hy, t, aggs, gb)
        assert_identical(out, oracle.aggregate(t, ac.agg_defs(hy, aggs), gb))


def test_empty_input(hy, oracle):
    base = ac.BaseTables(hy)
    t = base.table("1_2")
    empty = oracle.table_scan(t, 0, hy.PredicateCondition.LessThan, -(10**6), [])
    for gb in ([], [0]):
        aggs = [(1, "Max"), (2, "Sum"), (None, "Count"), (1, "CountDistinct")]
        out = run_device(hy, empty, aggs, gb)
        assert_identical(out, oracle.aggregate(empty, ac.agg_defs(hy, aggs), gb))


@pytest.mark.parametrize("reference_input", [False, True])
def test_dense_span_float_sums_mixed_integer_rows(hy, oracle, monkeypatch, reference_input):
    """agg_dense_span sums integer-valued float rows in an int64 word and the others in limbs; the folded result must
    be the exact sum rounded once (== math.fsum) and decode to the per-64-row kernel's results (HY_AGG_DENSE_ROWS=1)."""
    rng = np.random.default_rng(17)
    n = 250_000
    g = rng.integers(0, 4, n).astype(np.int32)
    ints = rng.integers(-60, 61, n).astype(np.float32)
    f = np.where(rng.random(n) < 0.7, ints, (rng.standard_normal(n) * 100).astype(np.float32)).astype(np.float32)
    big = rng.integers(-(1 << 40), 1 << 40, n).astype(np.float64)  # integers above 2^31 take the limb path
    d = np.where(rng.random(n) < 0.5, rng.integers(-1000, 1000, n).astype(np.float64), big)
    d = np.where(rng.random(n) < 0.1, d + 0.25, d)
    nulls = (rng.random(n) < 0.05).astype(np.uint8)
    t = hy.Table.from_arrays([("g", hy.DataType.Int, False), ("f", hy.DataType.Float, True),
                              ("d", hy.DataType.Double, False)], [g, f, d], [None, nulls, None], 60_000)
    hy.encode_chunks(t, list(range(t.chunk_count())), hy.EncodingType.Dictionary)
    src = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThanEquals, 0, []) if reference_input else t
    aggs = [(1, "Sum"), (2, "Sum"), (1, "Avg"), (2, "Avg"), (None, "Count")]

    def run():
        op = hy.Aggregate(wrap(hy, src), ac.agg_defs(hy, aggs), [0])
        op.execute()
        assert op.used_dense_path()
        return op.get_output()

    out = run()
    monkeypatch.setenv("HY_AGG_DENSE_ROWS", "1")
    out_rows_kernel = run()
    monkeypatch.delenv("HY_AGG_DENSE_ROWS")
    assert_identical(out, out_rows_kernel)
    for row in out.rows():
        sel = g == row[0]
        assert row[1] == math.fsum(f[sel & (nulls == 0)].astype(np.float64))
        assert row[2] == math.fsum(d[sel])


def test_hash_aggregate_grows_past_its_group_bound(hy, oracle, monkeypatch):
    """More groups than the hash table was sized for (HY_AGG_RECORD_BUDGET shrinks the derived bound to a few
    thousand groups): hy_aggregate reports HY_ERR_GROUP_BOUND, the operator retries with 4x larger tables, and the
    result equals the reference Aggregate's (groups in first-appearance order)."""
    monkeypatch.setenv("HY_AGG_RECORD_BUDGET", str(1 << 20))
    rng = np.random.default_rng(23)
    n = 600_000
    keys = rng.permutation(n).astype(np.int64) * 3 - 7
    vals = rng.integers(-1000, 1000, n).astype(np.int32)
    t = hy.Table.from_arrays([("k", hy.DataType.Long, False), ("v", hy.DataType.Int, False)], [keys, vals], [],
                             100_000)
    aggs = [(1, "Sum"), (None, "Count")]
    op = hy.Aggregate(wrap(hy, t), ac.agg_defs(hy, aggs), [0])
    op.execute()
    assert not op.used_dense_path()
    assert_identical(op.get_output(), oracle.aggregate(t, ac.agg_defs(hy, aggs), [0]))


@pytest.mark.parametrize("encoding", ["RunLength", "FrameOfReference"])
def test_encoded_inputs(hy, oracle, encoding):
    """Aggregates over RunLength / FrameOfReference chunks (decoded into HBM value mirrors), dense and hash paths,
    mixed with unencoded chunks (FrameOfReference leaves the float columns unencoded, as it supports ints only)."""
    rng = np.random.default_rng(41)
    t = q1_like(hy, 200_000, 50_000, rng, nulls=True)
    hy.encode_chunks(t, [0, 2, 3], getattr(hy.EncodingType, encoding))
    w = wrap(hy, t)
    scan = hy.TableScan(w, 6, hy.PredicateCondition.LessThanEquals, 10_471)
    scan.execute()
    agg = hy.Aggregate(scan, ac.agg_defs(hy, Q1_AGGS), [0, 1])
    agg.execute()
    ref_in = oracle.table_scan(t, 6, hy.PredicateCondition.LessThanEquals, 10_471, [])
    assert_identical(agg.get_output(), oracle.aggregate(ref_in, ac.agg_defs(hy, Q1_AGGS), [0, 1]))
    aggs = [(2, "Sum"), (3, "Min"), (6, "Max"), (None, "Count")]
    op = hy.Aggregate(w, ac.agg_defs(hy, aggs), [6])
    op.execute()
    assert_identical(op.get_output(), oracle.aggregate(t, ac.agg_defs(hy, aggs), [6]))
