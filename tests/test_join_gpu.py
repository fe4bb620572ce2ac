"""Device JoinHash parity: every reference join case (numeric join columns) produces the oracle's output
bit-for-bit — same output chunks (radix partitions), same PosLists in the same order — and matches the reference's
expected table; plus seeded synthetic joins with many partitions, duplicates and reference inputs."""
import numpy as np
import pytest

import join_cases as jc
from helpers import assert_identical, assert_table_eq_unordered, tbl, wrap

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", jc.CASES, ids=jc.CASE_IDS)
def test_device_join_matches_oracle(hy, oracle, case):
    """Includes the string join columns (and int / string joins through the reference's lexical cast): ids of
    distinct strings joined on the device, partitioned by the strings' murmur2 (hy_join_params.key_hash)."""
    name, left, right, mode, cols, expected = case
    base = jc.BaseTables(hy)
    plan = ("join", left, right, mode, cols)
    dev = jc.eval_device(hy, base, plan)
    exp = jc.eval_oracle(hy, oracle, base, plan)
    assert_identical(dev.get_output(), exp)
    if expected is not None:
        assert_table_eq_unordered(dev.get_output(), hy.load_table(tbl(expected), 1))


def orders_lineitem(hy, n_orders, chunk, rng):
    i = np.arange(1, n_orders + 1, dtype=np.int64)
    okey = (((i >> 3) << 5) + (i & 7)).astype(np.int32)  # dbgen sparse order keys (build.c)
    lines = rng.integers(1, 8, n_orders)
    lkey = np.repeat(okey, lines)
    qty = rng.integers(1, 51, lkey.size).astype(np.int32)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [okey], [], chunk)
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False), ("l_quantity", hy.DataType.Int, False)],
                                    [lkey, qty], [], chunk)
    return orders, lineitem


@pytest.mark.parametrize("n_orders,chunk", [(20_000, 10_000), (300_000, 65_536)])
def test_orders_lineitem_join(hy, oracle, n_orders, chunk):
    rng = np.random.default_rng(n_orders)
    orders, lineitem = orders_lineitem(hy, n_orders, chunk, rng)
    hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
    o, l = wrap(hy, orders), wrap(hy, lineitem)
    j = hy.JoinHash(o, l, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp, bits = oracle.join_hash(orders, lineitem, hy.JoinMode.Inner, (0, 0))
    assert j.used_radix_bits() == bits
    assert_identical(j.get_output(), exp)
    assert j.get_output().row_count() == lineitem.row_count()
    # Scan -> Join pipeline (reference input on the probe side)
    s = hy.TableScan(l, 1, hy.PredicateCondition.LessThan, 24)
    s.execute()
    j2 = hy.JoinHash(o, s, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j2.execute()
    exp2, _ = oracle.join_hash(orders, oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, []),
                               hy.JoinMode.Inner, (0, 0))
    assert_identical(j2.get_output(), exp2)


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("order", ["join_first", "scan_first", "semi"])
def test_deferred_scan_fused_into_join(hy, oracle, monkeypatch, fuse, order):
    """TableScan -> JoinHash through the operators: a scan over a data table is deferred (its output produced on
    first access), and the JoinHash that takes it as its probe side evaluates the predicate in its first radix pass
    and builds the scan's output from the join's by-product (HY_OP_FUSE_SCAN=0: the scan runs when it executes).
    Both outputs equal the oracle's whatever is read first; a Semi join (not fused) produces the scan on access."""
    monkeypatch.setenv("HY_OP_FUSE_SCAN", fuse)
    rng = np.random.default_rng(7)
    orders, lineitem = orders_lineitem(hy, 30_000, 10_000, rng)
    hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
    o, l = wrap(hy, orders), wrap(hy, lineitem)
    s = hy.TableScan(l, 1, hy.PredicateCondition.LessThan, 24)
    s.execute()
    exp_s = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, [])
    if order == "scan_first":  # the scan's output produced before the join reads it
        assert_identical(s.get_output(), exp_s)
    mode = hy.JoinMode.Semi if order == "semi" else hy.JoinMode.Inner
    j = hy.JoinHash(o, s, mode, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp_j, bits = oracle.join_hash(orders, exp_s, mode, (0, 0))
    assert j.used_radix_bits() == bits
    assert_identical(j.get_output(), exp_j)
    assert_identical(s.get_output(), exp_s)
    assert s.get_output().row_count() == exp_s.row_count()


@pytest.mark.parametrize("lds_budget", [None, 1024])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Right", "Semi", "Anti"])
def test_duplicates_and_nulls(hy, oracle, mode, lds_budget, monkeypatch):
    # lds_budget=1024 caps every LDS hash table at a few dozen build rows, so every partition runs as a chain of
    # sub-tables (the skewed-partition path) while the expected output stays the reference's
    if lds_budget is not None:
        monkeypatch.setenv("HY_JOIN_LDS_BUDGET", str(lds_budget))
    rng = np.random.default_rng(11)
    n1, n2 = 30_000, 50_000
    k1 = rng.integers(0, 8_000, n1).astype(np.int64)
    k2 = rng.integers(0, 12_000, n2).astype(np.int32)
    nl1 = (rng.random(n1) < 0.03).astype(np.uint8)
    nl2 = (rng.random(n2) < 0.03).astype(np.uint8)
    a = hy.Table.from_arrays([("k", hy.DataType.Long, True)], [k1], [nl1], 7_000)
    b = hy.Table.from_arrays([("k", hy.DataType.Int, True), ("v", hy.DataType.Int, False)],
                             [k2, np.arange(n2, dtype=np.int32)], [nl2, None], 9_999)
    for left, right in ((a, b), (b, a)):
        j = hy.JoinHash(wrap(hy, left), wrap(hy, right), getattr(hy.JoinMode, mode), (0, 0),
                        hy.PredicateCondition.Equals)
        j.execute()
        exp, _ = oracle.join_hash(left, right, getattr(hy.JoinMode, mode), (0, 0))
        assert_identical(j.get_output(), exp)


def test_float_keys(hy, oracle):
    rng = np.random.default_rng(3)
    ka = (rng.integers(-500, 500, 20_000) * 0.5).astype(np.float32)
    kb = (rng.integers(-500, 500, 25_000) * 0.5).astype(np.float64)
    a = hy.Table.from_arrays([("k", hy.DataType.Float, False)], [ka], [], 4_096)
    b = hy.Table.from_arrays([("k", hy.DataType.Double, False)], [kb], [], 5_000)
    j = hy.JoinHash(wrap(hy, a), wrap(hy, b), hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp, _ = oracle.join_hash(a, b, hy.JoinMode.Inner, (0, 0))
    assert_identical(j.get_output(), exp)


@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi", "Anti"])
def test_skewed_keys_use_sub_tables(hy, oracle, mode):
    # a few hot keys put >10k build rows into one radix partition: beyond one LDS table -> chained sub-tables
    rng = np.random.default_rng(5)
    build = np.where(rng.random(12_000) < 0.9, 42, rng.integers(0, 1000, 12_000)).astype(np.int32)
    probe = rng.integers(0, 1200, 3_000).astype(np.int32)
    a = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [probe], [], 1_000)
    b = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [build], [], 5_000)
    j = hy.JoinHash(wrap(hy, a), wrap(hy, b), getattr(hy.JoinMode, mode), (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp, _ = oracle.join_hash(a, b, getattr(hy.JoinMode, mode), (0, 0))
    assert_identical(j.get_output(), exp)


@pytest.mark.parametrize("cond,value", [("LessThan", 24), ("GreaterThanEquals", 7)])
def test_scan_over_join_output(hy, oracle, cond, value):
    """TableScan over a JoinHash output: every output chunk's PosList references hundreds of lineitem chunks, so the
    scan runs in the reference's split_pos_list_by_chunk_id group order (chunk_offset_mapping.cpp:5-21,
    base_single_column_table_scan_impl.cpp:36-60) - one device scan plus the stable group-order sort
    (hy_reference_scan_order) - and equals the oracle's scan of the oracle's join, RowID for RowID."""
    rng = np.random.default_rng(11)
    orders, lineitem = orders_lineitem(hy, 60_000, 700, rng)
    hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
    o, l = wrap(hy, orders), wrap(hy, lineitem)
    j = hy.JoinHash(o, l, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp_j, _ = oracle.join_hash(orders, lineitem, hy.JoinMode.Inner, (0, 0))
    assert_identical(j.get_output(), exp_j)
    pc = getattr(hy.PredicateCondition, cond)
    s = hy.TableScan(j, 2, pc, value)  # l_quantity of the join output (orders' column first)
    s.execute()
    exp_s = oracle.table_scan(exp_j, 2, pc, value, [])
    assert exp_s.row_count() > 0
    assert_identical(s.get_output(), exp_s)


@pytest.mark.parametrize("encoding", ["RunLength", "FrameOfReference"])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Anti"])
def test_encoded_join_columns(hy, oracle, encoding, mode):
    """RunLength / FrameOfReference chunks (decoded into HBM value mirrors) on both join sides, NULLs included."""
    rng = np.random.default_rng(23)
    n1, n2 = 20_000, 35_000
    k1 = np.sort(rng.integers(0, 3_000, n1)).astype(np.int64)  # sorted: long runs
    k2 = rng.integers(0, 4_000, n2).astype(np.int32)
    nl1 = (rng.random(n1) < 0.02).astype(np.uint8)
    nl2 = (rng.random(n2) < 0.02).astype(np.uint8)
    a = hy.Table.from_arrays([("k", hy.DataType.Long, True)], [k1], [nl1], 6_000)
    b = hy.Table.from_arrays([("k", hy.DataType.Int, True), ("v", hy.DataType.Int, False)],
                             [k2, np.arange(n2, dtype=np.int32)], [nl2, None], 8_191)
    hy.encode_chunks(a, [0, 2], getattr(hy.EncodingType, encoding))
    hy.encode_all_chunks(b, getattr(hy.EncodingType, encoding))
    for left, right in ((a, b), (b, a)):
        j = hy.JoinHash(wrap(hy, left), wrap(hy, right), getattr(hy.JoinMode, mode), (0, 0),
                        hy.PredicateCondition.Equals)
        j.execute()
        exp, _ = oracle.join_hash(left, right, getattr(hy.JoinMode, mode), (0, 0))
        assert_identical(j.get_output(), exp)


@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi", "Anti"])
def test_join_column_referencing_several_tables(hy, oracle, mode):
    """A reference input whose chunks reference different tables (e.g. two scans' outputs appended into one table):
    every row's key is read from its own chunk's table, as the reference's ReferenceColumn iterable does
    (join_hash.cpp:248-276); the output columns name chunk 0's table, as write_output_columns does (:595-598).
    RowID-exact against the oracle, with and without a single referenced chunk per PosList."""
    rng = np.random.default_rng(77)
    T = hy.DataType
    tabs = []
    for seed in range(3):
        k = rng.integers(0, 2_000, 9_000).astype(np.int32)
        v = np.arange(9_000, dtype=np.int32) + seed * 100_000
        tabs.append(hy.Table.from_arrays([("k", T.Int, False), ("v", T.Int, False)], [k, v], [], 3_000))
    hy.encode_chunks(tabs[1], [0, 2], hy.EncodingType.Dictionary)
    ref = hy.Table([("k", T.Int, False), ("v", T.Int, False)], hy.TableType.References)
    for i in range(7):
        t = tabs[i % 3]
        if i % 2:  # a PosList into one chunk of the table
            c = int(rng.integers(0, 3))
            pl = np.stack([np.full(1_500, c), rng.integers(0, 3_000, 1_500)], axis=1).astype(np.uint32)
        else:  # a PosList across the table's chunks, NULL RowIDs included
            pl = np.stack([rng.integers(0, 3, 2_000), rng.integers(0, 3_000, 2_000)], axis=1).astype(np.uint32)
            pl[rng.random(2_000) < 0.02] = 0xFFFFFFFF
        ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    other = hy.Table.from_arrays([("k", T.Int, False)], [rng.integers(0, 2_500, 12_000).astype(np.int32)], [], 4_000)
    for left, right in ((ref, other), (other, ref)):
        j = hy.JoinHash(wrap(hy, left), wrap(hy, right), getattr(hy.JoinMode, mode), (0, 0),
                        hy.PredicateCondition.Equals)
        j.execute()
        exp, _ = oracle.join_hash(left, right, getattr(hy.JoinMode, mode), (0, 0))
        assert_identical(j.get_output(), exp)


@pytest.mark.parametrize("mode", ["Inner", "Left", "Right", "Semi", "Anti"])
@pytest.mark.parametrize("tables", [1, 3])
def test_poslists_over_several_value_chunks(hy, oracle, mode, tables):
    """Reference inputs whose PosLists span several ValueColumn chunks (a join output as the next join's input, TPC-H
    3's second build side): the batched load path (RowIDs, chunk pointers, values as three load phases; join_host's
    LP_REFM), with NULL RowIDs, one or several referenced tables, on either side. RowID-exact against the oracle."""
    rng = np.random.default_rng(91 + tables)
    T = hy.DataType
    tabs = []
    for seed in range(tables):
        k = rng.integers(0, 3_000, 12_000).astype(np.int32)
        v = np.arange(12_000, dtype=np.int32) + seed * 100_000
        tabs.append(hy.Table.from_arrays([("k", T.Int, False), ("v", T.Int, False)], [k, v], [], 2_500))
    ref = hy.Table([("k", T.Int, False), ("v", T.Int, False)], hy.TableType.References)
    for i in range(6):
        t = tabs[i % tables]
        pl = np.stack([rng.integers(0, 5, 3_000), rng.integers(0, 2_000, 3_000)], axis=1).astype(np.uint32)
        pl[rng.random(3_000) < 0.03] = 0xFFFFFFFF
        ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    other = hy.Table.from_arrays([("k", T.Int, False)], [rng.integers(0, 3_500, 15_000).astype(np.int32)], [], 4_000)
    for left, right in ((ref, other), (other, ref)):
        j = hy.JoinHash(wrap(hy, left), wrap(hy, right), getattr(hy.JoinMode, mode), (0, 0),
                        hy.PredicateCondition.Equals)
        j.execute()
        exp, _ = oracle.join_hash(left, right, getattr(hy.JoinMode, mode), (0, 0))
        assert_identical(j.get_output(), exp)


@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi", "Anti"])
def test_probe_skew_needs_several_passes(hy, oracle, mode):
    """A few hot probe keys put tens of thousands of probe rows into single radix partitions while the average
    partition takes one pass: those partitions are listed by join_partition and joined by join_partition_multi
    (several probe passes), the rest in one pass; every partition's PosLists equal the oracle's."""
    rng = np.random.default_rng(31)
    build = rng.permutation(np.arange(200_000, dtype=np.int32))
    probe = np.where(rng.random(300_000) < 0.3, rng.integers(0, 3, 300_000), rng.integers(0, 260_000, 300_000))
    a = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [build], [], 50_000)
    b = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [probe.astype(np.int32)], [], 65_536)
    j = hy.JoinHash(wrap(hy, a), wrap(hy, b), getattr(hy.JoinMode, mode), (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    exp, _ = oracle.join_hash(a, b, getattr(hy.JoinMode, mode), (0, 0))
    assert_identical(j.get_output(), exp)


def test_join_plan_cache_reexecution(hy, oracle):
    """Re-executions of TableScan -> JoinHash of one shape run the cached prepared plan (JoinPlanCache, rebound to each
    execution's TableScan output): every execution's join and scan outputs equal the oracle's - also after another
    predicate (a new shape, a cache miss) ran in between - and earlier outputs stay valid while later ones are made."""
    rng = np.random.default_rng(23)
    orders, lineitem = orders_lineitem(hy, 30_000, 10_000, rng)
    hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
    o, l = wrap(hy, orders), wrap(hy, lineitem)
    hy.join_plan_cache_set_capacity(2)  # (opt-in: HY_OP_PLAN_CACHE, default off)
    hits0, misses0 = hy.join_plan_cache_stats()
    kept = []
    for i, value in enumerate([24, 24, 31, 24, 24]):
        s = hy.TableScan(l, 1, hy.PredicateCondition.LessThan, value)
        s.execute()
        j = hy.JoinHash(o, s, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
        j.execute()
        exp_s = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, value, [])
        exp_j, _ = oracle.join_hash(orders, exp_s, hy.JoinMode.Inner, (0, 0))
        assert_identical(j.get_output(), exp_j)
        assert_identical(s.get_output(), exp_s)
        kept.append((j, s, exp_j, exp_s))
    for j, s, exp_j, exp_s in kept:  # the cached plan wrote every execution's outputs into buffers of their own
        assert_identical(j.get_output(), exp_j)
        assert_identical(s.get_output(), exp_s)
    hits, misses = hy.join_plan_cache_stats()
    assert misses - misses0 == 2 and hits - hits0 == 3  # shapes <24 and <31
    hy.join_plan_cache_set_capacity(0)
