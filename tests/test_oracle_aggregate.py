"""Oracle Aggregate pinned to the expectations of the reference's aggregate_test.cpp (CPU only): every test_output
case on the stored table and, where the reference does, on TableScan(in, ColumnID{0}, >=, 0) of it."""
import pytest

import agg_cases as ac
from helpers import assert_table_eq_unordered, tbl


@pytest.mark.parametrize("case", ac.CASES, ids=ac.CASE_IDS)
def test_oracle_aggregate_matches_reference_expectation(hy, oracle, case):
    name, inp, aggs, groupby, expected, on_ref = case
    base = ac.BaseTables(hy)
    table = ac.input_table_oracle(hy, oracle, base, inp)
    exp = hy.load_table(tbl(expected), 1)
    out = oracle.aggregate(table, ac.agg_defs(hy, aggs), groupby)
    assert_table_eq_unordered(out, exp)
    if on_ref:
        ref = oracle.table_scan(table, 0, hy.PredicateCondition.GreaterThanEquals, 0, [])
        assert_table_eq_unordered(oracle.aggregate(ref, ac.agg_defs(hy, aggs), groupby), exp)


@pytest.mark.parametrize("case", ac.FAILING, ids=[c[0] for c in ac.FAILING])
def test_oracle_aggregate_rejects_string_sum_avg(hy, oracle, case):
    _, inp, aggs, groupby = case
    base = ac.BaseTables(hy)
    with pytest.raises(RuntimeError):
        oracle.aggregate(base.table(inp), ac.agg_defs(hy, aggs), groupby)


def test_no_groupby_and_no_aggregate_throws(hy):
    base = ac.BaseTables(hy)
    w = hy.TableWrapper(base.table("1_1"))
    w.execute()
    with pytest.raises(RuntimeError):
        hy.Aggregate(w, [], [])
