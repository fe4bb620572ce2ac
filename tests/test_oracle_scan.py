"""Oracle TableScan pinned to the expectations of the reference's table_scan_test.cpp (CPU only)."""
import pytest

import scan_cases as sc
from helpers import assert_table_eq_unordered, tbl, wrap


def run(oracle, op_or_table, col, cond, value):
    table = op_or_table.get_output() if hasattr(op_or_table, "get_output") else op_or_table
    return oracle.table_scan(table, col, cond, value, [])


@pytest.mark.parametrize("encoding", sc.ENCODINGS)
@pytest.mark.parametrize(
    "cases,value",
    [(sc.compressed_column_cases, 6), (sc.greater_than_max_cases, 30), (sc.less_than_min_cases, -10),
     (sc.around_bounds_cases, 0)],
)
def test_scan_on_compressed_column(hy, oracle, encoding, cases, value):
    full, partly = sc.int_int_tables(hy, encoding)
    for cond, expected in cases().items():
        for w in (full, partly):
            out = run(oracle, w, 0, getattr(hy.PredicateCondition, cond), value)
            assert sorted(sc.column_values(out, 1)) == sorted(expected), (cond, encoding)


@pytest.mark.parametrize("encoding", sc.ENCODINGS)
def test_scan_on_referenced_compressed_column(hy, oracle, encoding):
    full, partly = sc.int_int_tables(hy, encoding)
    for cond, expected in sc.referenced_compressed_cases().items():
        for w in (full, partly):
            s1 = run(oracle, w, 1, hy.PredicateCondition.LessThan, 108)
            out = oracle.table_scan(s1, 0, getattr(hy.PredicateCondition, cond), 4, [])
            assert sorted(sc.column_values(out, 1)) == sorted(expected), cond


@pytest.mark.parametrize("encoding", sc.ENCODINGS)
def test_scan_weird_pos_list(hy, oracle, encoding):
    _, partly = sc.int_int_tables(hy, encoding)
    w = sc.filtered_table(hy, partly)
    for cond, expected in sc.weird_pos_list_cases().items():
        out = run(oracle, w, 0, getattr(hy.PredicateCondition, cond), 10)
        assert sorted(sc.column_values(out, 1)) == sorted(expected), cond


def test_double_scan(hy, oracle):
    t = hy.load_table(tbl("int_float.tbl"), 2)
    s1 = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThanEquals, 1234, [])
    s2 = oracle.table_scan(s1, 1, hy.PredicateCondition.LessThan, 457.9, [])
    assert_table_eq_unordered(s2, hy.load_table(tbl("int_float_filtered.tbl"), 2))


def test_single_scan_row_count(hy, oracle):
    t = hy.load_table(tbl("int_float.tbl"), 2)
    out = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThanEquals, 1234, [])
    assert_table_eq_unordered(out, hy.load_table(tbl("int_float_filtered2.tbl"), 1))


def test_empty_results(hy, oracle):
    t = hy.load_table(tbl("int_float.tbl"), 2)
    s1 = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThan, 12345, [])
    assert s1.row_count() == 0
    s2 = oracle.table_scan(s1, 1, hy.PredicateCondition.Equals, 456.7, [])
    assert s2.row_count() == 0


@pytest.mark.parametrize("encoding", ["Dictionary"])
def test_wide_dictionary(hy, oracle, encoding):
    w16 = sc.dict_n_entries(hy, (1 << 8) + 1, encoding)
    assert w16.get_output().get_chunk(0).get_column(0).attribute_vector_width() == 2
    assert run(oracle, w16, 0, hy.PredicateCondition.GreaterThan, 200).row_count() == 57
    w32 = sc.dict_n_entries(hy, (1 << 16) + 1, encoding)
    assert w32.get_output().get_chunk(0).get_column(0).attribute_vector_width() == 4
    assert run(oracle, w32, 0, hy.PredicateCondition.GreaterThan, 65500).row_count() == 37


def test_between_throws(hy, oracle):
    t = hy.load_table(tbl("int_float.tbl"), 2)
    with pytest.raises(RuntimeError):
        oracle.table_scan(t, 0, hy.PredicateCondition.Between, 6, [])


def test_null_constant_matches_nothing(hy, oracle):
    t = hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4)
    for cond in ("Equals", "NotEquals", "LessThan", "GreaterThanEquals"):
        assert oracle.table_scan(t, 1, getattr(hy.PredicateCondition, cond), None, []).row_count() == 0


def test_excluded_chunks(hy, oracle):
    t = hy.load_table(tbl("int_int_shuffled.tbl"), 7)
    out = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThanEquals, 0, [0])
    assert out.row_count() == t.get_chunk(1).size()


def test_scan_for_null_values(hy, oracle):
    for name, t, cases in sc.null_scan_tables(hy):
        for cond, expected in cases.items():
            out = oracle.table_scan(t, 1, getattr(hy.PredicateCondition, cond), None, [])
            assert sc.multiset(sc.column_values(out, 0)) == sc.multiset(expected), (name, cond)


def test_is_null_reference_order(hy, oracle):
    """NULL RowIDs match IS NULL after the referenced columns' matches (is_null_table_scan_impl.cpp:20-33)."""
    t = hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4)
    out = oracle.table_scan(sc.referencing_table_w_null_row_id(hy, t), 1, hy.PredicateCondition.IsNull, None, [])
    assert [list(r) for r in out.get_chunk(0).get_column(1).pos_list()] == [[0, 1], [sc.NULL_ROW_ID] * 2]


def test_column_comparison(hy, oracle):
    for name, t in sc.column_compare_tables(hy):
        out = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThan, None, [], right_column_id=1)
        assert sc.multiset(sc.column_values(out, 0)) == sc.multiset(sc.COLUMN_COMPARE_EXPECTED), name


def test_column_comparison_mixed_types(hy, oracle):
    """int vs float compares as float (C++ usual arithmetic conversions, the reference's with_comparator)."""
    t = hy.Table([("a", hy.DataType.Int, False), ("b", hy.DataType.Float, False)], hy.TableType.Data)
    for a, b in ((1, 0.5), (2, 2.0), (3, 3.5), (16777217, 16777216.0)):
        t.append([a, b])
    gt = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThan, None, [], right_column_id=1)
    eq = oracle.table_scan(t, 0, hy.PredicateCondition.Equals, None, [], right_column_id=1)
    assert sc.column_values(gt, 0) == [1]
    assert sc.column_values(eq, 0) == [2, 16777217]  # 16777217 -> 16777216.0f


def _like_expect(hy, out, expected):
    if isinstance(expected, int):
        assert out.row_count() == expected
    else:
        assert_table_eq_unordered(out, hy.load_table(tbl(expected), 1))


def test_like(hy, oracle):
    """LIKE / NOT LIKE pinned to table_scan_string_test.cpp (unencoded, dictionary, referenced dictionary)."""
    for enc, t in sc.like_tables(hy):
        for cond, pattern, expected in sc.LIKE_CASES:
            out = oracle.table_scan(t, 1, getattr(hy.PredicateCondition, cond), pattern, [])
            _like_expect(hy, out, expected)
            s1 = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThan, 0, [])
            _like_expect(hy, oracle.table_scan(s1, 1, getattr(hy.PredicateCondition, cond), pattern, []), expected)
    special = hy.load_table(tbl("int_string_like_special_chars.tbl"), 2)
    for pattern, expected in sc.LIKE_SPECIAL_CASES:
        _like_expect(hy, oracle.table_scan(special, 1, hy.PredicateCondition.Like, pattern, []), expected)
    t = hy.load_table(tbl("int_string_like.tbl"), 2)
    assert oracle.table_scan(t, 1, hy.PredicateCondition.Like, 1234, []).row_count() == 1  # ScanLikeNonStringValue
    with pytest.raises(RuntimeError):  # ScanLikeNonStringColumn
        oracle.table_scan(hy.load_table(tbl("int_float.tbl"), 2), 0, hy.PredicateCondition.Like, "%test", [])
