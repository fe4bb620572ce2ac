"""Device TableScan parity: bit-exact PosLists against the oracle on the reference's test setups and on seeded
synthetic tables (all widths, NULLs, ragged chunks, reference inputs)."""
import numpy as np
import pytest

import scan_cases as sc
from helpers import assert_identical, assert_table_eq_unordered, tbl, wrap

pytestmark = pytest.mark.gpu

CONDS = ["Equals", "NotEquals", "LessThan", "LessThanEquals", "GreaterThan", "GreaterThanEquals"]


def device_scan(hy, op, col, cond, value, excluded=None):
    s = hy.TableScan(op, col, getattr(hy.PredicateCondition, cond), value)
    if excluded:
        s.set_excluded_chunk_ids(excluded)
    s.execute()
    return s


def check(hy, oracle, op, col, cond, value, excluded=None):
    s = device_scan(hy, op, col, cond, value, excluded)
    exp = oracle.table_scan(op.get_output(), col, getattr(hy.PredicateCondition, cond), value, excluded or [])
    assert_identical(s.get_output(), exp)
    return s


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
            s = check(hy, oracle, w, 0, cond, value)
            assert sorted(sc.column_values(s.get_output(), 1)) == sorted(expected)


@pytest.mark.parametrize("encoding", sc.ENCODINGS)
def test_scan_on_referenced_compressed_column(hy, oracle, encoding):
    full, partly = sc.int_int_tables(hy, encoding)
    for cond, expected in sc.referenced_compressed_cases().items():
        for w in (full, partly):
            s1 = device_scan(hy, w, 1, "LessThan", 108)
            s2 = check(hy, oracle, s1, 0, cond, 4)
            assert sorted(sc.column_values(s2.get_output(), 1)) == sorted(expected)


@pytest.mark.parametrize("encoding", sc.ENCODINGS)
def test_scan_weird_pos_list(hy, oracle, encoding):
    _, partly = sc.int_int_tables(hy, encoding)
    w = sc.filtered_table(hy, partly)
    for cond, expected in sc.weird_pos_list_cases().items():
        s = check(hy, oracle, w, 0, cond, 10)
        assert sorted(sc.column_values(s.get_output(), 1)) == sorted(expected)


def test_double_scan_and_empty(hy, oracle):
    w = wrap(hy, hy.load_table(tbl("int_float.tbl"), 2))
    s1 = check(hy, oracle, w, 0, "GreaterThanEquals", 1234)
    s2 = check(hy, oracle, s1, 1, "LessThan", 457.9)
    assert_table_eq_unordered(s2.get_output(), hy.load_table(tbl("int_float_filtered.tbl"), 2))
    e1 = check(hy, oracle, w, 0, "GreaterThan", 12345)
    assert e1.get_output().row_count() == 0
    e2 = check(hy, oracle, e1, 1, "Equals", 456.7)
    assert e2.get_output().row_count() == 0


def test_wide_dictionaries(hy, oracle):
    w16 = sc.dict_n_entries(hy, (1 << 8) + 1, "Dictionary")
    assert check(hy, oracle, w16, 0, "GreaterThan", 200).get_output().row_count() == 57
    w32 = sc.dict_n_entries(hy, (1 << 16) + 1, "Dictionary")
    assert check(hy, oracle, w32, 0, "GreaterThan", 65500).get_output().row_count() == 37


def test_between_and_null_constant(hy, oracle):
    w = wrap(hy, hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4))
    with pytest.raises(RuntimeError):
        device_scan(hy, w, 0, "Between", 6)
    for cond in CONDS:
        assert device_scan(hy, w, 1, cond, None).get_output().row_count() == 0


def test_nullable_columns_all_predicates(hy, oracle):
    for enc in (None, "Dictionary"):
        t = hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4)
        if enc:
            hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
        w = wrap(hy, t)
        for cond in CONDS:
            for v in (12, 123, 1234, 0, 99999):
                check(hy, oracle, w, 0, cond, v)
                check(hy, oracle, w, 1, cond, v)
        ref = wrap(hy, sc.to_referencing_table(hy, t))
        for cond in CONDS:
            check(hy, oracle, ref, 1, cond, 123)


def synthetic(hy, rng, n, chunk, dtype, distinct, null_frac, encode):
    dt = {"int": hy.DataType.Int, "long": hy.DataType.Long, "float": hy.DataType.Float,
          "double": hy.DataType.Double}[dtype]
    npt = {"int": np.int32, "long": np.int64, "float": np.float32, "double": np.float64}[dtype]
    vals = rng.integers(0, distinct, n).astype(npt)
    if dtype in ("float", "double"):
        vals = (vals * 0.25).astype(npt)
    nulls = (rng.random(n) < null_frac).astype(np.uint8) if null_frac else None
    t = hy.Table.from_arrays([("a", dt, nulls is not None), ("b", hy.DataType.Int, False)],
                             [vals, np.arange(n, dtype=np.int32)], [nulls, None], chunk)
    if encode:
        hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
    return t


@pytest.mark.parametrize("dtype", ["int", "long", "float", "double"])
@pytest.mark.parametrize("encode", [False, True])
def test_synthetic_scans(hy, oracle, dtype, encode):
    rng = np.random.default_rng(0x48595249)
    # ragged chunk size (not a multiple of 16) exercises tail tiles; distinct counts hit u8 / u16 / u32 widths
    for n, chunk, distinct in ((50_000, 10_007, 50), (70_000, 65_536, 300), (140_000, 70_000, 70_000)):
        t = synthetic(hy, rng, n, chunk, dtype, distinct, 0.05, encode)
        w = wrap(hy, t)
        for cond in CONDS:
            v = distinct // 3 if dtype in ("int", "long") else (distinct // 3) * 0.25
            check(hy, oracle, w, 0, cond, v)
        for cond in ("IsNull", "IsNotNull"):
            check(hy, oracle, w, 0, cond, None)
        check(hy, oracle, w, 0, "LessThan", v, excluded=[1])


@pytest.mark.parametrize("two_pass", ["1", "0"])
def test_scan_paths_one_and_two_pass(hy, oracle, monkeypatch, two_pass):
    """The count + write kernels (chunks of at most 64 segments) and the one-pass look-back kernel (HY_SCAN_TWO_PASS=0,
    or a class with a longer chunk) give the same PosLists: u8 / u16 ids and int values, a 1.2 M-row chunk (74 u8
    segments: its class takes the look-back kernel) beside 100,000- and 7-row chunks, RowID and offset outputs."""
    monkeypatch.setenv("HY_SCAN_TWO_PASS", two_pass)
    rng = np.random.default_rng(0x3250)
    for n, chunk, distinct, encode in ((400_000, 100_000, 50, True), (300_007, 100_000, 1_000, True),
                                       (250_000, 65_536, 1 << 20, False), (1_300_007, 1_200_000, 40, True)):
        t = synthetic(hy, rng, n, chunk, "int", distinct, 0.02, encode)
        w = wrap(hy, t)
        for cond, v in (("LessThan", distinct // 3), ("GreaterThanEquals", distinct // 2), ("Equals", 7),
                        ("NotEquals", 7), ("IsNull", None), ("IsNotNull", None)):
            check(hy, oracle, w, 0, cond, v)
        check(hy, oracle, w, 0, "LessThan", distinct // 3, excluded=[0])


def test_scan_then_reference_scan_large(hy, oracle):
    rng = np.random.default_rng(7)
    t = synthetic(hy, rng, 300_000, 100_000, "int", 50, 0.0, True)
    w = wrap(hy, t)
    s1 = check(hy, oracle, w, 0, "LessThan", 24)
    check(hy, oracle, s1, 1, "GreaterThanEquals", 150_000)


def test_scan_for_null_values(hy, oracle):
    """ScanForNullValues* (table_scan_test.cpp:503-601): data, dictionary, referencing and NULL-RowID inputs."""
    for name, t, cases in sc.null_scan_tables(hy):
        w = wrap(hy, t)
        for cond, expected in cases.items():
            s = check(hy, oracle, w, 1, cond, None)
            assert sc.multiset(sc.column_values(s.get_output(), 0)) == sc.multiset(expected), (name, cond)
        check(hy, oracle, w, 0, "IsNull", None)  # column a: nullable in the null tables, non-nullable in int_float


def test_is_null_reference_scan_large(hy, oracle):
    """IS [NOT] NULL over a multi-chunk PosList (unordered_map group order) with NULL RowIDs mixed in."""
    rng = np.random.default_rng(11)
    for encode in (False, True):
        t = synthetic(hy, rng, 120_000, 30_000, "int", 40, 0.1, encode)
        pl = np.stack([rng.integers(0, 4, 50_000), rng.integers(0, 30_000, 50_000)], axis=1).astype(np.uint32)
        pl[rng.random(50_000) < 0.05] = sc.NULL_ROW_ID
        ref = hy.Table([("a", hy.DataType.Int, True), ("b", hy.DataType.Int, False)], hy.TableType.References)
        ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
        w = wrap(hy, ref)
        for cond in ("IsNull", "IsNotNull"):
            check(hy, oracle, w, 0, cond, None)
        s1 = check(hy, oracle, wrap(hy, t), 0, "IsNotNull", None)
        check(hy, oracle, s1, 0, "LessThan", 20)


def check_cmp(hy, oracle, op, left, cond, right, excluded=None):
    s = hy.TableScan(op, left, getattr(hy.PredicateCondition, cond), hy.ColumnParameter(right))
    if excluded:
        s.set_excluded_chunk_ids(excluded)
    s.execute()
    exp = oracle.table_scan(op.get_output(), left, getattr(hy.PredicateCondition, cond), None, excluded or [],
                            right_column_id=right)
    assert_identical(s.get_output(), exp)
    return s


def test_column_comparison_reference_cases(hy, oracle):
    """Scan*ColumnWithFloatColumnWithNullValues (table_scan_test.cpp:383-439) plus every predicate."""
    for name, t in sc.column_compare_tables(hy):
        w = wrap(hy, t)
        s = check_cmp(hy, oracle, w, 0, "GreaterThan", 1)
        assert sc.multiset(sc.column_values(s.get_output(), 0)) == sc.multiset(sc.COLUMN_COMPARE_EXPECTED), name
        for cond in CONDS:
            check_cmp(hy, oracle, w, 1, cond, 0)
    w = wrap(hy, hy.load_table(tbl("int_float.tbl"), 2))
    for cond in CONDS:
        check_cmp(hy, oracle, w, 0, cond, 1)
        check_cmp(hy, oracle, w, 1, cond, 0)


@pytest.mark.parametrize("types", [("int", "int"), ("int", "float"), ("long", "double"), ("long", "float"),
                                   ("double", "int"), ("float", "long")])
def test_column_comparison_synthetic(hy, oracle, types):
    rng = np.random.default_rng(0x434D50)
    dts = {"int": hy.DataType.Int, "long": hy.DataType.Long, "float": hy.DataType.Float, "double": hy.DataType.Double}
    npt = {"int": np.int32, "long": np.int64, "float": np.float32, "double": np.float64}
    n, chunk = 90_000, 20_011
    cols = []
    for ty in types:
        v = rng.integers(0, 60, n).astype(npt[ty])
        if ty in ("float", "double"):
            v = (v * 0.5).astype(npt[ty])
        cols.append(v)
    nulls = [(rng.random(n) < 0.05).astype(np.uint8), (rng.random(n) < 0.05).astype(np.uint8)]
    t = hy.Table.from_arrays([("a", dts[types[0]], True), ("b", dts[types[1]], True)], cols, nulls, chunk)
    hy.encode_chunks(t, [1, 3], hy.EncodingType.Dictionary)  # mixed value / dictionary chunks
    w = wrap(hy, t)
    for cond in CONDS:
        check_cmp(hy, oracle, w, 0, cond, 1)
    check_cmp(hy, oracle, w, 0, "LessThan", 1, excluded=[0, 2])
    # reference input (a scan's output, then a weird PosList with NULL RowIDs across chunks)
    s1 = check(hy, oracle, w, 0, "IsNotNull", None)
    check_cmp(hy, oracle, s1, 1, "GreaterThanEquals", 0)
    pl = np.stack([rng.integers(0, 5, 30_000), rng.integers(0, 9_956, 30_000)], axis=1).astype(np.uint32)
    pl[rng.random(30_000) < 0.05] = sc.NULL_ROW_ID
    ref = hy.Table([("a", dts[types[0]], True), ("b", dts[types[1]], True)], hy.TableType.References)
    ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    for cond in ("Equals", "LessThan", "GreaterThan"):
        check_cmp(hy, oracle, wrap(hy, ref), 0, cond, 1)


def test_like_dictionary(hy, oracle):
    """LIKE / NOT LIKE over dictionary-encoded string columns (table_scan_string_test.cpp *OnDict* and
    *OnReferencedDict* cases + the special-character patterns), bit-exact against the oracle."""
    for enc, t in sc.like_tables(hy, encodings=("Dictionary", "FixedStringDictionary")):
        w = wrap(hy, t)
        for cond, pattern, _ in sc.LIKE_CASES:
            check(hy, oracle, w, 1, cond, pattern)
            s1 = check(hy, oracle, w, 0, "GreaterThan", 0)
            check(hy, oracle, s1, 1, cond, pattern)
    special = hy.load_table(tbl("int_string_like_special_chars.tbl"), 2)
    hy.encode_all_chunks(special, hy.EncodingType.Dictionary)
    for pattern, expected in sc.LIKE_SPECIAL_CASES:
        s = check(hy, oracle, wrap(hy, special), 1, "Like", pattern)
        assert_table_eq_unordered(s.get_output(), hy.load_table(tbl(expected), 1))
    with pytest.raises(RuntimeError):  # LIKE on a non-string column
        device_scan(hy, wrap(hy, hy.load_table(tbl("int_float.tbl"), 2)), 0, "Like", "%test")


def test_like_synthetic(hy, oracle):
    """Many dictionaries (u8 / u16 id widths), NULLs, every pattern shape incl. the regex fallback."""
    rng = np.random.default_rng(0x4C494B45)
    words = ["".join(rng.choice(list("abcXYZ_%.("), rng.integers(0, 9))) for _ in range(700)]
    n = 40_000
    t = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.Data, 7_001)
    for i in range(n):
        t.append([i, None if rng.random() < 0.03 else words[rng.integers(0, 700 if i < 20_000 else 60)]])
    hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    for pattern in ("a%", "%Z", "%bc%", "%a%X%", "a_c%", "_", "%(%", "%.%", "X%a%c", "%", "abcabcabcabc%"):
        for cond in ("Like", "NotLike"):
            check(hy, oracle, w, 1, cond, pattern)
    s1 = check(hy, oracle, w, 0, "GreaterThanEquals", 15_000)
    check(hy, oracle, s1, 1, "Like", "%b%")


@pytest.mark.parametrize("dtype", ["int", "long", "float"])
def test_compressed_scans_mixed_chunks(hy, oracle, dtype):
    """RunLength and FrameOfReference chunks scanned in compressed form (hy_table_scan's HY_COL_RLE / HY_COL_FOR
    classes) next to dictionary and unencoded chunks of the same column, in one call: clustered values (long runs)
    and short runs, NULL runs, ragged chunk sizes, every predicate, data and reference inputs."""
    rng = np.random.default_rng(0x524C45)
    dt = {"int": hy.DataType.Int, "long": hy.DataType.Long, "float": hy.DataType.Float}[dtype]
    npt = {"int": np.int32, "long": np.int64, "float": np.float32}[dtype]
    n, chunk = 120_000, 23_011
    runs = np.repeat(rng.integers(-50, 50, n // 7 + 1), rng.integers(1, 14, n // 7 + 1))[:n]
    runs = np.concatenate([runs, rng.integers(-50, 50, n - len(runs))]) if len(runs) < n else runs
    vals = runs.astype(npt)
    big = 3_000_000_000  # long: past int32, yet a FoR block (NULLs count as 0) spans < 2^32, as its encoder asserts
    if dtype == "long":
        vals = vals + np.int64(big)
    nulls = np.repeat((rng.random(n // 20 + 1) < 0.1).astype(np.uint8), 20)[:n]
    t = hy.Table.from_arrays([("a", dt, True), ("b", hy.DataType.Int, False)], [vals, np.arange(n, dtype=np.int32)],
                             [nulls, None], chunk)
    hy.encode_chunks(t, [0, 3], hy.EncodingType.RunLength)
    if dtype != "float":
        hy.encode_chunks(t, [1, 4], hy.EncodingType.FrameOfReference)
    hy.encode_chunks(t, [2], hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    for cond in CONDS:
        for v in (0, -17, 49, 60):
            c = v + big if dtype == "long" else v
            check(hy, oracle, w, 0, cond, c)
    for cond in ("IsNull", "IsNotNull"):
        check(hy, oracle, w, 0, cond, None)
    check(hy, oracle, w, 0, "GreaterThan", 3, excluded=[1])
    s1 = check(hy, oracle, w, 1, "GreaterThanEquals", 30_000)
    check(hy, oracle, s1, 0, "LessThan", 5)
    # valid RowIDs only: chunk 5 holds 120,000 - 5 * 23,011 = 4,945 rows
    pl = np.stack([rng.integers(0, 6, 40_000), rng.integers(0, 4_945, 40_000)], axis=1).astype(np.uint32)
    pl[rng.random(40_000) < 0.05] = sc.NULL_ROW_ID
    ref = hy.Table([("a", dt, True), ("b", hy.DataType.Int, False)], hy.TableType.References)
    ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    for cond, v in (("Equals", 7), ("LessThanEquals", -3), ("IsNull", None), ("NotEquals", 0)):
        c = v + big if (dtype == "long" and v is not None) else v
        check(hy, oracle, wrap(hy, ref), 0, cond, c)
