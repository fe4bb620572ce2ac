"""Device TableScans over std::string columns held in HBM (packed string arrays): comparisons, LIKE / NOT LIKE and
IS [NOT] NULL on unencoded, Dictionary, FixedStringDictionary and RunLength chunks (alone and mixed), reference
inputs, and string column-vs-column comparisons - bit-exact PosLists against the oracle, plus the reference's expected tables of
table_scan_string_test.cpp."""
import numpy as np
import pytest

import scan_cases as sc
from helpers import assert_identical, assert_table_eq_unordered, tbl, wrap
from test_scan_gpu import CONDS, check, check_cmp, device_scan

pytestmark = pytest.mark.gpu


def string_table(hy, encoding):
    """_gt_string_compressed of table_scan_string_test.cpp:46-57 (chunk 5, string column in `encoding`)."""
    return wrap(hy, sc.string_compressed(hy, encoding))


@pytest.mark.parametrize("encoding", sc.STRING_ENCODINGS)
def test_string_compare_reference_cases(hy, oracle, encoding):
    """ScanEquals / ScanNotEquals / ScanLessThan (table_scan_string_test.cpp:74-97) in the reference's four
    encodings (:69-72), then every comparison against the oracle."""
    w = string_table(hy, encoding)
    for cond, value, rows, expected in (("Equals", "Reeperbahn", 1, "int_string_like_equals.tbl"),
                                        ("NotEquals", "Reeperbahn", 5, "int_string_like_not_equals.tbl"),
                                        ("LessThan", "Schiff", 5, "int_string_like_less_than.tbl")):
        s = check(hy, oracle, w, 1, cond, value)
        assert s.get_output().row_count() == rows
        assert_table_eq_unordered(s.get_output(), hy.load_table(tbl(expected), 1))
    for cond in CONDS:
        for v in ("", "Dampf", "Reeperbahn", "zzz", "Schifffahrtsgesellschaft"):
            check(hy, oracle, w, 1, cond, v)


@pytest.mark.parametrize("encoding", sc.STRING_ENCODINGS)
def test_like_compressed_reference_cases(hy, oracle, encoding):
    """The *OnDict* / *OnReferencedDict* LIKE and NOT LIKE TEST_Ps of table_scan_string_test.cpp (:99-187), which the
    reference runs on _gt_string_compressed in all four encodings: the expected tables, and the oracle's PosLists."""
    w = string_table(hy, encoding)
    for cond, pattern, expected in sc.LIKE_CASES:
        s = check(hy, oracle, w, 1, cond, pattern)
        s1 = check(hy, oracle, w, 0, "GreaterThan", 0)
        s2 = check(hy, oracle, s1, 1, cond, pattern)
        for out in (s.get_output(), s2.get_output()):
            if isinstance(expected, int):
                assert out.row_count() == expected
            else:
                assert_table_eq_unordered(out, hy.load_table(tbl(expected), 1))


@pytest.mark.parametrize("encoding", ["FixedStringDictionary", "RunLength"])
def test_string_encoded_synthetic(hy, oracle, encoding):
    """Seeded string columns in FixedStringDictionary / RunLength chunks mixed with unencoded and dictionary chunks:
    runs of repeated values and NULL runs (RunLength), values of different lengths under one fixed width, ragged chunk
    tails; every comparison, IS [NOT] NULL, LIKE shapes, then a referencing table across the encodings."""
    rng = np.random.default_rng(0x46534452)
    words = random_strings(rng, 300)
    n, chunk = 40_000, 9_001
    t = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.Data, chunk)
    i = 0
    while i < n:  # runs of 1..40 equal values (NULL runs included)
        v = None if rng.random() < 0.06 else words[rng.integers(0, len(words))]
        for _ in range(int(rng.integers(1, 41))):
            if i < n:
                t.append([i, v])
                i += 1
    hy.encode_chunks(t, [0, 2, 4], getattr(hy.EncodingType, encoding))
    hy.encode_chunks(t, [1], hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    for cond in CONDS:
        for v in ("abc", "", words[5], "ZZZ", "a", words[11] + "\x00"):
            check(hy, oracle, w, 1, cond, v)
    for cond in ("IsNull", "IsNotNull"):
        check(hy, oracle, w, 1, cond, None)
    for pattern in ("a%", "%Z", "%bc%", "%a%X%", "a_c%", "_", "%(%", "%", "[ab]%", "%\n%"):
        for cond in ("Like", "NotLike"):
            check(hy, oracle, w, 1, cond, pattern)
    s1 = check(hy, oracle, w, 0, "GreaterThanEquals", 7_000)
    check(hy, oracle, s1, 1, "Like", "%b%")
    check(hy, oracle, s1, 1, "LessThan", "X")
    # valid RowIDs only: chunk 4 holds 40,000 - 4 * 9,001 = 3,996 rows
    pl = np.stack([rng.integers(0, 5, 20_000), rng.integers(0, 3_996, 20_000)], axis=1).astype(np.uint32)
    pl[rng.random(20_000) < 0.05] = sc.NULL_ROW_ID
    ref = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.References)
    ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    wr = wrap(hy, ref)
    for cond, v in (("Equals", words[7]), ("GreaterThanEquals", "b"), ("Like", "%a%"), ("IsNull", None)):
        check(hy, oracle, wr, 1, cond, v)


def test_like_unencoded(hy, oracle):
    """Every LIKE case of table_scan_string_test.cpp on the unencoded _gt_string (chunk 2) and on a referencing
    table over it, the special-character patterns (regex path) and ScanLikeNonStringValue."""
    t = hy.load_table(tbl("int_string_like.tbl"), 2)
    w = wrap(hy, t)
    for cond, pattern, expected in sc.LIKE_CASES:
        s = check(hy, oracle, w, 1, cond, pattern)
        if isinstance(expected, int):
            assert s.get_output().row_count() == expected
        else:
            assert_table_eq_unordered(s.get_output(), hy.load_table(tbl(expected), 1))
        s1 = check(hy, oracle, w, 0, "GreaterThan", 0)
        check(hy, oracle, s1, 1, cond, pattern)
    special = wrap(hy, hy.load_table(tbl("int_string_like_special_chars.tbl"), 2))
    for pattern, expected in sc.LIKE_SPECIAL_CASES:
        s = check(hy, oracle, special, 1, "Like", pattern)
        assert_table_eq_unordered(s.get_output(), hy.load_table(tbl(expected), 1))
    assert check(hy, oracle, w, 1, "Like", 1234).get_output().row_count() == 1  # ScanLikeNonStringValue


EDGE_VALUES = ["a]b", "a]bc", "ab", "a\nb", "a\rb", "a.b", "a*b", "ac", "", "[x", "a-b", "b", "\x80z", "a_b",
               "Dampf", "dampf", "Dampfschiff", "schifffahrt", "a%b", "%", "_"]
EDGE_PATTERNS = ["a]_%", "a]b", "a_b", "%%", "a[.]b", "a[%]b", "a[b-d]", "a[]b", "[[]x", "a[^b]", "_%_", "",
                 "a[-]b", "%\x80%", "a[\\]b", "a\nb", "%a%b", "%a%b%", "a%", "%b", "%_%", "D_mpf%", "__", "%[xz]",
                 "a[.-z]b", "a[_-z]b", "a[%-z]b", "[*-.]%", "a[^-b]"]


def edge_table(hy, rng, n, chunk, encode_chunks):
    t = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.Data, chunk)
    for i in range(n):
        t.append([i, None if rng.random() < 0.05 else EDGE_VALUES[rng.integers(0, len(EDGE_VALUES))]])
    if encode_chunks:
        hy.encode_chunks(t, encode_chunks, hy.EncodingType.Dictionary)
    return t


def test_like_edge_patterns(hy, oracle):
    """The regex path's corner cases (classes, ']' outside a class, '\\n' / '\\r' against '.', an empty class) and
    the simple patterns' (''; '%a%b' matching anywhere), on value chunks mixed with dictionary chunks."""
    rng = np.random.default_rng(0x535452)
    t = edge_table(hy, rng, 5_000, 997, [1, 3])
    w = wrap(hy, t)
    for pattern in EDGE_PATTERNS:
        for cond in ("Like", "NotLike"):
            check(hy, oracle, w, 1, cond, pattern)
    with pytest.raises(RuntimeError):  # the reference's std::regex rejects an unterminated class
        device_scan(hy, w, 1, "Like", "[a")
    with pytest.raises(RuntimeError):  # "[a-%]" is the regex class "[a-.*]": a range out of order
        device_scan(hy, w, 1, "Like", "a[a-%]b")


def test_like_long_patterns(hy, oracle):
    """Patterns of 64 to ~700 NFA positions (more than one 64-bit state word; the reference's std::regex takes any
    length): '_' runs, '%' between them, [...] classes, literal runs, on long strings - against the oracle's
    std::regex, on value chunks mixed with dictionary chunks."""
    rng = np.random.default_rng(0x4C4F4E)
    base = ["".join(rng.choice(list("ab"), rng.integers(40, 220))) for _ in range(300)]
    t = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.Data, 1_499)
    for i in range(6_000):
        t.append([i, None if rng.random() < 0.03 else base[rng.integers(0, len(base))]])
    hy.encode_chunks(t, [1], hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    v = base[0]
    patterns = [
        "_" * 130 + "%",                                   # strings of >= 130 bytes
        "%" + "a_" * 40 + "%",                             # 80 positions + stars
        v[:100].replace("b", "_", 7) + "%",                # a 101-position prefix pattern
        "[ab]" * 70 + "%",                                 # 70 classes
        "%" + "%".join(v[i:i + 9] for i in range(0, 90, 9)) + "%",  # ten literal runs with stars (multi-contains)
        v[:60] + "_%" + v[-5:] + "%_",                     # > 63 positions ending in stars
        v,                                                 # one exact long string as a regex-free pattern
        "%" + "_" * 700,                                   # 701 positions
        v[:64] + "%" + "[a]" * 64,
    ]
    for pattern in patterns:
        for cond in ("Like", "NotLike"):
            check(hy, oracle, w, 1, cond, pattern)


def random_strings(rng, k, alphabet="abcXYZ_%.(\n", max_len=12):
    chars = list(alphabet)
    return ["".join(rng.choice(chars, rng.integers(0, max_len))) for _ in range(k)]


def test_string_synthetic(hy, oracle):
    """Seeded tables: ragged chunks (tail tiles), unencoded and dictionary chunks mixed, NULLs, every comparison
    (prefix / length ordering), IS [NOT] NULL, LIKE shapes, then reference inputs with NULL RowIDs across chunks."""
    rng = np.random.default_rng(0x53594E)
    words = random_strings(rng, 900)
    n, chunk = 30_000, 7_001
    t = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.Data, chunk)
    for i in range(n):
        t.append([i, None if rng.random() < 0.04 else words[rng.integers(0, len(words))]])
    hy.encode_chunks(t, [0, 2], hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    for cond in CONDS:
        for v in ("abc", "", words[5], "ZZZ", "a"):
            check(hy, oracle, w, 1, cond, v)
    for cond in ("IsNull", "IsNotNull"):
        check(hy, oracle, w, 1, cond, None)
    for pattern in ("a%", "%Z", "%bc%", "%a%X%", "a_c%", "_", "%(%", "%.%", "X%a%c", "%", "[ab]%", "%\n%", "%%"):
        for cond in ("Like", "NotLike"):
            check(hy, oracle, w, 1, cond, pattern)
    check(hy, oracle, w, 1, "LessThan", "b", excluded=[1])
    s1 = check(hy, oracle, w, 0, "GreaterThanEquals", 9_000)
    check(hy, oracle, s1, 1, "Like", "%b%")
    check(hy, oracle, s1, 1, "GreaterThan", "X")
    # valid RowIDs only: chunk 4 holds 30,000 - 4 * 7,001 = 1,996 rows
    pl = np.stack([rng.integers(0, 5, 20_000), rng.integers(0, 1_996, 20_000)], axis=1).astype(np.uint32)
    pl[rng.random(20_000) < 0.05] = sc.NULL_ROW_ID
    ref = hy.Table([("a", hy.DataType.Int, False), ("s", hy.DataType.String, True)], hy.TableType.References)
    ref.append_chunk([hy.ReferenceColumn(t, 0, pl), hy.ReferenceColumn(t, 1, pl)])
    wr = wrap(hy, ref)
    for cond, v in (("Equals", words[7]), ("LessThanEquals", "b"), ("Like", "%a%"), ("NotLike", "_%"),
                    ("IsNull", None), ("IsNotNull", None)):
        check(hy, oracle, wr, 1, cond, v)


def test_string_column_comparison(hy, oracle):
    """ColumnComparisonTableScanImpl on two string columns (data, mixed encodings, reference input)."""
    rng = np.random.default_rng(0x434D53)
    words = random_strings(rng, 40, alphabet="abAB", max_len=4)
    n, chunk = 20_000, 4_099
    t = hy.Table([("x", hy.DataType.String, True), ("y", hy.DataType.String, True)], hy.TableType.Data, chunk)
    for _ in range(n):
        a = None if rng.random() < 0.05 else words[rng.integers(0, 40)]
        b = None if rng.random() < 0.05 else words[rng.integers(0, 40)]
        t.append([a, b])
    hy.encode_chunks(t, [1, 2], hy.EncodingType.Dictionary)
    w = wrap(hy, t)
    for cond in CONDS:
        check_cmp(hy, oracle, w, 0, cond, 1)
    s1 = check(hy, oracle, w, 0, "IsNotNull", None)
    for cond in ("Equals", "LessThan", "GreaterThanEquals"):
        check_cmp(hy, oracle, s1, 1, cond, 0)
    t2 = hy.Table([("x", hy.DataType.String, False), ("y", hy.DataType.Int, False)], hy.TableType.Data)
    t2.append(["a", 1])
    with pytest.raises(RuntimeError):  # a string and a numeric column: "Invalid column combination detected!"
        hy.TableScan(wrap(hy, t2), 0, hy.PredicateCondition.Equals, hy.ColumnParameter(1)).execute()
