"""TableScan cases of the reference's src/test/operators/table_scan_test.cpp (expected column-1 multisets copied
from the test's inline vectors), shared by the oracle tests (CPU) and the device parity tests (GPU)."""
from helpers import tbl, wrap

ENCODINGS = ["Unencoded", "Dictionary", "RunLength", "FrameOfReference"]  # table_scan_test.cpp:206-209


def int_int_tables(hy, encoding):
    """_int_int_compressed (chunk 7, chunks 0,1 encoded) and _int_int_partly_compressed (chunk 5, chunks 0,1)."""
    t7 = hy.load_table(tbl("int_int_shuffled.tbl"), 7)
    t5 = hy.load_table(tbl("int_int_shuffled_2.tbl"), 5)
    enc = getattr(hy.EncodingType, encoding)
    hy.encode_chunks(t7, [0, 1], enc)
    hy.encode_chunks(t5, [0, 1], enc)
    return wrap(hy, t7), wrap(hy, t5)


def filtered_table(hy, partly):
    """get_table_op_filtered: a reference table with a 'weird' PosList over the partly compressed table."""
    t = hy.Table([("a", hy.DataType.Int, False), ("b", hy.DataType.Int, False)], hy.TableType.References, 5)
    src = partly.get_output()
    pl = [[2, 0], [1, 1], [1, 3], [0, 2], [2, 2], [0, 0], [0, 4]]
    t.append_chunk([hy.ReferenceColumn(src, 0, pl), hy.ReferenceColumn(src, 1, pl)])
    return wrap(hy, t)


def to_referencing_table(hy, table):
    pl = []
    for c in range(table.chunk_count()):
        for o in range(table.get_chunk(c).size()):
            pl.append([c, o])
    defs = [(n, t, False) for (n, t, _) in table.column_definitions()]
    out = hy.Table(defs, hy.TableType.References)
    out.append_chunk([hy.ReferenceColumn(table, c, pl) for c in range(table.column_count())])
    return out


C = None  # filled lazily with PredicateCondition names


def compressed_column_cases():
    # ScanOnCompressedColumn (table_scan_test.cpp:226-268), column a vs 6
    return {
        "Equals": [106, 106],
        "NotEquals": [100, 102, 104, 108, 110, 112, 100, 102, 104, 108, 110, 112],
        "LessThan": [100, 102, 104, 100, 102, 104],
        "LessThanEquals": [100, 102, 104, 106, 100, 102, 104, 106],
        "GreaterThan": [108, 110, 112, 108, 110, 112],
        "GreaterThanEquals": [106, 108, 110, 112, 106, 108, 110, 112],
        "IsNull": [],
        "IsNotNull": [100, 102, 104, 106, 108, 110, 112, 100, 102, 104, 106, 108, 110, 112],
    }


def referenced_compressed_cases():
    # ScanOnReferencedCompressedColumn (:269-305): scan1 b < 108, then a OP 4
    return {
        "Equals": [104, 104],
        "NotEquals": [100, 102, 106, 100, 102, 106],
        "LessThan": [100, 102, 100, 102],
        "LessThanEquals": [100, 102, 104, 100, 102, 104],
        "GreaterThan": [106, 106],
        "GreaterThanEquals": [104, 106, 104, 106],
        "IsNull": [],
        "IsNotNull": [100, 102, 104, 106, 100, 102, 104, 106],
    }


def weird_pos_list_cases():
    # ScanWeirdPosList (:312-331): column a vs 10
    return {
        "Equals": [110, 110],
        "NotEquals": [100, 102, 106, 108, 112],
        "LessThan": [100, 102, 106, 108],
        "LessThanEquals": [100, 102, 106, 108, 110, 110],
        "GreaterThan": [112],
        "GreaterThanEquals": [110, 110, 112],
        "IsNull": [],
        "IsNotNull": [100, 102, 106, 108, 110, 110, 112],
    }


ALL_ROWS = [100, 102, 104, 106, 108, 110, 112, 100, 102, 104, 106, 108, 110, 112]


def greater_than_max_cases():  # :333-357, value 30
    return {"Equals": [], "NotEquals": ALL_ROWS, "LessThan": ALL_ROWS, "LessThanEquals": ALL_ROWS,
            "GreaterThan": [], "GreaterThanEquals": []}


def less_than_min_cases():  # :359-381, value -10
    return {"Equals": [], "NotEquals": ALL_ROWS, "LessThan": [], "LessThanEquals": [], "GreaterThan": ALL_ROWS,
            "GreaterThanEquals": ALL_ROWS}


def around_bounds_cases():  # ScanOnCompressedColumnAroundBounds, value 0
    return {
        "Equals": [100, 100],
        "LessThan": [],
        "LessThanEquals": [100, 100],
        "GreaterThan": [102, 104, 106, 108, 110, 112, 102, 104, 106, 108, 110, 112],
        "GreaterThanEquals": ALL_ROWS,
        "NotEquals": [102, 104, 106, 108, 110, 112, 102, 104, 106, 108, 110, 112],
    }


# ScanForNullValues* (table_scan_test.cpp:503-601): scan_for_null_values scans column b with IS [NOT] NULL and
# compares column a (multiset)
NULL_VALUE_CASES = {"IsNull": [12, 123], "IsNotNull": [12345, None, 1234, 12345, 12, 1234]}
NO_NULL_CASES = {"IsNull": [], "IsNotNull": [12345, 123, 1234]}
NULL_ROW_ID_CASES = {"IsNull": [123, 1234], "IsNotNull": [12345, None]}
NULL_ROW_ID = 0xFFFFFFFF


def null_scan_tables(hy):
    """(name, table, expected cases) for every ScanForNullValues* test of table_scan_test.cpp:503-601."""
    out = []
    for enc in (None, "Dictionary", "RunLength", "FrameOfReference"):
        t = hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4)
        if enc:
            hy.encode_all_chunks(t, getattr(hy.EncodingType, enc))
        out.append((f"w_null_{enc}", t, NULL_VALUE_CASES))
        out.append((f"ref_w_null_{enc}", to_referencing_table(hy, t), NULL_VALUE_CASES))
        out.append((f"null_row_id_{enc}", referencing_table_w_null_row_id(hy, t), NULL_ROW_ID_CASES))
    t = hy.load_table(tbl("int_float.tbl"), 4)
    out.append(("without_nulls", t, NO_NULL_CASES))
    out.append(("ref_without_nulls", to_referencing_table(hy, t), NO_NULL_CASES))
    return out


def referencing_table_w_null_row_id(hy, table):
    """create_referencing_table_w_null_row_id (table_scan_test.cpp:130-155): two ReferenceColumns with different
    PosLists, column b's starting with a NULL RowID."""
    pa = [[0, 1], [1, 0], [0, 2], [0, 3]]
    pb = [[NULL_ROW_ID, NULL_ROW_ID], [0, 0], [1, 2], [0, 1]]
    out = hy.Table([("a", hy.DataType.Int, True), ("b", hy.DataType.Int, True)], hy.TableType.References)
    out.append_chunk([hy.ReferenceColumn(table, 0, pa), hy.ReferenceColumn(table, 1, pb)])
    return out


# Scan*ColumnWithFloatColumnWithNullValues (table_scan_test.cpp:383-439): a > b over int_int_w_null_8_rows (chunk 4),
# as data / dictionary / referencing table; column a of the output
COLUMN_COMPARE_EXPECTED = [12345, 1234, 12345, 1234]


def column_compare_tables(hy):
    out = []
    for enc in (None, "Dictionary", "RunLength", "FrameOfReference"):
        t = hy.load_table(tbl("int_int_w_null_8_rows.tbl"), 4)
        if enc:
            hy.encode_all_chunks(t, getattr(hy.EncodingType, enc))
        out.append((f"data_{enc}", t))
        out.append((f"ref_{enc}", to_referencing_table(hy, t)))
    return out


# table_scan_string_test.cpp:100-330: (predicate, pattern, expected .tbl or a row count) on int_string_like.tbl
LIKE_CASES = [
    ("Like", "%", "int_string_like.tbl"),
    ("Like", "%D%_m_f%", "int_string_like_starting.tbl"),
    ("Like", "Dampf%", "int_string_like_starting.tbl"),
    ("Like", "%gesellschaft", "int_string_like_ending.tbl"),
    ("Like", "Schiff%schaft", "int_string_like_containing_wildcard.tbl"),
    ("Like", "%schifffahrtsgesellschaft%", "int_string_like_containing.tbl"),
    ("Like", "%not_there%", 0),
    ("NotLike", "%", 0),
    ("NotLike", "%foo%", "int_string_like.tbl"),
    ("NotLike", "D_m_f%", "int_string_like_not_starting.tbl"),
]
# ScanLikeOnSpecialChars (:189-213) on int_string_like_special_chars.tbl
LIKE_SPECIAL_CASES = [
    ("%2^2%", "int_string_like_special_chars_1.tbl"),
    ("%$%$%", "int_string_like_special_chars_1.tbl"),
    ("%(%)%", "int_string_like_special_chars_2.tbl"),
    ("%la\\.^$+?)({}.*__bl%", "int_string_like_special_chars_3.tbl"),
]


STRING_ENCODINGS = ("Unencoded", "Dictionary", "FixedStringDictionary", "RunLength")  # table_scan_string_test.cpp:69-72


def string_compressed(hy, enc):
    """_gt_string_compressed (table_scan_string_test.cpp:46-57): chunk size 5, the int column unencoded and the
    string column in `enc` (the reference's ChunkEncodingSpec {Unencoded, GetParam()})."""
    t = hy.load_table(tbl("int_string_like.tbl"), 5)
    if enc and enc != "Unencoded":
        hy.encode_columns(t, [1], getattr(hy.EncodingType, enc))
    return t


def like_tables(hy, encodings=(None,) + STRING_ENCODINGS):
    """_gt_string (chunk 2, unencoded) and _gt_string_compressed in each encoding, as tables."""
    out = []
    for enc in encodings:
        out.append((enc, string_compressed(hy, enc) if enc else hy.load_table(tbl("int_string_like.tbl"), 2)))
    return out


def multiset(values):
    return sorted(values, key=lambda v: (v is None, 0 if v is None else v))


def column_values(table, column_id):
    out = []
    for c in range(table.chunk_count()):
        out.extend(table.get_chunk(c).get_column(column_id).values())
    return out


def dict_n_entries(hy, n, encoding):
    """get_table_op_with_n_dict_entries: 0..n in one chunk."""
    t = hy.Table([("a", hy.DataType.Int, False)], hy.TableType.Data)
    for i in range(n + 1):
        t.append([i])
    hy.encode_chunks(t, [0], getattr(hy.EncodingType, encoding))
    return wrap(hy, t)
